/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, scalar, single thread) of the integer / byte / fixed-point parts of the
 * tracking path: Philox4x32-10, predict (H1), bilinear crop + im2col (H2/H3), estimate (H11) and the
 * exact-integer systematic resample (H12). Semantics: /root/repo/SPEC.md S1-S3, S6, S7.
 *
 * The reference (README-only, /root/reference/README.md:3, 8, 42) contains no implementation of any of
 * these; parity against it is therefore pinned by SPEC.md plus the published Random123 Philox
 * known-answer vectors (tests/test_oracle_pf.py), not by reference outputs.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, as the
 * checker. The product path never links it. Build: oracle/Makefile (-ffp-contract=off: every fused
 * multiply-add below is an explicit fmaf so the GPU kernels can reproduce the bits).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ---------------- Philox4x32-10 (SPEC S1) ---------------- */
static void philox_round(uint32_t c[4], const uint32_t k[2]) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k[0];
    uint32_t n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    uint32_t k[2] = {key[0], key[1]};
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u; }
        philox_round(c, k);
    }
    memcpy(out, c, sizeof(c));
}

static float uniform01(uint32_t r) { return (float)(2u * (r >> 9) + 1u) * 5.9604644775390625e-8f; }

/* ---------------- fixed fp32 elementary functions (SPEC S2) ---------------- */
static float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* ln(x), x in (0, 1]: Cephes logf polynomial, explicit fmaf */
float orc_logf(float x) {
    uint32_t b = f2bits(x);
    int e = (int)((b >> 23) & 0xff) - 126;        /* x = m * 2^e, m in [0.5, 1) */
    float m = bits2f((b & 0x007fffffu) | 0x3f000000u);
    if (m < 0.70710678118654752f) { e -= 1; m = m + m - 1.0f; } else { m = m - 1.0f; }
    float z = m * m;
    float p = 7.0376836292e-2f;
    p = fmaf(p, m, -1.1514610310e-1f);
    p = fmaf(p, m, 1.1676998740e-1f);
    p = fmaf(p, m, -1.2420140846e-1f);
    p = fmaf(p, m, 1.4249322787e-1f);
    p = fmaf(p, m, -1.6668057665e-1f);
    p = fmaf(p, m, 2.0000714765e-1f);
    p = fmaf(p, m, -2.4999993993e-1f);
    p = fmaf(p, m, 3.3333331174e-1f);
    float y = (m * z) * p;
    float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(z, -0.5f, y);
    float r = m + y;
    r = fmaf(fe, 0.693359375f, r);
    return r;
}

/* exp(x): Cephes expf, explicit fmaf; exact 0 below -87 */
float orc_expf(float x) {
    if (x < -87.0f) return 0.0f;
    if (x > 88.0f) x = 88.0f;
    float fn = floorf(fmaf(x, 1.44269504088896341f, 0.5f));
    float r = fmaf(fn, -0.693359375f, x);
    r = fmaf(fn, 2.12194440e-4f, r);
    float z = r * r;
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    float y = fmaf(p, z, r) + 1.0f;
    int n = (int)fn;
    /* y in [0.7, 1.5): scale by 2^n through the exponent field, two steps to stay normal */
    int n1 = n / 2, n2 = n - n1;
    y = y * bits2f((uint32_t)(n1 + 127) << 23);
    y = y * bits2f((uint32_t)(n2 + 127) << 23);
    return y;
}

/* (cos, sin)(2*pi*u), u in [0, 1): quadrant split, pi/4-centred Cephes polynomials */
void orc_sincos2pi(float u, float* c_out, float* s_out) {
    float t = u * 4.0f;
    float q = floorf(t);
    float r = t - q;                                   /* exact */
    float a = (r - 0.5f) * 1.57079632679489662f;        /* in [-pi/4, pi/4) */
    float z = a * a;
    float sp = -1.9515295891e-4f;
    sp = fmaf(sp, z, 8.3321608736e-3f);
    sp = fmaf(sp, z, -1.6666654611e-1f);
    float sa = fmaf(a * z, sp, a);
    float cp = 2.443315711809948e-5f;
    cp = fmaf(cp, z, -1.388731625493765e-3f);
    cp = fmaf(cp, z, 4.166664568298827e-2f);
    float ca = fmaf(z * z, cp, fmaf(z, -0.5f, 1.0f));
    /* angle = (pi/2)(q + 0.5) + a ; rotate by pi/4 then by q quadrants */
    const float h = 0.70710678118654752f;
    float c0 = (ca - sa) * h;   /* cos(pi/4 + a) */
    float s0 = (ca + sa) * h;   /* sin(pi/4 + a) */
    int qi = (int)q & 3;
    float c, s;
    switch (qi) {
        case 0: c = c0; s = s0; break;
        case 1: c = -s0; s = c0; break;
        case 2: c = -c0; s = -s0; break;
        default: c = s0; s = -c0; break;
    }
    *c_out = c; *s_out = s;
}

/* ---------------- predict (SPEC S2), particles SoA float[3][P] ---------------- */
void orc_predict(float* xs, float* ys, float* ss, int64_t n, int64_t global_begin, uint64_t seed,
                 uint32_t frame, float sig_x, float sig_y, float sig_s, float width, float height,
                 float smin, float smax) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t li = 0; li < n; ++li) {
        uint32_t ctr[4] = {(uint32_t)(global_begin + li), frame, 0u, 0u}, r[4];
        orc_philox4x32_10(ctr, key, r);
        float u0 = uniform01(r[0]), u1 = uniform01(r[1]), u2 = uniform01(r[2]), u3 = uniform01(r[3]);
        float ra = sqrtf(-2.0f * orc_logf(u0));
        float rb = sqrtf(-2.0f * orc_logf(u2));
        float c1, s1, c3, s3;
        orc_sincos2pi(u1, &c1, &s1);
        orc_sincos2pi(u3, &c3, &s3);
        float n0 = ra * c1, n1 = ra * s1, n2 = rb * c3;
        float x = fmaf(sig_x, n0, xs[li]);
        float y = fmaf(sig_y, n1, ys[li]);
        float s = ss[li] * orc_expf(sig_s * n2);
        x = fminf(fmaxf(x, 0.0f), width - 1.0f);
        y = fminf(fmaxf(y, 0.0f), height - 1.0f);
        s = fminf(fmaxf(s, smin), smax);
        xs[li] = x; ys[li] = y; ss[li] = s;
    }
}

/* ---------------- crop + im2col (SPEC S3), fp32 output ---------------- */
static float tap(const uint8_t* fr, int H, int W, int yy, int xx, int c) {
    if (yy < 0 || yy >= H || xx < 0 || xx >= W) return 0.0f;
    return (float)fr[((int64_t)yy * W + xx) * 3 + c];
}

/* out: float[n_part * g*g][Kp]; norm_a / norm_b: per-channel affine (SPEC S3) */
void orc_crop_patches(const uint8_t* frame, int H, int W, const float* xs, const float* ys,
                      const float* ss, int64_t n_part, float w0, float h0, int S, int patch, int Kp,
                      const float* norm_a, const float* norm_b, float* out) {
    int g = S / patch;
    int K = 3 * patch * patch;
    for (int64_t p = 0; p < n_part; ++p) {
        float bw = ss[p] * w0, bh = ss[p] * h0;
        float x0 = xs[p] - 0.5f * bw, y0 = ys[p] - 0.5f * bh;
        float dx = bw / (float)S, dy = bh / (float)S;
        for (int py = 0; py < g; ++py)
            for (int px = 0; px < g; ++px) {
                float* row = out + ((p * g * g) + py * g + px) * (int64_t)Kp;
                for (int k = K; k < Kp; ++k) row[k] = 0.0f;
                for (int c = 0; c < 3; ++c)
                    for (int ky = 0; ky < patch; ++ky) {
                        int oy = py * patch + ky;
                        float sy = (y0 + ((float)oy + 0.5f) * dy) - 0.5f;
                        float fy0 = floorf(sy);
                        float fy = sy - fy0;
                        int iy = (int)fy0;
                        for (int kx = 0; kx < patch; ++kx) {
                            int ox = px * patch + kx;
                            float sx = (x0 + ((float)ox + 0.5f) * dx) - 0.5f;
                            float fx0 = floorf(sx);
                            float fx = sx - fx0;
                            int ix = (int)fx0;
                            float p00 = tap(frame, H, W, iy, ix, c), p01 = tap(frame, H, W, iy, ix + 1, c);
                            float p10 = tap(frame, H, W, iy + 1, ix, c), p11 = tap(frame, H, W, iy + 1, ix + 1, c);
                            float top = (1.0f - fx) * p00 + fx * p01;
                            float bot = (1.0f - fx) * p10 + fx * p11;
                            float v = (1.0f - fy) * top + fy * bot;
                            row[c * patch * patch + ky * patch + kx] = fmaf(v, norm_a[c], norm_b[c]);
                        }
                    }
            }
    }
}

/* ---------------- estimate (SPEC S6) ---------------- */
/* out4 = {T (as exact int64 in out_T), sum Qx, sum Qy, sum Qs} */
void orc_shard_stats(const int64_t* Q, const float* xs, const float* ys, const float* ss, int64_t n,
                     int64_t* out_T, double* out_sums) {
    int64_t T = 0;
    double sx = 0, sy = 0, s_s = 0;
    for (int64_t i = 0; i < n; ++i) {
        T += Q[i];
        double q = (double)Q[i];
        sx += q * (double)xs[i]; sy += q * (double)ys[i]; s_s += q * (double)ss[i];
    }
    *out_T = T; out_sums[0] = sx; out_sums[1] = sy; out_sums[2] = s_s;
}

/* ---------------- systematic resample (SPEC S7) ---------------- */
static uint64_t offset_u(uint32_t U, uint64_t T) {
    return (uint64_t)U * (T >> 32) + (((uint64_t)U * (T & 0xffffffffu)) >> 32);
}

uint64_t orc_position(uint64_t j, uint64_t T, uint64_t P, uint32_t U) {
    uint64_t u = offset_u(U, T);
    uint64_t qT = T / P, rT = T % P, qu = u / P, ru = u % P;
    return j * qT + qu + (j * rT + ru) / P;
}

uint32_t orc_resample_U(uint64_t seed, uint32_t frame) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {0u, frame, 1u, 0u}, r[4];
    orc_philox4x32_10(ctr, key, r);
    return r[0];
}

/* Global resample over all P particles. Q may be all-zero (uniform fallback). anc: int32[P]. */
void orc_resample(const int64_t* Q, int64_t P, uint32_t U, int32_t* anc, int64_t* cdf_scratch) {
    int64_t T = 0;
    for (int64_t i = 0; i < P; ++i) T += Q[i];
    int uniform = (T == 0);
    int64_t acc = 0;
    for (int64_t i = 0; i < P; ++i) { acc += uniform ? 1 : Q[i]; cdf_scratch[i] = acc; }
    T = acc;
    for (int64_t j = 0; j < P; ++j) {
        uint64_t pos = orc_position((uint64_t)j, (uint64_t)T, (uint64_t)P, U);
        int64_t lo = 0, hi = P - 1;                 /* first i with C_i > pos */
        while (lo < hi) {
            int64_t mid = (lo + hi) >> 1;
            if ((uint64_t)cdf_scratch[mid] > pos) hi = mid; else lo = mid + 1;
        }
        anc[j] = (int32_t)lo;
    }
}
