// Particle-filter kernels (SPEC S2, S6, S7).
//
// predict: one thread per particle, counter-based Philox so the noise depends only on (seed, frame,
//   global index) and never on the sharding.
// shard_stats: one 1024-thread workgroup, fixed-order tree reduction (int64 exact + fp64 sums).
// resample: (1) single-workgroup inclusive int64 scan of the shard's Q into a workspace — wave scan
//   via DPP-free shuffles + one LDS carry per 4096-element chunk; (2) one thread per output slot:
//   exact 64-bit systematic position (SPEC S7), upper_bound in the shard CDF, gather of the ancestor
//   state. All integer; ancestors are bit-identical to oracle/pf_oracle.c for any shard count.
#pragma clang fp contract(off)
#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

__global__ __launch_bounds__(256) void k_predict(float* __restrict__ xs, float* __restrict__ ys,
                                                 float* __restrict__ ss, int64_t n, int64_t gbegin,
                                                 uint32_t k0, uint32_t k1, uint32_t frame, float sig_x,
                                                 float sig_y, float sig_s, float width, float height,
                                                 float smin, float smax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32x4 r = philox4x32_10((uint32_t)(gbegin + i), frame, 0u, 0u, k0, k1);
    const float u0 = uniform01(r.v[0]), u1 = uniform01(r.v[1]);
    const float u2 = uniform01(r.v[2]), u3 = uniform01(r.v[3]);
    const float ra = __builtin_sqrtf(-2.0f * fixed_logf(u0));
    const float rb = __builtin_sqrtf(-2.0f * fixed_logf(u2));
    float c1, s1, c3, s3;
    fixed_sincos2pi(u1, c1, s1);
    fixed_sincos2pi(u3, c3, s3);
    const float n0 = ra * c1, n1 = ra * s1, n2 = rb * c3;
    float x = fmaf(sig_x, n0, xs[i]);
    float y = fmaf(sig_y, n1, ys[i]);
    float s = ss[i] * fixed_expf(sig_s * n2);
    x = fminf(fmaxf(x, 0.0f), width - 1.0f);
    y = fminf(fmaxf(y, 0.0f), height - 1.0f);
    s = fminf(fmaxf(s, smin), smax);
    xs[i] = x; ys[i] = y; ss[i] = s;
}

VPF_API int vpf_predict(float* particles, int64_t n, int64_t ld, int64_t global_begin, uint64_t seed,
                        uint32_t frame, float sig_x, float sig_y, float sig_s, float width, float height,
                        float smin, float smax, void* stream) {
    if (n < 0 || ld < n || global_begin < 0 || (global_begin + n) > (int64_t)0xffffffffLL) return VPF_ERR_ARG;
    if (n == 0) return 0;
    const int threads = 256;
    const unsigned blocks = (unsigned)((n + threads - 1) / threads);
    hipLaunchKernelGGL(k_predict, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, particles,
                       particles + ld, particles + 2 * ld, n, global_begin, (uint32_t)seed,
                       (uint32_t)(seed >> 32), frame, sig_x, sig_y, sig_s, width, height, smin, smax);
    VPF_RETURN_LAUNCH();
}

// ---------------- shard stats (SPEC S6) ----------------
__global__ __launch_bounds__(1024) void k_shard_stats(const int64_t* __restrict__ Q,
                                                      const float* __restrict__ xs,
                                                      const float* __restrict__ ys,
                                                      const float* __restrict__ ss, int64_t n,
                                                      int64_t* out_T, double* out_sums) {
    __shared__ int64_t sT[1024];
    __shared__ double sx[1024], sy[1024], sz[1024];
    const int t = threadIdx.x;
    int64_t T = 0;
    double ax = 0, ay = 0, az = 0;
    for (int64_t i = t; i < n; i += 1024) {
        const int64_t q = Q[i];
        const double qd = (double)q;
        T += q;
        ax += qd * (double)xs[i]; ay += qd * (double)ys[i]; az += qd * (double)ss[i];
    }
    sT[t] = T; sx[t] = ax; sy[t] = ay; sz[t] = az;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (t < o) {
            sT[t] += sT[t + o]; sx[t] += sx[t + o]; sy[t] += sy[t + o]; sz[t] += sz[t + o];
        }
        __syncthreads();
    }
    if (t == 0) { out_T[0] = sT[0]; out_sums[0] = sx[0]; out_sums[1] = sy[0]; out_sums[2] = sz[0]; }
}

VPF_API int vpf_shard_stats(const int64_t* Q, const float* particles, int64_t ld, int64_t n,
                            int64_t* out_T, double* out_sums, void* stream) {
    if (n < 0 || ld < n) return VPF_ERR_ARG;
    hipLaunchKernelGGL(k_shard_stats, dim3(1), dim3(1024), 0, (hipStream_t)stream, Q, particles,
                       particles + ld, particles + 2 * ld, n, out_T, out_sums);
    VPF_RETURN_LAUNCH();
}

// ---------------- resample (SPEC S7) ----------------
__device__ __forceinline__ int64_t wave_incl_scan(int64_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

// Inclusive scan of Q (or of 1s when uniform) into cdf. One workgroup, 1024 threads, 4 per thread.
__global__ __launch_bounds__(1024) void k_scan(const int64_t* __restrict__ Q, int64_t n, int uniform,
                                               int64_t* __restrict__ cdf) {
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry_s;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (int64_t base = 0; base < n; base += 4096) {
        int64_t v[4];
        int64_t loc = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t i = base + (int64_t)t * 4 + e;
            const int64_t q = (i < n) ? (uniform ? (int64_t)1 : Q[i]) : (int64_t)0;
            loc += q;
            v[e] = loc;
        }
        const int64_t incl = wave_incl_scan(loc, lane);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        int64_t wprefix = 0;
        for (int w = 0; w < wid; ++w) wprefix += wsum[w];
        const int64_t excl = carry_s + wprefix + (incl - loc);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t i = base + (int64_t)t * 4 + e;
            if (i < n) cdf[i] = excl + v[e];
        }
        __syncthreads();
        if (t == 1023) {
            int64_t tot = 0;
            for (int w = 0; w < 16; ++w) tot += wsum[w];
            carry_s += tot;
        }
        __syncthreads();
    }
}

__device__ __forceinline__ uint64_t sys_position(uint64_t j, uint64_t T, uint64_t P, uint32_t U) {
    const uint64_t u = (uint64_t)U * (T >> 32) + (((uint64_t)U * (T & 0xffffffffull)) >> 32);
    const uint64_t qT = T / P, rT = T % P, qu = u / P, ru = u % P;
    return j * qT + qu + (j * rT + ru) / P;
}

__global__ __launch_bounds__(256) void k_resample_search(
    const int64_t* __restrict__ cdf, int64_t n_local, int64_t global_begin, int64_t offset, int64_t total,
    int64_t P, uint32_t U, int64_t slot_begin, int64_t slot_end, const float* __restrict__ xs,
    const float* __restrict__ ys, const float* __restrict__ ss, int32_t* __restrict__ anc,
    float* __restrict__ ox, float* __restrict__ oy, float* __restrict__ os) {
    const int64_t jj = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t j = slot_begin + jj;
    if (j >= slot_end) return;
    const uint64_t pos = sys_position((uint64_t)j, (uint64_t)total, (uint64_t)P, U);
    // local position; the caller guarantees pos in [offset, offset + shard total)
    const uint64_t lp = pos - (uint64_t)offset;
    int64_t lo = 0, hi = n_local - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((uint64_t)cdf[mid] > lp) hi = mid; else lo = mid + 1;
    }
    anc[jj] = (int32_t)(global_begin + lo);
    ox[jj] = xs[lo]; oy[jj] = ys[lo]; os[jj] = ss[lo];
}

VPF_API int vpf_resample(const int64_t* Q, int64_t n_local, int64_t global_begin, int64_t offset,
                         int64_t total, int64_t P, uint32_t U, int uniform, int64_t slot_begin,
                         int64_t slot_end, const float* particles, int64_t ld, int32_t* anc_out,
                         float* states_out, int64_t out_ld, int64_t* cdf_ws, void* stream) {
    if (n_local < 0 || ld < n_local || P <= 0 || total <= 0 || slot_begin < 0 || slot_end < slot_begin ||
        slot_end > P || out_ld < slot_end - slot_begin || offset < 0)
        return VPF_ERR_ARG;
    const int64_t cnt = slot_end - slot_begin;
    if (cnt == 0) return 0;
    if (n_local == 0) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, Q, n_local, uniform, cdf_ws);
    const unsigned blocks = (unsigned)((cnt + 255) / 256);
    hipLaunchKernelGGL(k_resample_search, dim3(blocks), dim3(256), 0, s, cdf_ws, n_local, global_begin,
                       offset, total, P, U, slot_begin, slot_end, particles, particles + ld,
                       particles + 2 * ld, anc_out, states_out, states_out + out_ld,
                       states_out + 2 * out_ld);
    VPF_RETURN_LAUNCH();
}

// ---------------- estimate + resample over the global particle set (SPEC S6 + S7, device-resident) -------------
// The product path (ParticleFilter): every rank holds the GLOBAL weights and states — its own arrays (world 1) or
// the all-gathered shard chunks (world > 1, one fixed-size all-gather of 20 B per particle) — so the totals, the
// CDF, the resample word and the ancestors of its own output slots are computed on the device with no host
// round trip in between, and every rank (and every world size) sums in the same fixed order over the global
// index: the estimate is bit-identical for any G. Global index i lives in shard r = i / n_shard at k = i % n_shard.
struct GlobalView {
    const int64_t* Q;
    int64_t q_stride;      // int64 elements from shard r's Q to shard r + 1's
    const float* p;        // shard 0's x row; y at + ld, s at + 2 ld
    int64_t ld;
    int64_t p_stride;      // floats from shard r's x row to shard r + 1's
    uint32_t n_shard;
    __device__ __forceinline__ int64_t off(uint32_t i, int64_t stride) const {
        const uint32_t r = i / n_shard;
        return (int64_t)r * stride + (int64_t)(i - r * n_shard);
    }
    __device__ __forceinline__ int64_t q(uint32_t i) const { return Q[off(i, q_stride)]; }
    __device__ __forceinline__ const float* state(uint32_t i) const { return p + off(i, p_stride); }
};

// One workgroup: SPEC S6 sums in k_shard_stats' fixed tree (thread t takes i = t, t + 1024, ... in order, then
// pairwise halving), repeated with every Q_i = 1 when T == 0 (the uniform fallback's plain sums); then the
// inclusive int64 CDF (k_scan's chunked wave scan). stats_out = {T, bits of the three fp64 sums}.
__global__ __launch_bounds__(1024) void k_stats_scan_global(GlobalView g, int64_t P, int64_t* __restrict__ cdf,
                                                            int64_t* __restrict__ stats_out) {
    __shared__ int64_t sT[1024];
    __shared__ double sx[1024], sy[1024], sz[1024];
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry_s;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    for (int pass = 0; pass < 2; ++pass) {
        int64_t T = 0;
        double ax = 0, ay = 0, az = 0;
        for (int64_t i = t; i < P; i += 1024) {
            const float* st = g.state((uint32_t)i);
            const int64_t q = pass == 0 ? g.q((uint32_t)i) : (int64_t)1;
            const double qd = (double)q;
            T += q;
            ax += qd * (double)st[0]; ay += qd * (double)st[g.ld]; az += qd * (double)st[2 * g.ld];
        }
        sT[t] = T; sx[t] = ax; sy[t] = ay; sz[t] = az;
        __syncthreads();
        for (int o = 512; o > 0; o >>= 1) {
            if (t < o) {
                sT[t] += sT[t + o]; sx[t] += sx[t + o]; sy[t] += sy[t + o]; sz[t] += sz[t + o];
            }
            __syncthreads();
        }
        const int64_t Tall = sT[0];
        if (pass == 0 && t == 0) stats_out[0] = Tall;
        if (pass == 1 || Tall != 0) {
            if (t == 0) {
                stats_out[1] = __double_as_longlong(sx[0]);
                stats_out[2] = __double_as_longlong(sy[0]);
                stats_out[3] = __double_as_longlong(sz[0]);
            }
            break;
        }
        __syncthreads();   // every thread has read sT[0] before pass 1 rewrites the tree
    }
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (int64_t base = 0; base < P; base += 4096) {
        int64_t v[4];
        int64_t loc = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t i = base + (int64_t)t * 4 + e;
            loc += (i < P) ? g.q((uint32_t)i) : (int64_t)0;
            v[e] = loc;
        }
        const int64_t incl = wave_incl_scan(loc, lane);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        int64_t wprefix = 0;
        for (int w = 0; w < wid; ++w) wprefix += wsum[w];
        const int64_t excl = carry_s + wprefix + (incl - loc);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t i = base + (int64_t)t * 4 + e;
            if (i < P) cdf[i] = excl + v[e];
        }
        __syncthreads();
        if (t == 1023) {
            int64_t tot = 0;
            for (int w = 0; w < 16; ++w) tot += wsum[w];
            carry_s += tot;
        }
        __syncthreads();
    }
}

// One thread per output slot j in [slot_begin, slot_end): T = cdf[P-1] (0 -> uniform: C_i = i + 1, so a_j =
// pos_j), U = Philox(ctr = (0, frame, 1, 0), key = seed) word 0 (SPEC S1), pos_j exact (SPEC S7), a_j =
// min{i : C_i > pos_j} by binary search over the global CDF, and the ancestor's state.
__global__ __launch_bounds__(256) void k_resample_global(const int64_t* __restrict__ cdf, int64_t P, uint32_t k0,
                                                         uint32_t k1, uint32_t frame, int64_t slot_begin,
                                                         int64_t slot_end, GlobalView g, int32_t* __restrict__ anc,
                                                         float* __restrict__ ox, float* __restrict__ oy,
                                                         float* __restrict__ os) {
    const int64_t jj = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t j = slot_begin + jj;
    if (j >= slot_end) return;
    const int64_t T = cdf[P - 1];
    const uint32_t U = philox4x32_10(0u, frame, 1u, 0u, k0, k1).v[0];
    const uint64_t pos = sys_position((uint64_t)j, (uint64_t)(T == 0 ? P : T), (uint64_t)P, U);
    int64_t lo;
    if (T == 0) {
        lo = (int64_t)pos;
    } else {
        int64_t hi = P - 1;
        lo = 0;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((uint64_t)cdf[mid] > pos) hi = mid; else lo = mid + 1;
        }
    }
    const float* st = g.state((uint32_t)lo);
    anc[jj] = (int32_t)lo;
    ox[jj] = st[0]; oy[jj] = st[g.ld]; os[jj] = st[2 * g.ld];
}

VPF_API int vpf_estimate_resample(const int64_t* Q, int64_t q_stride, const float* particles, int64_t ld,
                                  int64_t p_stride, int64_t n_shard, int64_t P, uint64_t seed, uint32_t frame,
                                  int64_t slot_begin, int64_t slot_end, int32_t* anc_out, float* states_out,
                                  int64_t out_ld, int64_t* cdf_ws, int64_t* stats_out, void* stream) {
    if (P <= 0 || P > 0x7fffffffLL || n_shard <= 0 || P % n_shard != 0 || ld < n_shard || slot_begin < 0 ||
        slot_end < slot_begin || slot_end > P || out_ld < slot_end - slot_begin)
        return VPF_ERR_ARG;
    if (P > n_shard && (q_stride < n_shard || p_stride < 2 * ld + n_shard)) return VPF_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const GlobalView g{Q, q_stride, particles, ld, p_stride, (uint32_t)n_shard};
    hipLaunchKernelGGL(k_stats_scan_global, dim3(1), dim3(1024), 0, s, g, P, cdf_ws, stats_out);
    const int64_t cnt = slot_end - slot_begin;
    if (cnt > 0)
        hipLaunchKernelGGL(k_resample_global, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, cdf_ws, P,
                           (uint32_t)seed, (uint32_t)(seed >> 32), frame, slot_begin, slot_end, g, anc_out,
                           states_out, states_out + out_ld, states_out + 2 * out_ld);
    VPF_RETURN_LAUNCH();
}

VPF_API const char* vpf_version(void) { return "libvpf 0.1.0 gfx950"; }
