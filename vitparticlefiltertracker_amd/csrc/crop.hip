// Particle crop gather (SPEC S3) and CLS rows (H3).
//
// vpf_crop_patches_*: the frame is first expanded into a zero-bordered RGBA workspace (one dword per pixel:
// every bilinear tap is one aligned load, no bounds branch), then each thread writes 8 consecutive im2col
// columns (16-B bf16 stores, coalesced across the wave): all three channels of 8 pixels on the fast path
// (patch % 8 == 0), 8 columns of one channel otherwise. The frame (150 KB at 224x224) stays L2-resident.
// Arithmetic order is SPEC S3's, contraction off, so the fp32 values are bit-identical to
// oracle/pf_oracle.c and the bf16 values are their RNE rounding.
#pragma clang fp contract(off)
#include <cstdlib>

#include "vpf_common.h"
#include "../../include/vpf.h"

using namespace vpf;

struct NormAB { float a[3]; float b[3]; };

// The frame as a zero-bordered RGBA image: rgba[(y+1)*(W+2) + (x+1)] = r | g << 8 | b << 16 for the pixel
// (y, x), 0 on the one-pixel border. A bilinear tap is then ONE aligned dword load with no bounds branch
// (coordinates clamp into the border, whose zeros are SPEC S3's zero padding).
__global__ __launch_bounds__(256) void k_frame_rgba(const uint8_t* __restrict__ frame, int H, int W,
                                                    uint32_t* __restrict__ rgba) {
    const int Wp = W + 2;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)(H + 2) * Wp) return;
    const int py = (int)(idx / Wp), px = (int)(idx - (int64_t)py * Wp);
    const int y = py - 1, x = px - 1;
    uint32_t v = 0;
    if (y >= 0 && y < H && x >= 0 && x < W) {
        const uint8_t* q = frame + ((int64_t)y * W + x) * 3;
        v = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16);
    }
    rgba[idx] = v;
}

__device__ __forceinline__ uint32_t rgba_tap(const uint32_t* __restrict__ rgba, int H, int W, int yy, int xx) {
    yy = min(max(yy, -1), H);
    xx = min(max(xx, -1), W);
    return rgba[(int64_t)(yy + 1) * (W + 2) + (xx + 1)];
}
__device__ __forceinline__ float chan(uint32_t px, int c) { return (float)((px >> (8 * c)) & 255u); }

// Fast path (patch % 8 == 0, Kp == 3 patch^2), LDS-staged: one 512-thread workgroup per particle; a thread writes 8
// consecutive output pixels of one patch row (ky, kx0..kx0+7) in all three channels, the source row (sy, fy, iy)
// computed once, each sample's column once, and one dword tap serving all three channels. The particle's source window (every
// bilinear tap of its S x S samples, clamped into the zero border as rgba_tap does) is copied from the RGBA workspace
// into LDS once, and the taps read LDS instead of issuing 32 gathered dword loads per thread through the vector
// memory path, which bound the global form (the im2col stores are the same). A window larger than CROP_LDS_DW dwords
// (a large template at a large scale) takes the global taps. Same per-value arithmetic (and order) as the generic
// kernel and the oracle.
constexpr int CROP_LDS_DW = 10240;   // 40 KiB: four workgroups per CU (0.45-0.49 vs 0.53 ms at 80 KiB and two per CU,
// profiles/r2_gemm_lab/crop_lds_window_ab.txt); windows up to ~101 x 101 (a 64 x 64 template to scale ~1.55)
// The particle's crop geometry and its source window (every bilinear tap of its S x S samples, clamped into the zero
// border as rgba_tap does), staged into LDS when it fits; shared by both LDS kernels.
struct CropWin {
    float x0, y0, dx, dy;
    int cx0, cy0, wx;
    bool staged;
};
template <int NT>
__device__ __forceinline__ CropWin stage_window(uint32_t* win, const uint32_t* __restrict__ rgba, int H, int W, float xc,
                                                float yc, float sc, float w0, float h0, int S) {
    CropWin cw;
    const float bw = sc * w0, bh = sc * h0;
    cw.x0 = xc - 0.5f * bw;
    cw.y0 = yc - 0.5f * bh;
    cw.dx = bw / (float)S;
    cw.dy = bh / (float)S;
    // tap range: the sample coordinate is monotone in the output index, so the first and last samples bound it
    const int ix_lo = (int)floorf((cw.x0 + (0.0f + 0.5f) * cw.dx) - 0.5f);
    const int ix_hi = (int)floorf((cw.x0 + ((float)(S - 1) + 0.5f) * cw.dx) - 0.5f) + 1;
    const int iy_lo = (int)floorf((cw.y0 + (0.0f + 0.5f) * cw.dy) - 0.5f);
    const int iy_hi = (int)floorf((cw.y0 + ((float)(S - 1) + 0.5f) * cw.dy) - 0.5f) + 1;
    cw.cx0 = min(max(ix_lo, -1), W);
    const int cx1 = min(max(ix_hi, -1), W);
    cw.cy0 = min(max(iy_lo, -1), H);
    const int cy1 = min(max(iy_hi, -1), H);
    cw.wx = cx1 - cw.cx0 + 1;
    const int wy = cy1 - cw.cy0 + 1;
    cw.staged = cw.wx * wy <= CROP_LDS_DW;   // workgroup-uniform
    if (cw.staged) {
        for (int i = threadIdx.x; i < cw.wx * wy; i += NT) {
            const int r = i / cw.wx, c = i - r * cw.wx;
            win[i] = rgba[(int64_t)(cw.cy0 + r + 1) * (W + 2) + (cw.cx0 + c + 1)];
        }
    }
    __syncthreads();
    return cw;
}
__device__ __forceinline__ uint32_t win_tap(const CropWin& cw, const uint32_t* win, const uint32_t* __restrict__ rgba,
                                            int H, int W, int yy, int xx) {
    if (cw.staged) return win[(min(max(yy, -1), H) - cw.cy0) * cw.wx + (min(max(xx, -1), W) - cw.cx0)];
    return rgba_tap(rgba, H, W, yy, xx);
}

template <typename OutT>
__global__ __launch_bounds__(512) void k_crop_patches_lds(const uint32_t* __restrict__ rgba, int H, int W,
                                                          const float* __restrict__ xs, const float* __restrict__ ys,
                                                          const float* __restrict__ ss, int n_patches, int g, float w0,
                                                          float h0, int S, int patch, NormAB nab,
                                                          OutT* __restrict__ out, int split) {
    __shared__ uint32_t win[CROP_LDS_DW];
    // `split` workgroups per particle (small batches: the 8-GPU share's 512 particles would fill 2 workgroups per CU),
    // each staging the window and writing a contiguous share of the particle's rows
    const int64_t p = blockIdx.x / split;
    const int part = blockIdx.x - (int)(p * split);
    const CropWin cw = stage_window<512>(win, rgba, H, W, xs[p], ys[p], ss[p], w0, h0, S);
    const float x0 = cw.x0, y0 = cw.y0, dx = cw.dx, dy = cw.dy;
    auto tap = [&](int yy, int xx) -> uint32_t { return win_tap(cw, win, rgba, H, W, yy, xx); };
    const int per_row = patch * (patch >> 3);             // threads per im2col row
    const int pp = patch * patch;
    const int total = n_patches * per_row;
    const int t_end = (int)((int64_t)total * (part + 1) / split);
    for (int t = (int)((int64_t)total * part / split) + threadIdx.x; t < t_end; t += 512) {
        const int pi = t / per_row;
        const int tt = t - pi * per_row;
        const int ky = tt / (patch >> 3), kx0 = (tt - ky * (patch >> 3)) * 8;
        const int py = pi / g, px = pi - (pi / g) * g;
        const int oy = py * patch + ky;
        const float sy = (y0 + ((float)oy + 0.5f) * dy) - 0.5f;
        const float fy0 = floorf(sy);
        const float fy = sy - fy0;
        const int iy = (int)fy0;
        float vals[3][8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int ox = px * patch + kx0 + e;
            const float sx = (x0 + ((float)ox + 0.5f) * dx) - 0.5f;
            const float fx0 = floorf(sx);
            const float fx = sx - fx0;
            const int ix = (int)fx0;
            const uint32_t t00 = tap(iy, ix), t01 = tap(iy, ix + 1);
            const uint32_t t10 = tap(iy + 1, ix), t11 = tap(iy + 1, ix + 1);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float top = (1.0f - fx) * chan(t00, c) + fx * chan(t01, c);
                const float bot = (1.0f - fx) * chan(t10, c) + fx * chan(t11, c);
                const float v = (1.0f - fy) * top + fy * bot;
                vals[c][e] = fmaf(v, nab.a[c], nab.b[c]);
            }
        }
        const int64_t row = p * n_patches + pi;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            OutT* dst = out + row * (int64_t)(3 * pp) + c * pp + ky * patch + kx0;
            if constexpr (sizeof(OutT) == 2) {
                uint4 pk;
                pk.x = pack_bf2(vals[c][0], vals[c][1]); pk.y = pack_bf2(vals[c][2], vals[c][3]);
                pk.z = pack_bf2(vals[c][4], vals[c][5]); pk.w = pack_bf2(vals[c][6], vals[c][7]);
                *reinterpret_cast<uint4*>(dst) = pk;
            } else {
                *reinterpret_cast<float4*>(dst) = make_float4(vals[c][0], vals[c][1], vals[c][2], vals[c][3]);
                *reinterpret_cast<float4*>(dst + 4) = make_float4(vals[c][4], vals[c][5], vals[c][6], vals[c][7]);
            }
        }
    }
}

// Any patch / Kp (ViT-L/14: patch 14, Kp = 640 > 3 x 196), LDS-staged like the fast path: one 512-thread workgroup
// per particle stages its source window, then a thread walks one patch row (ky) of one patch: each sample's source row
// and column are computed once and one dword tap serves all three channels; bf16 pairs go out as dword stores (even
// patch). The columns past 3 patch^2 are the zero padding. Same per-value arithmetic (and order) as the oracle.
// Round 5: replaces a global-tap form (4.8 ms per ViT-L frame) and a per-element form (4.35 ms) whose index and tap
// work was repeated for every channel.
template <typename OutT>
__global__ __launch_bounds__(512) void k_crop_patches_gen(const uint32_t* __restrict__ rgba, int H, int W,
                                                          const float* __restrict__ xs, const float* __restrict__ ys,
                                                          const float* __restrict__ ss, int n_patches, int g, float w0,
                                                          float h0, int S, int patch, int Kp, NormAB nab,
                                                          OutT* __restrict__ out) {
    __shared__ uint32_t win[CROP_LDS_DW];
    const int64_t p = blockIdx.x;
    const CropWin cw = stage_window<512>(win, rgba, H, W, xs[p], ys[p], ss[p], w0, h0, S);
    auto tap = [&](int yy, int xx) -> uint32_t { return win_tap(cw, win, rgba, H, W, yy, xx); };
    const int pp = patch * patch, K = 3 * pp;
    OutT* const base = out + p * n_patches * (int64_t)Kp;
    const bool pairs = sizeof(OutT) == 2 && (patch & 1) == 0;   // 4-B aligned bf16 pairs
    for (int t = threadIdx.x; t < n_patches * patch; t += 512) {
        const int pi = t / patch, ky = t - pi * patch;
        const int py = pi / g, px = pi - py * g;
        const float sy = (cw.y0 + ((float)(py * patch + ky) + 0.5f) * cw.dy) - 0.5f;
        const float fy0 = floorf(sy);
        const float fy = sy - fy0;
        const int iy = (int)fy0;
        OutT* const row = base + (int64_t)pi * Kp + ky * patch;
        for (int kx = 0; kx < patch; kx += 2) {
            float v[3][2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int ox = px * patch + min(kx + e, patch - 1);   // odd patch: the last pair repeats a column
                const float sx = (cw.x0 + ((float)ox + 0.5f) * cw.dx) - 0.5f;
                const float fx0 = floorf(sx);
                const float fx = sx - fx0;
                const int ix = (int)fx0;
                const uint32_t t00 = tap(iy, ix), t01 = tap(iy, ix + 1);
                const uint32_t t10 = tap(iy + 1, ix), t11 = tap(iy + 1, ix + 1);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float top = (1.0f - fx) * chan(t00, c) + fx * chan(t01, c);
                    const float bot = (1.0f - fx) * chan(t10, c) + fx * chan(t11, c);
                    const float vv = (1.0f - fy) * top + fy * bot;
                    v[c][e] = fmaf(vv, nab.a[c], nab.b[c]);
                }
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                OutT* dst = row + c * pp + kx;
                if constexpr (sizeof(OutT) == 2) {
                    const uint32_t pk = pack_bf2(v[c][0], v[c][1]);
                    if (pairs) {
                        *reinterpret_cast<uint32_t*>(dst) = pk;
                    } else {
                        dst[0] = (OutT)(pk & 0xffffu);
                        if (kx + 1 < patch) dst[1] = (OutT)(pk >> 16);
                    }
                } else {
                    dst[0] = v[c][0];
                    if (kx + 1 < patch) dst[1] = v[c][1];
                }
            }
        }
    }
    const int pad = Kp - K;
    for (int t = threadIdx.x; t < n_patches * pad; t += 512) {
        const int pi = t / pad;
        base[(int64_t)pi * Kp + K + (t - pi * pad)] = (OutT)0;
    }
}

template <typename OutT>
static int crop_launch(const uint8_t* frame, int H, int W, uint32_t* rgba_ws, const float* particles, int64_t ld,
                       int64_t n, float w0, float h0, int S, int patch, int Kp, const float* norm_ab_host, OutT* out,
                       void* stream) {
    if (H <= 0 || W <= 0 || n < 0 || ld < n || patch <= 0 || S % patch != 0 || Kp % 8 != 0 ||
        Kp < 3 * patch * patch || !norm_ab_host || !frame || !rgba_ws)
        return VPF_ERR_ARG;
    if ((int64_t)(H + 2) * (W + 2) > INT32_MAX) return VPF_ERR_ARG;
    if (n == 0) return 0;
    NormAB nab;
    for (int c = 0; c < 3; ++c) { nab.a[c] = norm_ab_host[c]; nab.b[c] = norm_ab_host[3 + c]; }
    hipStream_t st = (hipStream_t)stream;
    const int64_t npix = (int64_t)(H + 2) * (W + 2);
    hipLaunchKernelGGL(k_frame_rgba, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, frame, H, W, rgba_ws);
    const int g = S / patch;
    if (patch % 8 == 0 && Kp == 3 * patch * patch && n <= INT32_MAX / 4) {
        const int split = n >= 2048 ? 1 : n >= 1024 ? 2 : 4;   // at least ~4096 workgroups when the batch is small
        hipLaunchKernelGGL(k_crop_patches_lds<OutT>, dim3((unsigned)(n * split)), dim3(512), 0, st, rgba_ws, H, W,
                           particles, particles + ld, particles + 2 * ld, g * g, g, w0, h0, S, patch, nab, out, split);
    } else if (n <= INT32_MAX) {
        hipLaunchKernelGGL(k_crop_patches_gen<OutT>, dim3((unsigned)n), dim3(512), 0, st, rgba_ws, H, W, particles,
                           particles + ld, particles + 2 * ld, g * g, g, w0, h0, S, patch, Kp, nab, out);
    } else {
        return VPF_ERR_ARG;
    }
    VPF_RETURN_LAUNCH();
}

VPF_API int vpf_crop_patches_bf16(const uint8_t* frame, int H, int W, uint32_t* rgba_ws, const float* particles,
                                  int64_t ld, int64_t n, float w0, float h0, int S, int patch, int Kp,
                                  const float* norm_ab_host, uint16_t* out, void* stream) {
    return crop_launch<uint16_t>(frame, H, W, rgba_ws, particles, ld, n, w0, h0, S, patch, Kp, norm_ab_host, out,
                                 stream);
}

VPF_API int vpf_crop_patches_f32(const uint8_t* frame, int H, int W, uint32_t* rgba_ws, const float* particles,
                                 int64_t ld, int64_t n, float w0, float h0, int S, int patch, int Kp,
                                 const float* norm_ab_host, float* out, void* stream) {
    return crop_launch<float>(frame, H, W, rgba_ws, particles, ld, n, w0, h0, S, patch, Kp, norm_ab_host, out,
                              stream);
}

// ---------------- CLS rows: tokens[p][0][:] = cls + pos[0] ----------------
template <typename T>
__global__ __launch_bounds__(256) void k_cls_rows(T* __restrict__ tok, int64_t n_part, int N, int D,
                                                  const float* __restrict__ cls, const float* __restrict__ pos) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= n_part * D) return;
    const int64_t p = tid / D;
    const int d = (int)(tid - p * D);
    const float v = cls[d] + pos[d];
    if constexpr (sizeof(T) == 2) tok[p * (int64_t)N * D + d] = f2bf(v);
    else tok[p * (int64_t)N * D + d] = v;
}

// Stats-plane entries of the CLS rows (vpf_gemm_bf16 stats_out layout): every CLS row holds the same bf16
// values bf16(cls + pos[0]), so one workgroup reduces {sum, sumsq} once and writes it to plane 0 of each
// particle's CLS row (planes 1.. get 0: the consumer sums the planes).
__global__ __launch_bounds__(256) void k_cls_stats(int64_t n_part, int N, int D, const float* __restrict__ cls,
                                                   const float* __restrict__ pos, float2* __restrict__ st,
                                                   int parts) {
    __shared__ float red[2][4];
    float s = 0.f, q = 0.f;
    for (int d = threadIdx.x; d < D; d += 256) {
        const float v = bf2f(f2bf(cls[d] + pos[d]));
        s += v;
        q = fmaf(v, v, q);
    }
    s = wave_sum(s);
    q = wave_sum(q);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = s; red[1][w] = q; }
    __syncthreads();
    const float2 t = make_float2(red[0][0] + red[0][1] + red[0][2] + red[0][3],
                                 red[1][0] + red[1][1] + red[1][2] + red[1][3]);
    const int64_t rows = n_part * N;
    for (int64_t p = threadIdx.x; p < n_part; p += 256)
        for (int k = 0; k < parts; ++k) st[k * rows + p * N] = k == 0 ? t : make_float2(0.f, 0.f);
}

VPF_API int vpf_cls_rows_bf16(uint16_t* tokens, int64_t n_part, int N, int D, const float* cls,
                              const float* pos, float* stats_out, int parts, void* stream) {
    if (n_part < 0 || N <= 0 || D <= 0) return VPF_ERR_ARG;
    if (stats_out && (parts < 1 || parts > 64 || ((uintptr_t)stats_out & 7))) return VPF_ERR_ARG;
    if (n_part == 0) return 0;
    const unsigned blocks = (unsigned)((n_part * D + 255) / 256);
    hipLaunchKernelGGL(k_cls_rows<uint16_t>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, tokens, n_part, N,
                       D, cls, pos);
    if (stats_out) {
        const int e = (int)hipGetLastError();
        if (e) return e;
        hipLaunchKernelGGL(k_cls_stats, dim3(1), dim3(256), 0, (hipStream_t)stream, n_part, N, D, cls, pos,
                           reinterpret_cast<float2*>(stats_out), parts);
    }
    VPF_RETURN_LAUNCH();
}

VPF_API int vpf_cls_rows_f32(float* tokens, int64_t n_part, int N, int D, const float* cls, const float* pos,
                             void* stream) {
    if (n_part < 0 || N <= 0 || D <= 0) return VPF_ERR_ARG;
    if (n_part == 0) return 0;
    const unsigned blocks = (unsigned)((n_part * D + 255) / 256);
    hipLaunchKernelGGL(k_cls_rows<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, tokens, n_part, N, D,
                       cls, pos);
    VPF_RETURN_LAUNCH();
}
