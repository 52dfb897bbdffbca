// Loss and head backward.
//
//  * hkp_heat_loss   train.py:21,25 — nn.BCELoss()(pred.double(), gt) with the
//                    Gaussian target (dataset.py:36-44) read from a dense fp64
//                    tensor or recomputed in registers from (u, v); MSE (train.py:13)
//                    selectable.  fp64 loss, fp64 per-element gradient:
//                      BCE  l = (y-1)*max(log1p(-p),-100) - y*max(log p,-100)
//                           g = (p-y) / max((1-p)*p, 1e-12) / N
//                      MSE  l = (p-y)^2,  g = 2 (p-y) / N
//                    then cast to fp32 (the .double() cast's backward).
//  * hkp_head_bwd    sigmoid backward (g*(1-p))*p (model.py:21) fused with the
//                    adjoint of the align_corners=True upsample (resnet_dilated.py:27)
//                    as two separable gathers (rows, then columns; no atomics).
//  * hkp_head_fc_bwd fc 1x1 (resnet_dilated.py:16) grads: dfeat (NHWC), dW, db for
//                    the K used rows; rows >= K get exactly zero.
#include "common.h"

#pragma clang fp contract(off)

namespace hkp {

struct LerpB {
    int i0, i1;
    float l0, l1;
};

// identical to head.hip's lerp_index (ATen align_corners=True, fp32)
__device__ __forceinline__ LerpB lerp_b(int o, int in, int out, float scale) {
    LerpB r;
    if (in == out) {
        r.i0 = r.i1 = o;
        r.l0 = 1.f;
        r.l1 = 0.f;
        return r;
    }
    const float src = scale * (float)o;
    int i0 = (int)floorf(src);
    i0 = i0 < in - 1 ? i0 : in - 1;
    float l1 = src - (float)i0;
    l1 = fminf(fmaxf(l1, 0.f), 1.f);
    r.i0 = i0;
    r.i1 = i0 + (i0 < in - 1 ? 1 : 0);
    r.l1 = l1;
    r.l0 = 1.f - l1;
    return r;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
    v = wave_sum_d(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    return t;
}

template <int KIND, bool DENSE>
__global__ __launch_bounds__(256) void heat_loss_kernel(long total, int H, int W, float den, double inv_n,
                                                       const float* __restrict__ p, const double* __restrict__ gt,
                                                       const float* __restrict__ uv, float* __restrict__ dheat,
                                                       double* __restrict__ part) {
    __shared__ double red[4];
    const long HW = (long)H * W;
    const long stride = (long)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        double y;
        if constexpr (DENSE) {
            y = gt[i];
        } else {
            const long plane = i / HW;
            const long r = i - plane * HW;
            const int yy = (int)(r / W), xx = (int)(r - (long)yy * W);
            const float dx = (float)xx - uv[plane * 2], dy = (float)yy - uv[plane * 2 + 1];
            y = (double)expf(-(dx * dx + dy * dy) / den);
        }
        const double x = (double)p[i];
        double l, g;
        if constexpr (KIND == HKP_LOSS_BCE) {
            l = (y - 1.0) * fmax(log1p(-x), -100.0) - y * fmax(log(x), -100.0);
            g = (x - y) / fmax((1.0 - x) * x, 1e-12) * inv_n;
        } else {
            l = (x - y) * (x - y);
            g = 2.0 * inv_n * (x - y);
        }
        acc += l;
        if (dheat) dheat[i] = (float)g;
    }
    const double t = block_sum_d(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void loss_finalize_kernel(int nparts, double inv_n, const double* __restrict__ part, double* loss) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += part[i];
    const double t = block_sum_d(s, red);
    if (threadIdx.x == 0) loss[0] = t * inv_n;
}

// d_low[plane][i][j] = sum_oh wr_i(oh) * ( sum_ow wc_j(ow) * (g*(1-p))*p at (oh, ow) ),
// separable in two gathers (no atomics), each in the loop order of the direct
// double sum so the result is the same bit for bit:
//   pass 1 (rows): rs[plane][oh][j] = sum over the ow whose lerp touches j
//   pass 2 (cols): d_low[plane][i][j] = sum over the oh whose lerp touches i of wr * rs
// Each high-res element is read by <= 2 pass-1 threads (vs ~4 node gathers that
// each recomputed every candidate's lerp in the direct form).
__device__ __forceinline__ void cand_range(int i, int in, int out, float inv, int* o0, int* o1) {
    if (out != in) {
        *o0 = max(0, (int)floorf((float)(i - 1) * inv) - 1);
        *o1 = min(out - 1, (int)ceilf((float)(i + 1) * inv) + 1);
    } else {
        *o0 = *o1 = i;
    }
}

template <bool SIG>
__global__ __launch_bounds__(256) void head_bwd_rows_kernel(int planes, int w, int H, int W, float sw, float iw,
                                                           const float* __restrict__ g, const float* __restrict__ p,
                                                           float* __restrict__ rs) {
    const long total = (long)planes * H * w;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const int j = (int)(t % w);
        const long prow = t / w;                          // plane * H + oh
        int ow0, ow1;
        cand_range(j, w, W, iw, &ow0, &ow1);
        const float* gp = g + prow * (long)W;
        const float* pp = p + prow * (long)W;
        float row = 0.f;
        for (int ow = ow0; ow <= ow1; ++ow) {
            const LerpB lc = lerp_b(ow, w, W, sw);
            if (lc.i0 != j && lc.i1 != j) continue;
            const float wc = (lc.i0 == j ? lc.l0 : 0.f) + (lc.i1 == j ? lc.l1 : 0.f);
            float dzv = gp[ow];
            if constexpr (SIG) {
                const float pv = pp[ow];
                dzv = dzv * (1.f - pv) * pv;
            }
            row += wc * dzv;
        }
        rs[t] = row;
    }
}

__global__ __launch_bounds__(256) void head_bwd_cols_kernel(int planes, int h, int w, int H, float sh, float ih,
                                                           const float* __restrict__ rs, float* __restrict__ dlow) {
    const long total = (long)planes * h * w;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const int j = (int)(t % w);
        const long q = t / w;
        const int i = (int)(q % h);
        const long plane = q / h;
        int oh0, oh1;
        cand_range(i, h, H, ih, &oh0, &oh1);
        const float* r = rs + plane * (long)H * w + j;
        float acc = 0.f;
        for (int oh = oh0; oh <= oh1; ++oh) {
            const LerpB lr = lerp_b(oh, h, H, sh);
            if (lr.i0 != i && lr.i1 != i) continue;
            const float wr = (lr.i0 == i ? lr.l0 : 0.f) + (lr.i1 == i ? lr.l1 : 0.f);
            acc += wr * r[(long)oh * w];
        }
        dlow[t] = acc;
    }
}

// dfeat[m][c] = sum_k dlow[n][k][p] * W[k][c]
__global__ __launch_bounds__(256) void head_dfeat_kernel(long npix, int hw, int C, int K,
                                                        const float* __restrict__ dlow, const float* __restrict__ wgt,
                                                        float* __restrict__ dfeat) {
    const int C4 = C >> 2;
    const long total = npix * C4;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int c4 = (int)(i % C4);
        const long m = i / C4;
        const long n = m / hw, q = m - n * hw;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < K; ++k) {
            const float d = dlow[(n * K + k) * hw + q];
            const f32x4 ww = *(const f32x4*)(wgt + (long)k * C + 4 * c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] += d * ww[e];
        }
        *(f32x4*)(dfeat + i * 4) = acc;
    }
}

// partial dW[k][c] and db[k] over a pixel chunk; grid (splits, ceil(C4/256))
template <int KMAX>
__global__ __launch_bounds__(256) void head_dw_kernel(long npix, int hw, int C, int K, long pix_per_split,
                                                     const float* __restrict__ dlow, const float* __restrict__ feat,
                                                     float* __restrict__ ws_w, float* __restrict__ ws_b) {
    __shared__ float red[256 * 4];
    const int C4 = C >> 2;
    const int tprow = min(C4, 256);
    const int rpar = 256 / tprow;
    const int tid = threadIdx.x;
    const int rl = tid / tprow;
    const int c4 = blockIdx.y * tprow + (tid - rl * tprow);
    const long m0 = (long)blockIdx.x * pix_per_split;
    const long m1 = min(npix, m0 + pix_per_split);
    f32x4 acc[KMAX];
    float bacc[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        bacc[k] = 0.f;
    }
    if (c4 < C4) {
        for (long m = m0 + rl; m < m1; m += rpar) {
            const long n = m / hw, q = m - n * hw;
            const f32x4 f = *(const f32x4*)(feat + m * C + 4 * c4);
#pragma unroll
            for (int k = 0; k < KMAX; ++k) {
                if (k < K) {
                    const float d = dlow[(n * K + k) * hw + q];
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[k][e] += d * f[e];
                    bacc[k] += d;
                }
            }
        }
    }
    float* outw = ws_w + (long)blockIdx.x * K * C;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        if (k >= K) continue;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 4; ++e) red[tid * 4 + e] = acc[k][e];
        __syncthreads();
        if (rl == 0 && c4 < C4) {
            f32x4 s = {0.f, 0.f, 0.f, 0.f};
            for (int r = 0; r < rpar; ++r)
#pragma unroll
                for (int e = 0; e < 4; ++e) s[e] += red[(r * tprow + tid) * 4 + e];
            *(f32x4*)(outw + (long)k * C + 4 * c4) = s;
        }
    }
    if (blockIdx.y == 0) {
        // bias: one lane per row group (the c4 == 0 lane) saw each pixel once
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (k >= K) continue;
            __syncthreads();
            red[tid] = bacc[k];
            __syncthreads();
            if (tid == 0) {
                float s = 0.f;
                for (int r = 0; r < rpar; ++r) s += red[r * tprow];
                ws_b[(long)blockIdx.x * K + k] = s;
            }
        }
    }
}

// out[i] = sum_s ws[s][i] in a fixed order: 4 lanes per element each sum every
// 4th split, then the lane sums pairwise (the split count runs to hundreds)
__global__ __launch_bounds__(256) void sum_splits_kernel(long n, int splits, const float* __restrict__ ws,
                                                        float* __restrict__ out) {
    __shared__ float red[4][64];
    const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
    const long i = (long)blockIdx.x * 64 + l;
    float s = 0.f;
    if (i < n) {
#pragma unroll 8
        for (int k = q; k < splits; k += 4) s += ws[(long)k * n + i];
    }
    red[q][l] = s;
    __syncthreads();
    if (q == 0 && i < n) out[i] = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
}

static inline int gcap(long work) {
    long g = (work + 255) / 256;
    if (g > 4096) g = 4096;
    return (int)(g < 1 ? 1 : g);
}

constexpr int LOSS_BLOCKS = 1024;
constexpr long HEAD_DW_PIX = 128;   // pixels per dW partial (C2/C3 shard: 300 blocks)

}  // namespace hkp

using namespace hkp;

extern "C" int64_t hkp_heat_loss_workspace(void) { return (int64_t)LOSS_BLOCKS * sizeof(double); }

extern "C" int hkp_heat_loss(int32_t n, int32_t k, int32_t H, int32_t W, int32_t loss_kind, const float* heat,
                             const double* target, const float* uv, float sigma, double* loss, float* dheat,
                             void* workspace, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && k > 0 && H > 0 && W > 0, "hkp_heat_loss: bad sizes");
    HKP_CHECK_ARG(heat && loss && workspace, "hkp_heat_loss: null tensor");
    HKP_CHECK_ARG(target || (uv && sigma > 0.f), "hkp_heat_loss: need a dense target or (uv, sigma)");
    HKP_CHECK_ARG(loss_kind == HKP_LOSS_BCE || loss_kind == HKP_LOSS_MSE, "hkp_heat_loss: bad loss kind");
    const long total = (long)n * k * H * W;
    const double inv_n = 1.0 / (double)total;
    const float den = (float)(2.0 * (double)sigma * (double)sigma);
    double* part = (double*)workspace;
    hipStream_t st = as_stream(stream);
#define HKP_LOSS(KD, DN)                                                                                          \
    hipLaunchKernelGGL((heat_loss_kernel<KD, DN>), dim3(LOSS_BLOCKS), dim3(256), 0, st, total, H, W, den, inv_n, \
                       heat, target, uv, dheat, part)
    if (loss_kind == HKP_LOSS_BCE) {
        if (target) HKP_LOSS(HKP_LOSS_BCE, true); else HKP_LOSS(HKP_LOSS_BCE, false);
    } else {
        if (target) HKP_LOSS(HKP_LOSS_MSE, true); else HKP_LOSS(HKP_LOSS_MSE, false);
    }
#undef HKP_LOSS
    HKP_LAUNCH_CHECK("hkp_heat_loss");
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, st, LOSS_BLOCKS, inv_n, part, loss);
    HKP_LAUNCH_CHECK("hkp_heat_loss(finalize)");
    return HKP_OK;
}

extern "C" int64_t hkp_head_bwd_workspace(int32_t n, int32_t k, int32_t w, int32_t H) {
    return (int64_t)n * k * H * w * (int64_t)sizeof(float);
}

extern "C" int hkp_head_bwd(int32_t n, int32_t k, int32_t h, int32_t w, int32_t H, int32_t W, const float* dheat,
                            const float* heat, float* dlow, void* workspace, int64_t ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && k > 0 && h > 0 && w > 0 && H >= h && W >= w, "hkp_head_bwd: bad sizes");
    HKP_CHECK_ARG(dheat && dlow && workspace, "hkp_head_bwd: null tensor");
    HKP_CHECK_ARG(ws_bytes >= hkp_head_bwd_workspace(n, k, w, H), "hkp_head_bwd: workspace too small");
    const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
    const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
    const float ih = h > 1 ? (float)(H - 1) / (float)(h - 1) : 0.f;
    const float iw = w > 1 ? (float)(W - 1) / (float)(w - 1) : 0.f;
    float* rs = (float*)workspace;
    hipStream_t st = as_stream(stream);
    const long rows = (long)n * k * H * w;
    if (heat)
        hipLaunchKernelGGL((head_bwd_rows_kernel<true>), dim3(gcap(rows)), dim3(256), 0, st, n * k, w, H, W, sw, iw,
                           dheat, heat, rs);
    else
        hipLaunchKernelGGL((head_bwd_rows_kernel<false>), dim3(gcap(rows)), dim3(256), 0, st, n * k, w, H, W, sw, iw,
                           dheat, heat, rs);
    HKP_LAUNCH_CHECK("hkp_head_bwd(rows)");
    const long total = (long)n * k * h * w;
    hipLaunchKernelGGL(head_bwd_cols_kernel, dim3(gcap(total)), dim3(256), 0, st, n * k, h, w, H, sh, ih, rs, dlow);
    HKP_LAUNCH_CHECK("hkp_head_bwd(cols)");
    return HKP_OK;
}

extern "C" int64_t hkp_head_fc_bwd_workspace(int32_t n, int32_t hw, int32_t c, int32_t k) {
    const long npix = (long)n * hw;
    const long splits = (npix + HEAD_DW_PIX - 1) / HEAD_DW_PIX;
    return (int64_t)splits * k * (c + 1) * (int64_t)sizeof(float);
}

extern "C" int hkp_head_fc_bwd(int32_t n, int32_t hw, int32_t c, int32_t k, const float* dlow, const float* feat,
                               const float* w, float* dfeat, float* dw, float* db, void* workspace, int64_t ws_bytes,
                               hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && hw > 0 && c > 0 && c % 4 == 0 && k > 0 && k <= 16, "hkp_head_fc_bwd: bad sizes");
    HKP_CHECK_ARG(dlow && feat && w && dfeat && dw && db && workspace, "hkp_head_fc_bwd: null tensor");
    HKP_CHECK_ARG(ws_bytes >= hkp_head_fc_bwd_workspace(n, hw, c, k), "hkp_head_fc_bwd: workspace too small");
    const long npix = (long)n * hw;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(head_dfeat_kernel, dim3(gcap(npix * (c / 4))), dim3(256), 0, st, npix, hw, c, k, dlow, w,
                       dfeat);
    HKP_LAUNCH_CHECK("hkp_head_fc_bwd(dfeat)");
    const long splits = (npix + HEAD_DW_PIX - 1) / HEAD_DW_PIX;
    float* ws_w = (float*)workspace;
    float* ws_b = ws_w + splits * k * c;
    const int C4 = c / 4;
    dim3 grid((unsigned)splits, (unsigned)((C4 + 255) / 256));
    if (k <= 4)
        hipLaunchKernelGGL(head_dw_kernel<4>, grid, dim3(256), 0, st, npix, hw, c, k, HEAD_DW_PIX, dlow, feat, ws_w,
                           ws_b);
    else if (k <= 8)
        hipLaunchKernelGGL(head_dw_kernel<8>, grid, dim3(256), 0, st, npix, hw, c, k, HEAD_DW_PIX, dlow, feat, ws_w,
                           ws_b);
    else
        hipLaunchKernelGGL(head_dw_kernel<16>, grid, dim3(256), 0, st, npix, hw, c, k, HEAD_DW_PIX, dlow, feat, ws_w,
                           ws_b);
    HKP_LAUNCH_CHECK("hkp_head_fc_bwd(dw)");
    hipLaunchKernelGGL(sum_splits_kernel, dim3((unsigned)(((long)k * c + 63) / 64)), dim3(256), 0, st, (long)k * c,
                       (int)splits, ws_w, dw);
    hipLaunchKernelGGL(sum_splits_kernel, dim3((unsigned)((k + 63) / 64)), dim3(256), 0, st, (long)k, (int)splits,
                       ws_b, db);
    HKP_LAUNCH_CHECK("hkp_head_fc_bwd(reduce)");
    return HKP_OK;
}
