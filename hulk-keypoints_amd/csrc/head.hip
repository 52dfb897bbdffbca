// Heatmap head: K-channel 1x1 scoring conv, bilinear (align_corners=True)
// upsample + sigmoid + argmax decode, and the Gaussian target.
//
//  * hkp_head_fc          src/resnet_dilated.py:16 (fc 1x1 + bias), only the K
//                         rows src/model.py:21 keeps (per-channel ops,
//                         so dropping rows >= K changes no kept value).
//  * hkp_upsample_sigmoid src/resnet_dilated.py:27 + src/model.py:21 + the
//                         argmax of src/prediction.py:46.  The interpolation
//                         reproduces ATen's CPU arithmetic bit for bit:
//                         t(h) = fma(x[h][w0], lw0, x[h][w1]*lw1),
//                         out  = fma(t(h0), lh0, t(h1)*lh1), weights in fp32
//                         (verified against torch 2.10 CPU on 4 shapes).
//  * hkp_gauss_target     src/dataset.py:36-44.
#include "common.h"

// Exact-arithmetic file: no implicit a*b+c → fma contraction (hipcc's default
// -ffp-contract=fast would fuse e.g. scale*o - i0 and break bit parity with
// ATen).  Every fused multiply-add below is an explicit __builtin_fmaf.
#pragma clang fp contract(off)

namespace hkp {

// one wave per pixel; W (K x C) and bias staged in LDS
template <int KMAX>
__global__ __launch_bounds__(256) void head_fc_kernel(int npix, int hw, int C, int K, const float* __restrict__ feat,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float wl[];  // [K][C]
    for (int i = threadIdx.x; i < K * C; i += blockDim.x) wl[i] = w[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int waves = blockDim.x >> 6;
    for (int p = blockIdx.x * waves + wid; p < npix; p += gridDim.x * waves) {
        float acc[KMAX];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) acc[k] = 0.f;
        const float* f = feat + (long)p * C;
        for (int c = lane * 4; c < C; c += 256) {
            const f32x4 v = *(const f32x4*)(f + c);
#pragma unroll
            for (int k = 0; k < KMAX; ++k) {
                if (k < K) {
                    const f32x4 ww = *(const f32x4*)(wl + k * C + c);
                    acc[k] += v[0] * ww[0] + v[1] * ww[1] + v[2] * ww[2] + v[3] * ww[3];
                }
            }
        }
        const int n = p / hw, q = p - n * hw;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (k < K) {
                const float s = wave_sum(acc[k]);
                if (lane == k) out[((long)n * K + k) * hw + q] = s + bias[k];
            }
        }
    }
}

struct Lerp {
    int i0, i1;
    float l0, l1;
};

// ATen compute_indices_weights_linear, align_corners=True, fp32 opmath
__device__ __forceinline__ Lerp lerp_index(int o, int in, int out, float scale) {
    Lerp r;
    if (in == out) {
        r.i0 = r.i1 = o;
        r.l0 = 1.f;
        r.l1 = 0.f;
        return r;
    }
    const float src = __fmul_rn(scale, (float)o);
    int i0 = (int)floorf(src);
    i0 = i0 < in - 1 ? i0 : in - 1;
    float l1 = __fsub_rn(src, (float)i0);
    l1 = fminf(fmaxf(l1, 0.f), 1.f);
    r.i0 = i0;
    r.i1 = i0 + (i0 < in - 1 ? 1 : 0);
    r.l1 = l1;
    r.l0 = __fsub_rn(1.f, l1);
    return r;
}

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) {
    return a > b ? a : b;
}

__device__ __forceinline__ float bilerp(const float* r0, const float* r1, const Lerp& lh, const Lerp& lw) {
    // ATen CPU order: t(h) = fma(x[h][w0], lw0, x[h][w1]*lw1); out = fma(t(h0), lh0, t(h1)*lh1)
    const float t0 = __builtin_fmaf(r0[lw.i0], lw.l0, r0[lw.i1] * lw.l1);
    const float t1 = __builtin_fmaf(r1[lw.i0], lw.l0, r1[lw.i1] * lw.l1);
    return __builtin_fmaf(t0, lh.l0, t1 * lh.l1);
}

__device__ __forceinline__ unsigned long long argmax_key(float p, unsigned idx) {
    // values are sigmoid outputs (>= 0, or NaN): their bit patterns order like the values,
    // and NaN sorts highest (numpy's argmax also returns the first NaN)
    return ((unsigned long long)__float_as_uint(p) << 32) | (unsigned long long)(0xFFFFFFFFu - idx);
}

// grid: x over ceil(H*W/1024) chunks of 4 outputs per thread, y over n*k planes.
// ROW4: W % 4 == 0, so a thread's 4 outputs share one output row.
template <bool SIGMOID, bool ROW4>
__global__ __launch_bounds__(256) void upsample_sigmoid_kernel(int h, int w, int H, int W, float sh, float sw,
                                                              const float* __restrict__ low, float* __restrict__ heat,
                                                              unsigned long long* __restrict__ keys) {
    const int plane = blockIdx.y;
    const unsigned HW = (unsigned)H * (unsigned)W;
    const float* x = low + (size_t)plane * h * w;
    const unsigned base = (blockIdx.x * 256u + threadIdx.x) * 4u;
    unsigned long long best = 0ull;
    if (base < HW) {
        float v[4];
        if constexpr (ROW4) {
            const unsigned oh = base / (unsigned)W, ow0 = base - oh * (unsigned)W;
            const Lerp lh = lerp_index((int)oh, h, H, sh);
            const float* r0 = x + lh.i0 * w;
            const float* r1 = x + lh.i1 * w;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const Lerp lw = lerp_index((int)ow0 + e, w, W, sw);
                const float z = bilerp(r0, r1, lh, lw);
                v[e] = SIGMOID ? sigmoid_f(z) : z;
                best = umax64(best, argmax_key(v[e], base + e));
            }
            if (heat) *(f32x4*)(heat + (size_t)plane * HW + base) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const unsigned o = base + e;
                if (o < HW) {
                    const unsigned oh = o / (unsigned)W, ow = o - oh * (unsigned)W;
                    const Lerp lh = lerp_index((int)oh, h, H, sh), lw = lerp_index((int)ow, w, W, sw);
                    const float z = bilerp(x + lh.i0 * w, x + lh.i1 * w, lh, lw);
                    v[e] = SIGMOID ? sigmoid_f(z) : z;
                    best = umax64(best, argmax_key(v[e], o));
                    if (heat) heat[(size_t)plane * HW + o] = v[e];
                }
            }
        }
    }
    if (keys) {
        unsigned lo = (unsigned)best, hi = (unsigned)(best >> 32);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned ol = __shfl_xor(lo, off), oh = __shfl_xor(hi, off);
            const unsigned long long m =
                umax64(((unsigned long long)hi << 32) | lo, ((unsigned long long)oh << 32) | ol);
            lo = (unsigned)m;
            hi = (unsigned)(m >> 32);
        }
        // block max in fixed order, one key per block (no atomics: same-address
        // device atomics from every wave serialised this kernel)
        __shared__ unsigned long long wkey[4];
        if ((threadIdx.x & 63) == 0) wkey[threadIdx.x >> 6] = ((unsigned long long)hi << 32) | lo;
        __syncthreads();
        if (threadIdx.x == 0)
            keys[(size_t)plane * gridDim.x + blockIdx.x] = umax64(umax64(wkey[0], wkey[1]), umax64(wkey[2], wkey[3]));
    }
}

// one block per (n,k) plane: max over the plane's per-block keys, decode (y, x)
__global__ __launch_bounds__(256) void argmax_decode_kernel(int nblk, int W, const unsigned long long* __restrict__ keys,
                                                           int* __restrict__ yx) {
    const int plane = blockIdx.x;
    unsigned long long best = 0ull;
    for (int b = threadIdx.x; b < nblk; b += 256) best = umax64(best, keys[(size_t)plane * nblk + b]);
    unsigned lo = (unsigned)best, hi = (unsigned)(best >> 32);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned ol = __shfl_xor(lo, off), oh = __shfl_xor(hi, off);
        const unsigned long long m = umax64(((unsigned long long)hi << 32) | lo, ((unsigned long long)oh << 32) | ol);
        lo = (unsigned)m;
        hi = (unsigned)(m >> 32);
    }
    __shared__ unsigned long long wkey[4];
    if ((threadIdx.x & 63) == 0) wkey[threadIdx.x >> 6] = ((unsigned long long)hi << 32) | lo;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long k = umax64(umax64(wkey[0], wkey[1]), umax64(wkey[2], wkey[3]));
        const unsigned idx = 0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull);
        yx[2 * plane] = (int)(idx / (unsigned)W);
        yx[2 * plane + 1] = (int)(idx % (unsigned)W);
    }
}

__global__ __launch_bounds__(256) void gauss_target_kernel(int K, int H, int W, float den,
                                                          const float* __restrict__ uv, double* __restrict__ out,
                                                          long total) {
    const long stride = (long)gridDim.x * blockDim.x;
    const long HW = (long)H * W;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const long plane = i / HW;
        const long r = i - plane * HW;
        const int y = (int)(r / W), x = (int)(r - (long)y * W);
        const float u = uv[plane * 2], v = uv[plane * 2 + 1];
        const float dx = __fsub_rn((float)x, u), dy = __fsub_rn((float)y, v);
        const float t = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
        out[i] = (double)expf(__fdiv_rn(-t, den));
    }
}

}  // namespace hkp

using namespace hkp;

extern "C" int hkp_head_fc(int32_t n, int32_t hw, int32_t c, int32_t k, const float* feat, const float* w,
                           const float* bias, float* lowres, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && hw > 0 && c > 0 && k > 0, "hkp_head_fc: bad sizes");
    HKP_CHECK_ARG(k <= 16, "hkp_head_fc: at most 16 keypoints (got %d)", k);
    HKP_CHECK_ARG(c % 4 == 0 && (long)k * c <= 16384, "hkp_head_fc: need c%%4==0 and k*c<=16384");
    HKP_CHECK_ARG(feat && w && bias && lowres, "hkp_head_fc: null tensor");
    const int npix = n * hw;
    int grid = (npix + 3) / 4;
    if (grid > 2048) grid = 2048;
    const size_t lds = (size_t)k * c * sizeof(float);
    hipStream_t st = as_stream(stream);
    if (k <= 4)
        hipLaunchKernelGGL(head_fc_kernel<4>, dim3(grid), dim3(256), lds, st, npix, hw, c, k, feat, w, bias, lowres);
    else if (k <= 8)
        hipLaunchKernelGGL(head_fc_kernel<8>, dim3(grid), dim3(256), lds, st, npix, hw, c, k, feat, w, bias, lowres);
    else
        hipLaunchKernelGGL(head_fc_kernel<16>, dim3(grid), dim3(256), lds, st, npix, hw, c, k, feat, w, bias, lowres);
    HKP_LAUNCH_CHECK("hkp_head_fc");
    return HKP_OK;
}

extern "C" int hkp_upsample_sigmoid(int32_t n, int32_t k, int32_t h, int32_t w, int32_t H, int32_t W,
                                    int32_t apply_sigmoid, const float* lowres, float* heat, uint64_t* argmax_ws, int32_t* argmax_yx,
                                    hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && k > 0 && h > 0 && w > 0 && H > 0 && W > 0, "hkp_upsample_sigmoid: bad sizes");
    HKP_CHECK_ARG(lowres != nullptr, "hkp_upsample_sigmoid: null lowres");
    HKP_CHECK_ARG(argmax_yx == nullptr || argmax_ws != nullptr, "hkp_upsample_sigmoid: argmax needs workspace");
    HKP_CHECK_ARG(argmax_yx == nullptr || apply_sigmoid, "hkp_upsample_sigmoid: argmax keys need sigmoid outputs");
    HKP_CHECK_ARG((long)H * W < 0x7FFFFFFFL && (long)h * w < 0x7FFFFFFFL, "hkp_upsample_sigmoid: plane too large");
    hipStream_t st = as_stream(stream);
    const int nk = n * k;
    unsigned long long* keys = argmax_yx ? (unsigned long long*)argmax_ws : nullptr;
    // area_pixel_compute_scale (align_corners): (in-1)/(out-1) in fp32
    const float sh = H > 1 ? (float)(h - 1) / (float)(H - 1) : 0.f;
    const float sw = W > 1 ? (float)(w - 1) / (float)(W - 1) : 0.f;
    const long HW = (long)H * W;
    dim3 grid((unsigned)((HW + 1023) / 1024), (unsigned)nk);
    const bool row4 = (W & 3) == 0;
#define HKP_UPS(SG, R4) \
    hipLaunchKernelGGL((upsample_sigmoid_kernel<SG, R4>), grid, dim3(256), 0, st, h, w, H, W, sh, sw, lowres, heat, keys)
    if (apply_sigmoid) {
        if (row4) HKP_UPS(true, true); else HKP_UPS(true, false);
    } else {
        if (row4) HKP_UPS(false, true); else HKP_UPS(false, false);
    }
#undef HKP_UPS
    HKP_LAUNCH_CHECK("hkp_upsample_sigmoid");
    if (keys) {
        hipLaunchKernelGGL(argmax_decode_kernel, dim3(nk), dim3(256), 0, st, (int)grid.x, W, keys, argmax_yx);
        HKP_LAUNCH_CHECK("hkp_upsample_sigmoid(decode)");
    }
    return HKP_OK;
}

extern "C" int hkp_gauss_target(int32_t n, int32_t k, int32_t H, int32_t W, float sigma, const float* uv,
                                double* out, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && k > 0 && H > 0 && W > 0 && sigma > 0.f, "hkp_gauss_target: bad sizes");
    HKP_CHECK_ARG(uv && out, "hkp_gauss_target: null tensor");
    const long total = (long)n * k * H * W;
    long g = (total + 255) / 256;
    if (g > 4096) g = 4096;
    // 2.0*sigma**2 as the reference computes it (python float → fp32 divisor)
    const float den = (float)(2.0 * (double)sigma * (double)sigma);
    hipLaunchKernelGGL(gauss_target_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), k, H, W, den, uv, out,
                       total);
    HKP_LAUNCH_CHECK("hkp_gauss_target");
    return HKP_OK;
}

extern "C" int64_t hkp_upsample_argmax_ws_bytes(int32_t n, int32_t k, int32_t H, int32_t W) {
    if (n <= 0 || k <= 0 || H <= 0 || W <= 0) return -1;
    return (int64_t)n * k * (((int64_t)H * W + 1023) / 1024) * (int64_t)sizeof(uint64_t);
}
