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

// Sum of v[0..KP) over the 64 lanes of a wave, reduce-scatter form: at offset
// 32, 16, ... each lane keeps half of its values (plus its partner's copy of
// that half) until one is left, then the remaining offsets fold it whole —
// KP-1 + log2(64/KP) shuffles instead of 6 per value.  Lane l ends with the
// sum for k = ksel(l); the fold order is fixed (deterministic).
template <int KP>
__device__ __forceinline__ float wave_reduce_scatter(float (&v)[KP], int lane) {
    int o = 32;
#pragma unroll
    for (int n = KP; n > 1; n >>= 1, o >>= 1) {
        const int half = n >> 1;
        const bool upper = (lane & o) != 0;
#pragma unroll
        for (int i = 0; i < half; ++i) {
            const float send = upper ? v[i] : v[half + i];
            const float keep = upper ? v[half + i] : v[i];
            v[i] = keep + __shfl_xor(send, o);
        }
    }
    float s = v[0];
    for (; o > 0; o >>= 1) s += __shfl_xor(s, o);
    return s;
}

// the k whose total lane l holds after wave_reduce_scatter<KP>
template <int KP>
__device__ __forceinline__ int wave_reduce_scatter_k(int lane) {
    int k = 0, o = 32;
#pragma unroll
    for (int n = KP; n > 1; n >>= 1, o >>= 1) k += (lane & o) ? (n >> 1) : 0;
    return k;
}

// Inference tail: the last block's BN apply (+ residual, ReLU; the arithmetic of
// hkp_bn_apply / hkp_bn_apply_f16 exactly) fused with the K-row head, so the
// backbone's final activation (the only fp32 feature map of the forward: 315 MB
// at C2, 5 GB at C4) is never written nor read back.  A lane owns 8 channels,
// a wave 512, G = C/512 waves one pixel; each wave group runs PB pixels per
// iteration (their loads in flight together), folds each pixel's K partial dots
// with wave_reduce_scatter, and the G waves' totals are summed in wave order
// through LDS.  YH: y (and a raw residual) fp16 (config C4) instead of fp32.
// RES: 0 none, 1 raw residual, 2 residual*rscale + rshift, 3 packed split (hi+lo)
// raw residual (fp32 path).
constexpr int HEAD_PB = 4;
template <bool YH, int RES, int KP>
__global__ __launch_bounds__(256) void bn_apply_head_kernel(long M, int hw, int C, int K, const void* __restrict__ yv,
                                                            const float* __restrict__ ss, const void* __restrict__ resv,
                                                            const float* __restrict__ rss, const float* __restrict__ w,
                                                            const float* __restrict__ bias, float* __restrict__ low) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    __shared__ float red[4][HEAD_PB][KP];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int G = C >> 9, GPB = 4 / G;                       // waves per pixel, pixel groups per block
    const int c0 = (wv % G) * 512 + lane * 8;
    float sc[8], sh[8], rsc[8], rsh[8], wk[KP][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sc[e] = ss[c0 + e];
        sh[e] = ss[C + c0 + e];
        rsc[e] = RES == 2 ? rss[c0 + e] : 0.f;
        rsh[e] = RES == 2 ? rss[C + c0 + e] : 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) wk[k][e] = k < K ? w[(long)k * C + c0 + e] : 0.f;
    }
    const long chunks = (M + HEAD_PB - 1) / HEAD_PB;
    const int ks = wave_reduce_scatter_k<KP>(lane);
    constexpr int LOW_LANES = 64 / KP;                       // lanes holding the same k after the fold
    for (long ch0 = (long)blockIdx.x * GPB; ch0 < chunks; ch0 += (long)gridDim.x * GPB) {
        const long ch = ch0 + wv / G;
        float v[HEAD_PB][8], r[HEAD_PB][8];
#pragma unroll
        for (int u = 0; u < HEAD_PB; ++u) {
            const long p = ch * HEAD_PB + u;
            const bool ok = ch < chunks && p < M;
            const long e0 = (ok ? p : 0) * C + c0;
            if constexpr (YH) {
                const h8 t = ok ? *(const h8*)((const _Float16*)yv + e0) : h8{};
#pragma unroll
                for (int e = 0; e < 8; ++e) v[u][e] = (float)t[e];
            } else {
                const f32x4 a = ok ? *(const f32x4*)((const float*)yv + e0) : f32x4{};
                const f32x4 b = ok ? *(const f32x4*)((const float*)yv + e0 + 4) : f32x4{};
#pragma unroll
                for (int e = 0; e < 4; ++e) { v[u][e] = a[e]; v[u][4 + e] = b[e]; }
            }
            if constexpr (RES == 3) {
                const long off = 2 * e0 - (e0 & 31);
                const h8 h = ok ? *(const h8*)((const _Float16*)resv + off) : h8{};
                const h8 l = ok ? *(const h8*)((const _Float16*)resv + off + 32) : h8{};
#pragma unroll
                for (int e = 0; e < 8; ++e) r[u][e] = __fadd_rn((float)h[e], (float)l[e]);
            } else if constexpr (RES != 0 && YH) {
                const h8 t = ok ? *(const h8*)((const _Float16*)resv + e0) : h8{};
#pragma unroll
                for (int e = 0; e < 8; ++e) r[u][e] = (float)t[e];
            } else if constexpr (RES != 0) {
                const f32x4 a = ok ? *(const f32x4*)((const float*)resv + e0) : f32x4{};
                const f32x4 b = ok ? *(const f32x4*)((const float*)resv + e0 + 4) : f32x4{};
#pragma unroll
                for (int e = 0; e < 4; ++e) { r[u][e] = a[e]; r[u][4 + e] = b[e]; }
            }
        }
#pragma unroll
        for (int u = 0; u < HEAD_PB; ++u) {
            float part[KP];
#pragma unroll
            for (int k = 0; k < KP; ++k) part[k] = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float o = __fadd_rn(__fmul_rn(v[u][e], sc[e]), sh[e]);
                if constexpr (RES == 1 || RES == 3) o = __fadd_rn(o, r[u][e]);
                else if constexpr (RES == 2) o = __fadd_rn(o, __fadd_rn(__fmul_rn(r[u][e], rsc[e]), rsh[e]));
                o = o > 0.f ? o : 0.f;
#pragma unroll
                for (int k = 0; k < KP; ++k) part[k] = __fadd_rn(part[k], __fmul_rn(o, wk[k][e]));
            }
            const float s = wave_reduce_scatter<KP>(part, lane);
            if (lane % LOW_LANES == 0) red[wv][u][ks] = s;
        }
        __syncthreads();
        for (int t = threadIdx.x; t < GPB * HEAD_PB * K; t += 256) {
            const int g = t / (HEAD_PB * K), rem = t - g * HEAD_PB * K, u = rem / K, k = rem - u * K;
            const long p = (ch0 + g) * HEAD_PB + u;
            if (ch0 + g < chunks && p < M) {
                float s = red[g * G][u][k];
                for (int i = 1; i < G; ++i) s = __fadd_rn(s, red[g * G + i][u][k]);
                const long n = p / hw, q = p - n * hw;
                low[(n * K + k) * hw + q] = __fadd_rn(s, bias[k]);
            }
        }
        __syncthreads();
    }
}

// Config C4's inference tail (y fp16): the same fp32 BN apply (+ residual, ReLU)
// as bn_apply_head_kernel<true, …>, then the activation rounded to fp16 (the
// dtype autocast gives the ReLU output) and the K-row head as
// v_mfma_f32_16x16x32_f16 against the fp16-rounded head rows (autocast's 1x1
// conv; fp32 accumulation).  The VALU form spent 16 of its ~22 lane operations
// per channel on the K dot products and held ~180 VGPRs (two waves per SIMD):
// at C = 2048 it read its 5 GB at 3.1 TB/s.  Here a wave scores 16 pixels: lane
// l feeds pixel l & 15, channels 8 (l >> 4) .. +7 of each 32-channel step (A),
// and head row l & 15 of the same channels (B, from LDS; zero rows k >= K); its
// accumulator ends holding pixels 4 (l >> 4) + 0..3 of row l & 15.  The scale /
// shift (and residual scale / shift) sit in LDS, broadcast to the 16 lanes of a
// channel group; y and the residual are read once, non-temporally, 128 channels
// (8 x 16 B per lane) in flight per wave; waves stride over 16-pixel groups.
constexpr int HM_WAVES = 8;
template <int RES, int KP>
__global__ __launch_bounds__(64 * HM_WAVES, 2) void head_f16_mfma_kernel(long M, int hw, int C, int K,
                                                                        const _Float16* __restrict__ y,
                                                                        const float* __restrict__ ss,
                                                                        const _Float16* __restrict__ res,
                                                                        const float* __restrict__ rss,
                                                                        const float* __restrict__ w,
                                                                        const float* __restrict__ bias,
                                                                        float* __restrict__ low) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) char hsm[];
    constexpr int NSS = RES == 2 ? 4 : 2;
    float* const cst = (float*)hsm;                       // [NSS][C]: scale, shift (, rscale, rshift)
    h8* const wl = (h8*)(hsm + (long)NSS * C * 4);        // [C/8][KP]: channels 8q..8q+7 of head row k
    const int tid = threadIdx.x;
    for (int i = tid; i < C; i += 64 * HM_WAVES) {
        cst[i] = ss[i];
        cst[C + i] = ss[C + i];
        if constexpr (RES == 2) {
            cst[2 * C + i] = rss[i];
            cst[3 * C + i] = rss[C + i];
        }
    }
    for (int i = tid; i < (C / 8) * KP; i += 64 * HM_WAVES) {
        const int q = i / KP, k = i - q * KP;
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = k < K ? (_Float16)w[(long)k * C + 8 * q + e] : (_Float16)0.f;
        wl[i] = v;
    }
    __syncthreads();
    const int lane = tid & 63, wv = tid >> 6;
    const int r16 = lane & 15, g = lane >> 4;
    const h8 zero8 = {};
    const long groups = (M + 15) / 16;
    for (long grp = (long)blockIdx.x * HM_WAVES + wv; grp < groups; grp += (long)gridDim.x * HM_WAVES) {
        const long p = grp * 16 + r16;
        const bool ok = p < M;
        const long e0 = (ok ? p : 0) * C + 8 * g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int c0 = 0; c0 < C; c0 += 128) {
            h8 yv[4], rv[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                yv[t] = ok ? __builtin_nontemporal_load((const h8*)(y + e0 + c0 + 32 * t)) : zero8;
                if constexpr (RES != 0) rv[t] = ok ? __builtin_nontemporal_load((const h8*)(res + e0 + c0 + 32 * t)) : zero8;
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int cb = c0 + 32 * t + 8 * g;
                h8 o16;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float o = __fadd_rn(__fmul_rn((float)yv[t][e], cst[cb + e]), cst[C + cb + e]);
                    if constexpr (RES == 1) o = __fadd_rn(o, (float)rv[t][e]);
                    else if constexpr (RES == 2)
                        o = __fadd_rn(o, __fadd_rn(__fmul_rn((float)rv[t][e], cst[2 * C + cb + e]), cst[3 * C + cb + e]));
                    o16[e] = (_Float16)(o > 0.f ? o : 0.f);
                }
                const h8 wb = r16 < KP ? wl[(cb >> 3) * KP + r16] : zero8;
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(o16, wb, acc, 0, 0, 0);
            }
        }
        if (r16 < K) {
            const float b = bias[r16];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const long pp = grp * 16 + 4 * g + i;
                if (pp < M) {
                    const long n = pp / hw, q = pp - n * hw;
                    low[(n * K + r16) * hw + q] = __fadd_rn(acc[i], b);
                }
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

// grid: x over ceil(H*W/(1024 UPS_G)) chunks — UPS_G sub-chunks of 1024 outputs, 4
// consecutive outputs per thread in each — y over n*k planes.  (One 1024-output
// chunk per block, 38,400 blocks of ~4 KB of stores each at C2: 70.5 -> 62 us with 4;
// the kernel is VALU-bound — lerp indices, IEEE expf and division per output — and
// loading a thread's 3 source columns once for its 4 outputs measured slower,
// 62 -> 80 us, on its select chains; profiles/r05_ups_*.)
// ROW4: W % 4 == 0, so a thread's 4 outputs share one output row.
constexpr int UPS_G = 4;
template <bool SIGMOID, bool ROW4>
__global__ __launch_bounds__(256) void upsample_sigmoid_kernel(int h, int w, int H, int W, float sh, float sw,
                                                              const float* __restrict__ low, float* __restrict__ heat,
                                                              unsigned long long* __restrict__ keys) {
    const int plane = blockIdx.y;
    const unsigned HW = (unsigned)H * (unsigned)W;
    const float* x = low + (size_t)plane * h * w;
    unsigned long long best = 0ull;
#pragma unroll
    for (int g = 0; g < UPS_G; ++g) {
    const unsigned base = ((blockIdx.x * UPS_G + g) * 256u + threadIdx.x) * 4u;
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

extern "C" int hkp_bn_apply_head(int32_t n, int32_t hw, int32_t c, int32_t k, int32_t y_f16, const void* y,
                                 const float* scale_shift, const void* res, const float* res_scale_shift,
                                 int32_t res_kind, const float* w, const float* bias, float* lowres,
                                 hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && hw > 0 && k > 0 && k <= 16, "hkp_bn_apply_head: bad sizes (n=%d hw=%d k=%d)", n, hw, k);
    HKP_CHECK_ARG(c > 0 && c % 512 == 0 && c <= 2048, "hkp_bn_apply_head: need c %% 512 == 0 and c <= 2048 (c=%d)", c);
    HKP_CHECK_ARG(y && scale_shift && w && bias && lowres, "hkp_bn_apply_head: null tensor");
    HKP_CHECK_ARG(res_kind >= 0 && res_kind <= 3 && (res_kind == 0) == (res == nullptr) &&
                      (res_kind == 2) == (res_scale_shift != nullptr) && !(res_kind == 3 && y_f16),
                  "hkp_bn_apply_head: bad residual (kind %d)", res_kind);
    const long M = (long)n * hw;
    if (y_f16 && k <= 8) {                 // config C4: the MFMA head (LDS <= 64 KiB at c = 2048)
        static const int cus = [] {
            int dev = 0, v = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
                v = 256;
            return v;
        }();
        const long groups = (M + 15) / 16;
        long gb = (groups + HM_WAVES - 1) / HM_WAVES;
        if (gb > 2L * cus) gb = 2L * cus;
        const size_t lds = (size_t)(res_kind == 2 ? 4 : 2) * c * 4 + (size_t)(c / 8) * 8 * 16;
        hipStream_t hst = as_stream(stream);
#define HKP_HM(RES)                                                                                               \
    hipLaunchKernelGGL((head_f16_mfma_kernel<RES, 8>), dim3((unsigned)gb), dim3(64 * HM_WAVES), lds, hst, M, hw, c, k, \
                       (const _Float16*)y, scale_shift, (const _Float16*)res, res_scale_shift, w, bias, lowres)
        if (res_kind == 0) HKP_HM(0);
        else if (res_kind == 1) HKP_HM(1);
        else HKP_HM(2);
#undef HKP_HM
        HKP_LAUNCH_CHECK("hkp_bn_apply_head(f16)");
        return HKP_OK;
    }
    const int gpb = 4 / (c / 512);
    long chunks = (M + HEAD_PB - 1) / HEAD_PB;
    long g = (chunks + gpb - 1) / gpb;
    if (g > 256L * 8) g = 256L * 8;
    hipStream_t st = as_stream(stream);
#define HKP_AH(YH, RES, KP)                                                                                       \
    hipLaunchKernelGGL((bn_apply_head_kernel<YH, RES, KP>), dim3((unsigned)g), dim3(256), 0, st, M, hw, c, k, y, \
                       scale_shift, res, res_scale_shift, w, bias, lowres)
#define HKP_AH_K(YH, RES) \
    if (k <= 4) HKP_AH(YH, RES, 4); else if (k <= 8) HKP_AH(YH, RES, 8); else HKP_AH(YH, RES, 16)
    if (y_f16) {
        if (res_kind == 0) HKP_AH_K(true, 0); else if (res_kind == 1) HKP_AH_K(true, 1); else HKP_AH_K(true, 2);
    } else {
        if (res_kind == 0) HKP_AH_K(false, 0);
        else if (res_kind == 1) HKP_AH_K(false, 1);
        else if (res_kind == 2) HKP_AH_K(false, 2);
        else HKP_AH_K(false, 3);
    }
#undef HKP_AH_K
#undef HKP_AH
    HKP_LAUNCH_CHECK("hkp_bn_apply_head");
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
    dim3 grid((unsigned)((HW + 1024 * UPS_G - 1) / (1024 * UPS_G)), (unsigned)nk);
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
