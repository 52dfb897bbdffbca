// BatchNorm backward (train mode) and the stem maxpool backward.
//
// For a BN layer z = y*alpha + beta (alpha = gamma*invstd) followed by ReLU
// (src/resnet.py:57-58,64-67,97-110), given g = dL/d(relu out):
//   dz        = g * (out > 0)                       (threshold_backward)
//   dbeta     = sum dz,   dgamma = invstd * sum dz*(y - mean)
//   dy        = (dz - sum(dz)/N - (y - mean) * k) * invstd*gamma,
//               k = invstd^2 * sum dz*(y - mean) / N     (ATen batch_norm_backward)
// Sums run per pixel tile in fp32, merged per channel in fp64 in fixed order.
#include <algorithm>

#include "common.h"

// the maxpool backward must recompute relu(y*a+b) exactly as bn.hip's forward
// did (two roundings) so its window argmax agrees: no fma contraction here.
#pragma clang fp contract(off)

namespace hkp {

constexpr int BNB_TILE = 64;   // pixels per reduction tile (small: enough blocks to fill the chip at batch 8)

// G = channel groups of 4 per thread (C/4 / threads-per-row); MASK: dz = g*(out>0)
// MAXIMA: also per tile and channel max|dz| and max|y - mean| (the inputs of
// finalize's upper bound on max|dy|)
// MASK 2: the ReLU mask recomputed from y as the forward's bn_apply did,
// round(round(y*scale) + shift) > 0 (out = the forward's [scale | shift]), so an
// inner BN's fp32 activation is not read back (bit-identical mask)
template <int G, int MASK, bool MAXIMA = false>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(long M, int C, const float* __restrict__ g,
                                                           const float* __restrict__ out, const float* __restrict__ y,
                                                           const float* __restrict__ mean, float* __restrict__ dz,
                                                           float* __restrict__ part, float* __restrict__ pmax,
                                                           unsigned* __restrict__ bound_reset) {
    __shared__ float red[2][256 * 4 * G];
    const int C4 = C >> 2;
    const int tpr = C4 / G;          // threads per row
    const int rpar = 256 / tpr;      // rows in flight per block
    const int tid = threadIdx.x;
    const int rl = tid / tpr, cg = tid - rl * tpr;
    const long m0 = (long)blockIdx.x * BNB_TILE;
    const long m1 = min(M, m0 + BNB_TILE);
    if (MAXIMA && bound_reset && blockIdx.x == 0 && tid == 0) *bound_reset = 0u;
    f32x4 s[G], q[G], mu[G], xd[G], xv[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        s[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        q[k] = s[k];
        xd[k] = s[k];
        xv[k] = s[k];
        mu[k] = *(const f32x4*)(mean + 4 * (cg + k * tpr));
    }
    f32x4 msc[G], msh[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        if constexpr (MASK == 2) {
            msc[k] = *(const f32x4*)(out + 4 * (cg + k * tpr));
            msh[k] = *(const f32x4*)(out + C + 4 * (cg + k * tpr));
        }
    }
    for (long m = m0 + rl; m < m1; m += rpar) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const long off = m * C + 4 * (cg + k * tpr);
            f32x4 d = *(const f32x4*)(g + off);
            const f32x4 v = *(const f32x4*)(y + off);
            if constexpr (MASK == 1) {
                const f32x4 o = *(const f32x4*)(out + off);
#pragma unroll
                for (int e = 0; e < 4; ++e) d[e] = o[e] > 0.f ? d[e] : 0.f;
            } else if constexpr (MASK == 2) {
#pragma unroll
                for (int e = 0; e < 4; ++e) d[e] = __fadd_rn(__fmul_rn(v[e], msc[k][e]), msh[k][e]) > 0.f ? d[e] : 0.f;
            }
            if (dz) *(f32x4*)(dz + off) = d;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                s[k][e] += d[e];
                q[k][e] += d[e] * (v[e] - mu[k][e]);
                if constexpr (MAXIMA) {
                    xd[k][e] = fmaxf(xd[k][e], fabsf(d[e]));
                    xv[k][e] = fmaxf(xv[k][e], fabsf(v[e] - mu[k][e]));
                }
            }
        }
    }
    // combine the rpar partial rows of each channel in fixed order
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int c = 4 * (cg + k * tpr) + e;
            red[0][rl * C + c] = s[k][e];
            red[1][rl * C + c] = q[k][e];
        }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        float a = 0.f, b = 0.f;
        for (int r = 0; r < rpar; ++r) {
            a += red[0][r * C + c];
            b += red[1][r * C + c];
        }
        part[((long)blockIdx.x * C + c) * 2] = a;
        part[((long)blockIdx.x * C + c) * 2 + 1] = b;
    }
    if constexpr (MAXIMA) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < G; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = 4 * (cg + k * tpr) + e;
                red[0][rl * C + c] = xd[k][e];
                red[1][rl * C + c] = xv[k][e];
            }
        __syncthreads();
        for (int c = tid; c < C; c += 256) {
            float a = 0.f, b = 0.f;
            for (int r = 0; r < rpar; ++r) {
                a = fmaxf(a, red[0][r * C + c]);
                b = fmaxf(b, red[1][r * C + c]);
            }
            pmax[((long)blockIdx.x * C + c) * 2] = a;
            pmax[((long)blockIdx.x * C + c) * 2 + 1] = b;
        }
    }
}

// per channel: dgamma, dbeta, and the apply coefficients (grad_mean, k, invstd*gamma)
// NB > 0 (tiles <= NB * TL): the lane's partials (and maxima) loaded in one round
// into registers — the same sums and maxima in the same order, so the same bits
template <int CPB, int NT = 256, int NB = 0>
__global__ __launch_bounds__(NT) void bn_bwd_finalize_kernel(int C, long M, long tiles, const float* __restrict__ part,
                                                             const float* __restrict__ mi, const float* gamma,
                                                             float* dgamma, float* dbeta, float* coef,
                                                             const float* __restrict__ pmax, unsigned* amax,
                                                             double* stats) {
    constexpr int TL = NT / CPB, NW = NT / 64;
    __shared__ double red[NW][8];
    __shared__ float bmax[8];
    const int cl = threadIdx.x % CPB, tl = threadIdx.x / CPB, c = blockIdx.x * CPB + cl;
    const bool ok = c < C;
    if (!pmax && amax && !stats && blockIdx.x == 0 && threadIdx.x == 0) *amax = 0u;   // apply's atomicMax starts from 0
    double s = 0.0, d = 0.0;
    double md = 0.0, mv = 0.0;
    if constexpr (NB > 0) {
        float2 v[NB], x[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const long t = tl + (long)j * TL;
            const bool in = ok && t < tiles;
            v[j] = in ? *(const float2*)(part + (t * C + c) * 2) : make_float2(0.f, 0.f);
            x[j] = in && pmax ? *(const float2*)(pmax + (t * C + c) * 2) : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            s += (double)v[j].x;
            d += (double)v[j].y;
            md = fmax(md, (double)x[j].x);       // maxima of non-negative values: 0 past the end is exact
            mv = fmax(mv, (double)x[j].y);
        }
    } else if (ok) {   // 8 loads in flight per batch (latency-bound loop); zero-filled past the end
        for (long t0 = tl; t0 < tiles; t0 += 8 * TL) {
            float2 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const long t = t0 + (long)j * TL;
                v[j] = t < tiles ? *(const float2*)(part + (t * C + c) * 2) : make_float2(0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                s += (double)v[j].x;
                d += (double)v[j].y;
            }
        }
        if (pmax)   // per-channel maxima over the tiles (max: any order is exact)
            for (long t = tl; t < tiles; t += TL) {
                const float2 v = *(const float2*)(pmax + (t * C + c) * 2);
                md = fmax(md, (double)v.x);
                mv = fmax(mv, (double)v.y);
            }
    }
    const double S = lanes_sum_d<CPB, NW>(s, red);
    const double D = lanes_sum_d<CPB, NW>(d, red);
    if (pmax) {
        md = lanes_max_d<CPB, NW>(md, red);
        mv = lanes_max_d<CPB, NW>(mv, red);
    }
    if (stats) {                 // SyncBN: this rank's sums for the cross-rank merge (bn_bwd_fin_ranks_kernel)
        if (tl == 0 && ok) {
            stats[c] = S;
            stats[C + c] = D;
            stats[2 * C + c] = md;
            stats[3 * C + c] = mv;
            if (c == 0) stats[4 * C] = (double)M;
        }
        return;
    }
    if (tl == 0 && ok) {
        const double inv = (double)mi[C + c];
        const float gm = gamma ? gamma[c] : 1.f;
        if (dgamma) dgamma[c] = (float)(D * inv);
        if (dbeta) dbeta[c] = (float)S;
        const float cg = (float)(S / (double)M), ck = (float)(D * inv * inv / (double)M), cs = (float)(inv * (double)gm);
        coef[c] = cg;                 // grad_mean
        coef[C + c] = ck;             // k
        coef[2 * C + c] = cs;         // invstd * gamma
        if (pmax)   // |dy| <= (max|dz| + |gm| + max|y-mean|*|k|) * |invstd*gamma|, with slack for fp32 rounding
            bmax[cl] = (float)((md + fabs((double)cg) + mv * fabs((double)ck)) * fabs((double)cs) * 1.0001);
    }
    if (pmax && amax) {
        __syncthreads();
        if (threadIdx.x == 0) {
            float b = 0.f;
            for (int i = 0; i < CPB && blockIdx.x * CPB + i < C; ++i) b = fmaxf(b, bmax[i]);
            atomicMax(amax, __float_as_uint(b));   // the word was zeroed by the reduce kernel
        }
    }
}

// SyncBN backward: the ranks' [S | D | max|dz| | max|y-mean| | M] blocks (st,
// [R][4C+1], rank order) summed in fixed rank order — the apply coefficients
// from the global sums and count (torch SyncBatchNorm's all-reduced sum_dy /
// sum_dy_xmu), dgamma / dbeta from this rank's own block (DDP then averages them
// with the other parameters' gradients), the split-scale bound from this rank's
// maxima with the global coefficients.  One rank: bn_bwd_finalize_kernel's bits.
__global__ __launch_bounds__(256) void bn_bwd_fin_ranks_kernel(int C, int R, const double* __restrict__ st,
                                                               const double* __restrict__ own, int has_max,
                                                               const float* __restrict__ mi, const float* gamma,
                                                               float* dgamma, float* dbeta, float* coef,
                                                               unsigned* amax) {
    __shared__ float bmax[256];
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    float b = 0.f;
    if (c < C) {
        const long L = 4L * C + 1;
        double S = 0.0, D = 0.0, M = 0.0;
        for (int r = 0; r < R; ++r) {
            S += st[r * L + c];
            D += st[r * L + C + c];
            M += st[r * L + 4 * C];
        }
        const double inv = (double)mi[C + c];
        const float gm = gamma ? gamma[c] : 1.f;
        if (dgamma) dgamma[c] = (float)(own[C + c] * inv);
        if (dbeta) dbeta[c] = (float)own[c];
        const float cg = (float)(S / M), ck = (float)(D * inv * inv / M), cs = (float)(inv * (double)gm);
        coef[c] = cg;
        coef[C + c] = ck;
        coef[2 * C + c] = cs;
        if (has_max)
            b = (float)((own[2 * C + c] + fabs((double)cg) + own[3 * C + c] * fabs((double)ck)) * fabs((double)cs) *
                        1.0001);
    }
    if (!amax) return;
    if (!has_max) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *amax = 0u;   // the apply's atomicMax starts from 0
        return;
    }
    bmax[threadIdx.x] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = 0.f;
        for (int i = 0; i < 256; ++i) m = fmaxf(m, bmax[i]);
        atomicMax(amax, __float_as_uint(m));                  // zeroed by the reduce kernel
    }
}

// dy = ((dz - gm) - (y - mean)*k) * (invstd*gamma), dz = g*(out>0) (MASK) or g.
// AMAX: also max|dy| (IEEE bits, block-reduced, one atomicMax per block; the grid
// is capped at 512 blocks since same-address device atomics serialise) — the
// power-of-two scale of the f16x3 backward convs' gradient operand, so they need
// no separate absmax pass over dy
// SPLIT: dy is written as the packed f16x3 split of dy * 2^e, e from the upper
// bound finalize left in *amax (the operand of the x3 backward convs, which need
// no separate hkp_split_pack_x3 pass); the fp32 dy only if dy != NULL
template <int MASK, bool AMAX, bool SPLIT = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(long n4, int C4, const f32x4* __restrict__ g,
                                                          const f32x4* __restrict__ out, const f32x4* __restrict__ y,
                                                          const f32x4* __restrict__ mean,
                                                          const f32x4* __restrict__ coef, f32x4* __restrict__ dy,
                                                          unsigned* __restrict__ amax, _Float16* __restrict__ dsplit) {
    const long stride = (long)gridDim.x * blockDim.x;
    unsigned mx = 0;
    const float gsc = SPLIT ? pow2_scale_for(amax) : 1.f;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const int c4 = (int)(i % C4);
        f32x4 d = g[i];
        const f32x4 v = y[i], mu = mean[c4], gm = coef[c4], kk = coef[C4 + c4], sc = coef[2 * C4 + c4];
        if constexpr (MASK == 1) {
            const f32x4 o = out[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) d[e] = o[e] > 0.f ? d[e] : 0.f;
        } else if constexpr (MASK == 2) {   // out = the forward's [scale | shift]
            const f32x4 ma = out[c4], mb = out[C4 + c4];
#pragma unroll
            for (int e = 0; e < 4; ++e) d[e] = __fadd_rn(__fmul_rn(v[e], ma[e]), mb[e]) > 0.f ? d[e] : 0.f;
        }
        f32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = ((d[e] - gm[e]) - (v[e] - mu[e]) * kk[e]) * sc[e];
        if (!SPLIT || dy) dy[i] = r;
        if constexpr (SPLIT) {
            f32x4 rs;
#pragma unroll
            for (int e = 0; e < 4; ++e) rs[e] = r[e] * gsc;
            store_split4(rs, i, dsplit, 3);
        }
        if constexpr (AMAX) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const unsigned b = __float_as_uint(r[e]) & 0x7FFFFFFFu;
                mx = b > mx ? b : mx;
            }
        }
    }
    if constexpr (AMAX) {
        __shared__ unsigned red[4];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned t = __shfl_xor(mx, o);
            mx = t > mx ? t : mx;
        }
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned a = red[0] > red[1] ? red[0] : red[1], b = red[2] > red[3] ? red[2] : red[3];
            atomicMax(amax, a > b ? a : b);
        }
    }
}

// Stem maxpool(3x3,s2,p1) ∘ relu ∘ BN-affine backward, as a gather over the ≤2x2
// pooling windows that contain each input pixel.  Emits dz = dL/d(BN output)
// (ReLU mask applied).  Window argmax = first max in (dr, ds) scan order, NaN
// wins — ATen's CPU max_pool2d rule.
// dz at input pixel (h, w): the sum of dpool over the (<= 4) windows whose
// routed tap (written by the forward, hkp_bn_relu_maxpool) is this pixel, in
// window order (ho, wo) ascending; 0xFF routes nothing (window max <= 0: the
// ReLU derivative is 0 at its argmax).
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(int N, int H, int W, int C, int Ho, int Wo,
                                                         const float* __restrict__ dpool,
                                                         const uchar4* __restrict__ route, float* __restrict__ dz) {
    const int C4 = C >> 2;
    const long total = (long)N * H * W * C4;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int c4 = (int)(i % C4);
        long p = i / C4;
        const int w = (int)(p % W);
        p /= W;
        const int h = (int)(p % H);
        const int n = (int)(p / H);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const int ho0 = h >> 1, ho1 = min((h + 1) >> 1, Ho - 1);
        const int wo0 = w >> 1, wo1 = min((w + 1) >> 1, Wo - 1);
        for (int ho = ho0; ho <= ho1; ++ho) {
            for (int wo = wo0; wo <= wo1; ++wo) {
                const long o = (((long)n * Ho + ho) * Wo + wo) * C4 + c4;
                const uchar4 r = route[o];
                const unsigned me = (unsigned)((h - (ho * 2 - 1)) * 3 + (w - (wo * 2 - 1)));
                if (r.x == me || r.y == me || r.z == me || r.w == me) {
                    const f32x4 d = *(const f32x4*)(dpool + o * 4);
                    if (r.x == me) acc[0] += d[0];
                    if (r.y == me) acc[1] += d[1];
                    if (r.z == me) acc[2] += d[2];
                    if (r.w == me) acc[3] += d[3];
                }
            }
        }
        *(f32x4*)(dz + i * 4) = acc;
    }
}

static inline int grid_cap(long work) {
    long g = (work + 255) / 256;
    if (g > 4096) g = 4096;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace hkp

using namespace hkp;

extern "C" int64_t hkp_bn_bwd_tiles(int64_t m) { return (m + BNB_TILE - 1) / BNB_TILE; }

extern "C" int hkp_bn_bwd_reduce(int64_t m, int32_t c, const float* g, const float* out_mask, const float* relu_ss,
                                 const float* y, const float* mean_invstd, float* dz, float* partials, float* maxima,
                                 uint32_t* dy_bound_bits, hkp_stream_t stream) {
    HKP_CHECK_ARG(m > 0 && c > 0 && c % 4 == 0, "hkp_bn_bwd_reduce: bad sizes");
    HKP_CHECK_ARG(!(out_mask && relu_ss), "hkp_bn_bwd_reduce: out_mask and relu_ss are exclusive");
    HKP_CHECK_ARG(g && y && mean_invstd && partials, "hkp_bn_bwd_reduce: null tensor");
    const int C4 = c / 4;
    HKP_CHECK_ARG((C4 <= 256 && 256 % C4 == 0) || C4 == 512, "hkp_bn_bwd_reduce: unsupported C=%d", c);
    const long tiles = (m + BNB_TILE - 1) / BNB_TILE;
    hipStream_t st = as_stream(stream);
    HKP_CHECK_ARG(!dy_bound_bits || maxima, "hkp_bn_bwd_reduce: dy_bound_bits needs maxima");
    const float* mk = out_mask ? out_mask : relu_ss;
#define HKP_BNR(G, MK, MX)                                                                                          \
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<G, MK, MX>), dim3((unsigned)tiles), dim3(256), 0, st, (long)m, c, g,   \
                       mk, y, mean_invstd, dz, partials, maxima, (unsigned*)dy_bound_bits)
#define HKP_BNR2(G, MK)                  \
    if (maxima) HKP_BNR(G, MK, true);    \
    else HKP_BNR(G, MK, false)
#define HKP_BNR3(G)                                           \
    if (out_mask) { HKP_BNR2(G, 1); }                         \
    else if (relu_ss) { HKP_BNR2(G, 2); }                     \
    else { HKP_BNR2(G, 0); }
    if (C4 == 512) {
        HKP_BNR3(2);
    } else {
        HKP_BNR3(1);
    }
#undef HKP_BNR3
#undef HKP_BNR2
#undef HKP_BNR
    HKP_LAUNCH_CHECK("hkp_bn_bwd_reduce");
    return HKP_OK;
}

int hkp_fin_regs();   // bn.hip: hkp_debug_fin_regs

static int bwd_fin(int32_t c, int64_t m, const float* partials, const float* maxima, const float* mean_invstd,
                   const float* gamma, float* dgamma, float* dbeta, float* coef, uint32_t* dy_amax_bits,
                   double* stats, hkp_stream_t stream) {
    const long tiles = (m + BNB_TILE - 1) / BNB_TILE;
    const int cpb = partials_cpb(c);
    const long per = hkp_fin_regs() ? (tiles + 256 / cpb - 1) / (256 / cpb) : 1L << 40;   // partials per tile lane
#define HKP_BFIN1(CPB, NT, NB)                                                                                     \
    hipLaunchKernelGGL((bn_bwd_finalize_kernel<CPB, NT, NB>), dim3((c + CPB - 1) / CPB), dim3(NT), 0,               \
                       as_stream(stream), c, (long)m, tiles, partials, mean_invstd, gamma, dgamma, dbeta, coef,       \
                       maxima, (unsigned*)dy_amax_bits, stats)
#define HKP_BFIN(CPB)                                  \
    if (tiles >= 4096) { HKP_BFIN1(CPB, 1024, 0); } \
    else if (per <= 8) { HKP_BFIN1(CPB, 256, 8); } \
    else if (per <= 16) { HKP_BFIN1(CPB, 256, 16); } \
    else { HKP_BFIN1(CPB, 256, 0); }
    if (cpb == 8) { HKP_BFIN(8); }
    else if (cpb == 4) { HKP_BFIN(4); }
    else if (cpb == 2) { HKP_BFIN(2); }
    else { HKP_BFIN(1); }
#undef HKP_BFIN
#undef HKP_BFIN1
    HKP_LAUNCH_CHECK("hkp_bn_bwd_finalize");
    return HKP_OK;
}

extern "C" int hkp_bn_bwd_finalize(int32_t c, int64_t m, const float* partials, const float* maxima,
                                   const float* mean_invstd, const float* gamma, float* dgamma, float* dbeta,
                                   float* coef, uint32_t* dy_amax_bits, hkp_stream_t stream) {
    HKP_CHECK_ARG(c > 0 && m > 0 && partials && mean_invstd && coef, "hkp_bn_bwd_finalize: bad args");
    return bwd_fin(c, m, partials, maxima, mean_invstd, gamma, dgamma, dbeta, coef, dy_amax_bits, nullptr, stream);
}

extern "C" int hkp_bn_bwd_stats(int32_t c, int64_t m, const float* partials, const float* maxima,
                                const float* mean_invstd, double* stats, hkp_stream_t stream) {
    HKP_CHECK_ARG(c > 0 && m > 0 && partials && mean_invstd && stats, "hkp_bn_bwd_stats: bad args");
    return bwd_fin(c, m, partials, maxima, mean_invstd, nullptr, nullptr, nullptr, nullptr, nullptr, stats, stream);
}

extern "C" int hkp_bn_bwd_finalize_ranks(int32_t c, int32_t nranks, const double* stats, const double* own,
                                         int32_t has_maxima, const float* mean_invstd, const float* gamma,
                                         float* dgamma, float* dbeta, float* coef, uint32_t* dy_amax_bits,
                                         hkp_stream_t stream) {
    HKP_CHECK_ARG(c > 0 && nranks > 0 && stats && own && mean_invstd && coef, "hkp_bn_bwd_finalize_ranks: bad args");
    hipLaunchKernelGGL(bn_bwd_fin_ranks_kernel, dim3((c + 255) / 256), dim3(256), 0, as_stream(stream), c, nranks,
                       stats, own, has_maxima ? 1 : 0, mean_invstd, gamma, dgamma, dbeta, coef,
                       (unsigned*)dy_amax_bits);
    HKP_LAUNCH_CHECK("hkp_bn_bwd_finalize_ranks");
    return HKP_OK;
}

extern "C" int hkp_bn_bwd_apply(int64_t m, int32_t c, const float* g, const float* out_mask, const float* relu_ss,
                                const float* y, const float* mean_invstd, const float* coef, float* dy,
                                uint32_t* dy_amax_bits, uint16_t* dy_split, hkp_stream_t stream) {
    HKP_CHECK_ARG(m > 0 && c > 0 && c % 4 == 0, "hkp_bn_bwd_apply: bad sizes");
    HKP_CHECK_ARG(!(out_mask && relu_ss), "hkp_bn_bwd_apply: out_mask and relu_ss are exclusive");
    const float* mk = out_mask ? out_mask : relu_ss;
    const int mmode = out_mask ? 1 : (relu_ss ? 2 : 0);
    HKP_CHECK_ARG(g && y && mean_invstd && coef && (dy || dy_split), "hkp_bn_bwd_apply: null tensor");
    HKP_CHECK_ARG(!dy_split || (dy_amax_bits && c % 32 == 0), "hkp_bn_bwd_apply: dy_split needs the bound and c%%32==0");
    const long n4 = m * (long)c / 4;
    hipStream_t st = as_stream(stream);
#define HKP_BWD_APPLY3(MASK, AMAX, SPLIT)                                                                            \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<MASK, AMAX, SPLIT>),                                                    \
                       dim3(AMAX ? std::min(grid_cap(n4), 512) : grid_cap(n4)), dim3(256), 0, st, n4, c / 4,       \
                       (const f32x4*)g, (const f32x4*)mk, (const f32x4*)y, (const f32x4*)mean_invstd,             \
                       (const f32x4*)coef, (f32x4*)dy, (unsigned*)dy_amax_bits, (_Float16*)dy_split)
#define HKP_BWD_APPLY(MASK, AMAX) HKP_BWD_APPLY3(MASK, AMAX, false)
#define HKP_BWD_MODES(AMAX, SPLIT)                                                    \
    if (mmode == 1) { HKP_BWD_APPLY3(1, AMAX, SPLIT); }                              \
    else if (mmode == 2) { HKP_BWD_APPLY3(2, AMAX, SPLIT); }                         \
    else { HKP_BWD_APPLY3(0, AMAX, SPLIT); }
    if (dy_split) {
        HKP_BWD_MODES(false, true);
    } else if (dy_amax_bits) {
        HKP_BWD_MODES(true, false);
    } else {
        HKP_BWD_MODES(false, false);
    }
#undef HKP_BWD_MODES
#undef HKP_BWD_APPLY
#undef HKP_BWD_APPLY3
    HKP_LAUNCH_CHECK("hkp_bn_bwd_apply");
    return HKP_OK;
}

extern "C" int hkp_maxpool_bwd(int32_t n, int32_t h, int32_t w, int32_t c, const float* dpool, const uint8_t* route,
                               float* dz, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0, "hkp_maxpool_bwd: bad sizes");
    HKP_CHECK_ARG(dpool && route && dz, "hkp_maxpool_bwd: null tensor");
    const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
    const long work = (long)n * h * w * (c / 4);
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_cap(work)), dim3(256), 0, as_stream(stream), n, h, w, c, ho, wo,
                       dpool, (const uchar4*)route, dz);
    HKP_LAUNCH_CHECK("hkp_maxpool_bwd");
    return HKP_OK;
}
