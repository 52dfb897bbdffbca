// BatchNorm (train-mode statistics, apply+ReLU+residual, stem BN+ReLU+maxpool).
//
// Reference semantics: nn.BatchNorm2d in TRAIN mode everywhere
// (the reference never calls .eval()): normalise with the biased
// batch variance over (N,H,W), eps 1e-5; running stats with momentum 0.1 and the
// unbiased variance; num_batches_tracked += 1.  Output = x*alpha + beta with
// alpha = invstd*gamma, beta = bias - mean*alpha (fp32, two roundings, as
// ATen's batch_norm_cpu_transform_input).
#include <cstdlib>

#include "common.h"

// x*alpha + beta as two roundings (ATen's Vectorized mul then add): no contraction.
#pragma clang fp contract(off)

namespace hkp {

// SyncBN: instead of the scale/shift, a rank's statistics for the
// cross-rank merge (hkp_bn_finalize_ranks): [mean[C] | M2[C] | count], fp64
__device__ __forceinline__ void bn_rank_stats_store(int c, int C, long count, double mean, double m2, double* stats) {
    stats[c] = mean;
    stats[C + c] = m2;
    if (c == 0) stats[2 * C] = (double)count;
}

// CPB channels per block (partials_cpb); deterministic fixed-order fp64 merge
// NT threads per block: 256, or 1024 for long tile lists (the stem's 19,200
// tiles at C2: per-thread load chains of 75 tiles took 75 us with 256 threads).
// (A one-pass form — each lane's tiles folded by Chan's pairwise merge, the lanes
// merged the same way — measured no faster: B=8 shard 1494 -> 1484 img/s, C2 / C4 /
// C3 unchanged; profiles/r05_fin_*.)
// NB > 0 (tiles <= NB * TL): every partial of the lane loaded in ONE round and
// kept in registers for the second pass — the same sums in the same order (so the
// same bits) with one exposed load latency instead of 2 x ceil(tiles / (8 TL));
// tile means of full tiles (tile_rows a power of two) by an exact multiply
template <int CPB, int NT = 256, int NB = 0>
__global__ __launch_bounds__(NT) void bn_finalize_kernel(int C, long count, long tiles, int tile_rows,
                                                         const float* __restrict__ part, const float* gamma,
                                                         const float* beta, float momentum, float eps, float* rmean,
                                                         float* rvar, int64_t* nbt, float* ss, float* mi,
                                                         double* stats) {
    constexpr int TL = NT / CPB, NW = NT / 64;
    __shared__ double red[NW][8];
    const int cl = threadIdx.x % CPB, tl = threadIdx.x / CPB, c = blockIdx.x * CPB + cl;
    const bool ok = c < C;
    if constexpr (NB > 0) {
        float2 v[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const long t = tl + (long)j * TL;
            v[j] = ok && t < tiles ? *(const float2*)(part + (t * C + c) * 2) : make_float2(0.f, 0.f);
        }
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < NB; ++j) s += (double)v[j].x;
        const double mean = lanes_sum_d<CPB, NW>(s, red) / (double)count;
        const bool pow2 = (tile_rows & (tile_rows - 1)) == 0;
        const double inv_rows = 1.0 / (double)tile_rows;   // exact for a power of two
        double q = 0.0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const long t = tl + (long)j * TL;
            if (ok && t < tiles) {
                const long n_t = min((long)tile_rows, count - t * tile_rows);
                const double tm = pow2 && n_t == tile_rows ? (double)v[j].x * inv_rows : (double)v[j].x / (double)n_t;
                const double dm = tm - mean;
                q += (double)v[j].y + (double)n_t * dm * dm;
            }
        }
        const double m2 = lanes_sum_d<CPB, NW>(q, red);
        if (tl == 0 && ok) {
            if (stats) bn_rank_stats_store(c, C, count, mean, m2, stats);
            else bn_fin_store(c, C, count, mean, m2, gamma, beta, momentum, eps, rmean, rvar, nbt, ss, mi);
        }
        return;
    }
    // tiles t = tl, tl + TL, ... in order; 8 loads in flight per batch (the loop
    // is latency-bound), zero-filled past the end (exact: s + 0 = s)
    double s = 0.0;
    if (ok)
        for (long t0 = tl; t0 < tiles; t0 += 8 * TL) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const long t = t0 + (long)j * TL;
                v[j] = t < tiles ? part[(t * C + c) * 2] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) s += (double)v[j];
        }
    const double mean = lanes_sum_d<CPB, NW>(s, red) / (double)count;
    double q = 0.0;
    if (ok)
        for (long t0 = tl; t0 < tiles; t0 += 8 * TL) {
            float2 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const long t = t0 + (long)j * TL;
                v[j] = t < tiles ? *(const float2*)(part + (t * C + c) * 2) : make_float2(0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const long t = t0 + (long)j * TL;
                if (t < tiles) {
                    const long n_t = min((long)tile_rows, count - t * tile_rows);
                    const double dm = (double)v[j].x / (double)n_t - mean;
                    q += (double)v[j].y + (double)n_t * dm * dm;
                }
            }
        }
    const double m2 = lanes_sum_d<CPB, NW>(q, red);
    if (tl == 0 && ok) {
        if (stats) bn_rank_stats_store(c, C, count, mean, m2, stats);
        else bn_fin_store(c, C, count, mean, m2, gamma, beta, momentum, eps, rmean, rvar, nbt, ss, mi);
    }
}

// Two-level form for long tile lists (hkp_bn_finalize_ws).  The one-kernel merge
// above runs C/CPB blocks whose threads walk `tiles` partials in dependent load
// batches: the stem and layer1 (C = 64, 19,200 / 4,800 tiles at C2) used 64 CUs
// for 23 us, and R50's C = 2048 convs (C4: 4,800 tiles, 78 MB of partials) 30-60 us.
// Level 1 (bn_fin_chunk_kernel, grid [C/64][chunks]): a block = 64 channel lanes x
// 16 tile lanes reduces one chunk of FIN_CHUNK tiles — each lane holds its 8
// partials in registers — to the chunk's (sum, M2 about the chunk mean), both
// fixed-order fp64 (Chan, as the one-kernel form does over all tiles).  A wave
// reads one tile row of 64 channels: 512 contiguous bytes.
// Level 2 (bn_fin_merge_kernel, grid C/64): the chunks merged by the same formula
// in fixed order -> mean, M2 -> bn_fin_store.  Deterministic run to run.
constexpr int FIN_TL = 16, FIN_TPL = 8, FIN_CHUNK = FIN_TL * FIN_TPL;

__device__ __forceinline__ double fin_col_sum(double v, double (*red)[64], int tl, int cl) {
    __syncthreads();                               // red free (a previous call's readers are done)
    red[tl][cl] = v;
    __syncthreads();
    double a[FIN_TL];
#pragma unroll
    for (int i = 0; i < FIN_TL; ++i) a[i] = red[i][cl];
#pragma unroll
    for (int w = FIN_TL / 2; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) a[i] = a[2 * i] + a[2 * i + 1];
    return a[0];
}

__global__ __launch_bounds__(1024) void bn_fin_chunk_kernel(int C, long count, long tiles, int tile_rows,
                                                            const float* __restrict__ part, double2* __restrict__ ws) {
    __shared__ double red[FIN_TL][64];
    const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
    const bool ok = c < C;
    const long t0 = (long)blockIdx.y * FIN_CHUNK;
    float2 v[FIN_TPL];
#pragma unroll
    for (int j = 0; j < FIN_TPL; ++j) {
        const long t = t0 + tl + (long)FIN_TL * j;
        v[j] = ok && t < tiles ? *(const float2*)(part + (t * C + c) * 2) : make_float2(0.f, 0.f);
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < FIN_TPL; ++j) s += (double)v[j].x;
    const double S = fin_col_sum(s, red, tl, cl);
    const long te = min(tiles, t0 + FIN_CHUNK);
    const long nk = min(count, te * (long)tile_rows) - t0 * (long)tile_rows;   // rows in this chunk
    const double mk = S / (double)nk;
    double q = 0.0;
#pragma unroll
    for (int j = 0; j < FIN_TPL; ++j) {
        const long t = t0 + tl + (long)FIN_TL * j;
        if (t < tiles) {
            const long n_t = min((long)tile_rows, count - t * tile_rows);
            const double dm = (double)v[j].x / (double)n_t - mk;
            q += (double)v[j].y + (double)n_t * dm * dm;
        }
    }
    const double Q = fin_col_sum(q, red, tl, cl);
    if (tl == 0 && ok) ws[blockIdx.y * (long)C + c] = make_double2(S, Q);
}

__global__ __launch_bounds__(1024) void bn_fin_merge_kernel(int C, long count, long chunks, int tile_rows,
                                                            const double2* __restrict__ ws, const float* gamma,
                                                            const float* beta, float momentum, float eps,
                                                            float* rmean, float* rvar, int64_t* nbt, float* ss,
                                                            float* mi, double* stats) {
    __shared__ double red[FIN_TL][64];
    const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
    const bool ok = c < C;
    const long rows = (long)FIN_CHUNK * tile_rows;     // rows per full chunk
    double s = 0.0;
    if (ok)
        for (long k = tl; k < chunks; k += FIN_TL) s += ws[k * C + c].x;
    const double mean = fin_col_sum(s, red, tl, cl) / (double)count;
    double q = 0.0;
    if (ok)
        for (long k = tl; k < chunks; k += FIN_TL) {
            const double2 w = ws[k * C + c];
            const long nk = min(rows, count - k * rows);
            const double dm = w.x / (double)nk - mean;
            q += w.y + (double)nk * dm * dm;
        }
    const double m2 = fin_col_sum(q, red, tl, cl);
    if (tl == 0 && ok) {
        if (stats) bn_rank_stats_store(c, C, count, mean, m2, stats);
        else bn_fin_store(c, C, count, mean, m2, gamma, beta, momentum, eps, rmean, rvar, nbt, ss, mi);
    }
}

// Cross-rank merge of SyncBN statistics: st = [R][2C+1] (each rank's
// bn_rank_stats_store block, gathered in rank order).  Fixed order over ranks,
// the same two-pass form as the chunk merge: mean = sum_r n_r*mean_r / N,
// M2 = sum_r (M2_r + n_r*(mean_r - mean)^2).  Every rank merges the same bytes
// in the same order, so every rank gets the same scale/shift and running stats.
__global__ void bn_fin_ranks_kernel(int C, int R, const double* __restrict__ st, const float* gamma, const float* beta,
                                    float momentum, float eps, float* rmean, float* rvar, int64_t* nbt, float* ss,
                                    float* mi) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const long L = 2L * C + 1;
    double n = 0.0, s = 0.0;
    for (int r = 0; r < R; ++r) {
        const double nr = st[r * L + 2 * C];
        n += nr;
        s += nr * st[r * L + c];
    }
    const double mean = R == 1 ? st[c] : s / n;
    double m2 = 0.0;
    for (int r = 0; r < R; ++r) {
        const double nr = st[r * L + 2 * C], dm = st[r * L + c] - mean;
        m2 += st[r * L + C + c] + nr * dm * dm;
    }
    bn_fin_store(c, C, (long)n, mean, m2, gamma, beta, momentum, eps, rmean, rvar, nbt, ss, mi);
}

__global__ void bn_eval_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                               float eps, float* ss, float* mi) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float inv = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    const float alpha = __fmul_rn(inv, g);
    ss[c] = alpha;
    ss[C + c] = __fsub_rn(b, __fmul_rn(rm[c], alpha));
    if (mi) {
        mi[c] = rm[c];
        mi[C + c] = inv;
    }
}

// RES: 0 none, 1 raw residual, 2 affine residual (downsample BN), 3 raw residual
// read from its packed split (hi + lo, written by the producer of the block input)
// FIX: the grid stride is a multiple of C/4 — every vector a thread visits has
// the same 4 channels: scale/shift loaded once, and two vectors (i, i + stride)
// in flight per thread.
template <int RES, bool RELU, bool FIX>
__global__ __launch_bounds__(256) void bn_apply_kernel(long n4, int C4, const f32x4* __restrict__ y,
                                                       const f32x4* __restrict__ sc, const f32x4* __restrict__ sh,
                                                       const f32x4* __restrict__ res, const f32x4* __restrict__ rsc,
                                                       const f32x4* __restrict__ rsh, const _Float16* __restrict__ rsplit,
                                                       f32x4* __restrict__ out, _Float16* __restrict__ osplit,
                                                       int passes) {
    const long stride = (long)gridDim.x * blockDim.x;
    const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    struct In {
        f32x4 v, r;
        h16x4 h, l;
    };
    auto load = [&](long i) {
        In x;
        x.v = y[i];
        if constexpr (RES == 1 || RES == 2) x.r = res[i];
        if constexpr (RES == 3) {
            const long e0 = i * 4, off = 2 * e0 - (e0 & 31);
            x.h = *(const h16x4*)(rsplit + off);
            x.l = *(const h16x4*)(rsplit + off + 32);
        }
        return x;
    };
    auto one = [&](long i, const In& x, const f32x4& a, const f32x4& b, const f32x4& ra, const f32x4& rb) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = __fadd_rn(__fmul_rn(x.v[e], a[e]), b[e]);
        if constexpr (RES == 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = __fadd_rn(o[e], x.r[e]);
        } else if constexpr (RES == 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = __fadd_rn(o[e], __fadd_rn(__fmul_rn(x.r[e], ra[e]), rb[e]));
        } else if constexpr (RES == 3) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = __fadd_rn(o[e], __fadd_rn((float)x.h[e], (float)x.l[e]));
        }
        if constexpr (RELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = o[e] > 0.f ? o[e] : 0.f;
        }
        if (out) out[i] = o;
        if (osplit) store_split4(o, i, osplit, passes);   // operand split for the next conv
    };
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if constexpr (FIX) {
        const int c4 = (int)(i0 % C4);
        const f32x4 a = sc[c4], b = sh[c4];
        const f32x4 ra = RES == 2 ? rsc[c4] : z, rb = RES == 2 ? rsh[c4] : z;
        long i = i0;
        for (; i + stride < n4; i += 2 * stride) {
            const In x0 = load(i), x1 = load(i + stride);
            one(i, x0, a, b, ra, rb);
            one(i + stride, x1, a, b, ra, rb);
        }
        if (i < n4) one(i, load(i), a, b, ra, rb);
    } else {
        for (long i = i0; i < n4; i += stride) {
            const int c4 = (int)(i % C4);
            one(i, load(i), sc[c4], sh[c4], RES == 2 ? rsc[c4] : z, RES == 2 ? rsh[c4] : z);
        }
    }
}

// Plain-fp16 path (BASELINE config C4, autocast semantics): y is the fp16 conv
// output, the result is written in fp16 (the next conv's operand) and, for the
// block feeding the head, also in fp32.  RES: 0 none, 1 raw fp16 residual (the
// block input), 2 affine fp16 residual (the downsample conv's y with its BN).
// The BN arithmetic itself is fp32 (x*alpha + beta, two roundings, as above).
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
// FIX: the grid stride is a multiple of C/8, so every element a thread visits
// has the same 8 channels — their scale/shift are loaded once, not per element
// (16-32 scalar loads per 16-B vector otherwise).
template <int RES, bool RELU, bool FIX>
__global__ __launch_bounds__(256) void bn_apply_f16_kernel(long n8, int C8, const h16x8* __restrict__ y,
                                                           const float* __restrict__ ss, const h16x8* __restrict__ res,
                                                           const float* __restrict__ rss, h16x8* __restrict__ out,
                                                           f32x4* __restrict__ out32) {
    const int C = C8 * 8;
    const long stride = (long)gridDim.x * blockDim.x;
    const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    float a[8], b[8], ra[8], rb[8];
    auto load_ss = [&](int c0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            a[e] = ss[c0 + e];
            b[e] = ss[C + c0 + e];
            if constexpr (RES == 2) {
                ra[e] = rss[c0 + e];
                rb[e] = rss[C + c0 + e];
            }
        }
    };
    auto one = [&](long i, const h16x8& v, const h16x8& r) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = __fadd_rn(__fmul_rn((float)v[e], a[e]), b[e]);
        if constexpr (RES == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = __fadd_rn(o[e], (float)r[e]);
        } else if constexpr (RES == 2) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = __fadd_rn(o[e], __fadd_rn(__fmul_rn((float)r[e], ra[e]), rb[e]));
        }
        h16x8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if constexpr (RELU) o[e] = o[e] > 0.f ? o[e] : 0.f;
            h[e] = (_Float16)o[e];
        }
        __builtin_nontemporal_store(h, out + i);
        if (out32) {
            out32[2 * i] = f32x4{o[0], o[1], o[2], o[3]};
            out32[2 * i + 1] = f32x4{o[4], o[5], o[6], o[7]};
        }
    };
    if constexpr (FIX) {
        // two vectors per thread in flight (i and i + stride share the channels)
        load_ss((int)(i0 % C8) * 8);
        long i = i0;
        for (; i + stride < n8; i += 2 * stride) {
            const h16x8 v0 = __builtin_nontemporal_load(y + i), v1 = __builtin_nontemporal_load(y + i + stride);
            h16x8 r0{}, r1{};
            if constexpr (RES != 0) {
                r0 = __builtin_nontemporal_load(res + i);
                r1 = __builtin_nontemporal_load(res + i + stride);
            }
            one(i, v0, r0);
            one(i + stride, v1, r1);
        }
        if (i < n8) {
            h16x8 r0{};
            if constexpr (RES != 0) r0 = res[i];
            one(i, y[i], r0);
        }
    } else {
        for (long i = i0; i < n8; i += stride) {
            load_ss((int)(i % C8) * 8);
            h16x8 r0{};
            if constexpr (RES != 0) r0 = res[i];
            one(i, y[i], r0);
        }
    }
}

// maxpool 3x3 / s2 / p1 (-inf padding) of relu(y*a+b); one thread per 4 channels of one output pixel.
// IDX: the index type of the (pixel, channel-group) decomposition — 32-bit when
// the output and input element counts fit (the stem maps: 64-bit divisions were
// ~4 per element group)
template <typename IDX>
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(int N, int H, int W, int C, int Ho, int Wo,
                                                             const float* __restrict__ y,
                                                             const float* __restrict__ ss,
                                                             float* __restrict__ out, _Float16* __restrict__ osplit,
                                                             int passes, uchar4* __restrict__ route) {
    const IDX C4 = (IDX)(C >> 2);
    const IDX total = (IDX)N * (IDX)Ho * (IDX)Wo * C4;
    const IDX stride = (IDX)gridDim.x * (IDX)blockDim.x;
    for (IDX i = (IDX)blockIdx.x * (IDX)blockDim.x + (IDX)threadIdx.x; i < total; i += stride) {
        const int c4 = (int)(i % C4);
        IDX p = i / C4;
        const int wo = (int)(p % (IDX)Wo);
        p /= (IDX)Wo;
        const int ho = (int)(p % (IDX)Ho);
        const int n = (int)(p / (IDX)Ho);
        const f32x4 a = *(const f32x4*)(ss + 4 * c4), b = *(const f32x4*)(ss + C + 4 * c4);
        f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        int tap[4] = {0, 0, 0, 0};
#pragma unroll
        for (int dr = 0; dr < 3; ++dr) {
            const int hi = ho * 2 - 1 + dr;
            if ((unsigned)hi >= (unsigned)H) continue;
#pragma unroll
            for (int ds = 0; ds < 3; ++ds) {
                const int wi = wo * 2 - 1 + ds;
                if ((unsigned)wi >= (unsigned)W) continue;
                const f32x4 v = *(const f32x4*)(y + (((long)n * H + hi) * W + wi) * C + 4 * c4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float t = __fadd_rn(__fmul_rn(v[e], a[e]), b[e]);
                    t = t > 0.f ? t : 0.f;
                    if (t > m[e]) {            // first maximum wins (ATen's window scan)
                        m[e] = t;
                        tap[e] = dr * 3 + ds;
                    }
                }
            }
        }
        if (out) *(f32x4*)(out + (long)i * 4) = m;
        if (osplit) store_split4(m, (long)i, osplit, passes);
        if (route)   // the tap the window's gradient goes to; 0xFF: max <= 0, ReLU blocks it
            route[i] = make_uchar4(m[0] > 0.f ? tap[0] : 255, m[1] > 0.f ? tap[1] : 255,
                                   m[2] > 0.f ? tap[2] : 255, m[3] > 0.f ? tap[3] : 255);
    }
}

static inline int grid_for(long work, int block = 256, long cap = 256L * 16) {
    long g = (work + block - 1) / block;
    if (g > cap) g = cap;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace hkp

using namespace hkp;

// Debug / A/B (tools/ only): 0 runs the finalize merges' batched-load loops where
// the register-held forms (NB > 0) would run — the same bits
HKP_AB_KNOB(int, g_fin_regs, 1);
#ifdef HKP_AB_KNOBS
extern "C" void hkp_debug_fin_regs(int32_t on) { g_fin_regs = on != 0; }
#endif
int hkp_fin_regs() { return g_fin_regs; }

// The one-kernel (fin_one) and two-level (fin_two) merges of the tile partials:
// scale/shift (+ running stats), or (stats != null) the rank's SyncBN statistics.
static int fin_one(const char* who, int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                   const float* gamma, const float* beta, float momentum, float eps, float* running_mean,
                   float* running_var, int64_t* num_batches_tracked, float* scale_shift, float* mean_invstd,
                   double* stats, hkp_stream_t stream) {
    HKP_CHECK_ARG(c > 0 && count > 0 && tiles > 0 && tile_rows > 0, "%s: bad sizes", who);
    HKP_CHECK_ARG(partials && (scale_shift || stats), "%s: null tensor", who);
    HKP_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr), "%s: running stats pair", who);
    HKP_CHECK_ARG((tiles - 1) * (int64_t)tile_rows < count && tiles * (int64_t)tile_rows >= count,
                  "%s: tiles/tile_rows inconsistent with count", who);
    const int cpb = partials_cpb(c);
    // partials per tile lane of the 256-thread form: held in registers up to 32
    const long per = g_fin_regs ? (tiles + 256 / cpb - 1) / (256 / cpb) : 1L << 40;
#define HKP_FIN1(CPB, NT, NB)                                                                                      \
    hipLaunchKernelGGL((bn_finalize_kernel<CPB, NT, NB>), dim3((c + CPB - 1) / CPB), dim3(NT), 0, as_stream(stream), \
                       c, (long)count, (long)tiles, tile_rows, partials, gamma, beta, momentum, eps, running_mean,   \
                       running_var, num_batches_tracked, scale_shift, mean_invstd, stats)
#define HKP_FIN(CPB)                                  \
    if (tiles >= 4096) { HKP_FIN1(CPB, 1024, 0); } \
    else if (per <= 8) { HKP_FIN1(CPB, 256, 8); } \
    else if (per <= 16) { HKP_FIN1(CPB, 256, 16); } \
    else if (per <= 32) { HKP_FIN1(CPB, 256, 32); } \
    else { HKP_FIN1(CPB, 256, 0); }
    if (cpb == 8) { HKP_FIN(8); }
    else if (cpb == 4) { HKP_FIN(4); }
    else if (cpb == 2) { HKP_FIN(2); }
    else { HKP_FIN(1); }
#undef HKP_FIN
#undef HKP_FIN1
    HKP_LAUNCH_CHECK(who);
    return HKP_OK;
}

extern "C" int64_t hkp_bn_finalize_workspace_bytes(int32_t c, int64_t tiles) {
    if (c <= 0 || tiles <= 0) return -1;
    return ((tiles + FIN_CHUNK - 1) / FIN_CHUNK) * (int64_t)c * (int64_t)sizeof(double2);
}

static int fin_two(const char* who, int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                   const float* gamma, const float* beta, float momentum, float eps, float* running_mean,
                   float* running_var, int64_t* num_batches_tracked, float* scale_shift, float* mean_invstd,
                   double* stats, void* workspace, int64_t ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(c > 0 && count > 0 && tiles > 0 && tile_rows > 0, "%s: bad sizes", who);
    HKP_CHECK_ARG(partials && (scale_shift || stats) && workspace, "%s: null tensor", who);
    HKP_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr), "%s: running stats pair", who);
    HKP_CHECK_ARG((tiles - 1) * (int64_t)tile_rows < count && tiles * (int64_t)tile_rows >= count,
                  "%s: tiles/tile_rows inconsistent with count", who);
    const int64_t need = hkp_bn_finalize_workspace_bytes(c, tiles);
    HKP_CHECK_ARG(ws_bytes >= need, "%s: workspace %ld < %ld", who, (long)ws_bytes, (long)need);
    const long chunks = (tiles + FIN_CHUNK - 1) / FIN_CHUNK;
    hipStream_t st = as_stream(stream);
    const unsigned cg = (unsigned)((c + 63) / 64);
    hipLaunchKernelGGL(bn_fin_chunk_kernel, dim3(cg, (unsigned)chunks), dim3(1024), 0, st, c, (long)count,
                       (long)tiles, tile_rows, partials, (double2*)workspace);
    HKP_LAUNCH_CHECK(who);
    hipLaunchKernelGGL(bn_fin_merge_kernel, dim3(cg), dim3(1024), 0, st, c, (long)count, chunks, tile_rows,
                       (const double2*)workspace, gamma, beta, momentum, eps, running_mean, running_var,
                       num_batches_tracked, scale_shift, mean_invstd, stats);
    HKP_LAUNCH_CHECK(who);
    return HKP_OK;
}

extern "C" int hkp_bn_finalize(int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                               const float* gamma, const float* beta, float momentum, float eps, float* running_mean,
                               float* running_var, int64_t* num_batches_tracked, float* scale_shift,
                               float* mean_invstd, hkp_stream_t stream) {
    HKP_CHECK_ARG(scale_shift, "hkp_bn_finalize: null tensor");
    return fin_one("hkp_bn_finalize", c, count, tiles, tile_rows, partials, gamma, beta, momentum, eps, running_mean,
                   running_var, num_batches_tracked, scale_shift, mean_invstd, nullptr, stream);
}

extern "C" int hkp_bn_finalize_ws(int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                                  const float* gamma, const float* beta, float momentum, float eps,
                                  float* running_mean, float* running_var, int64_t* num_batches_tracked,
                                  float* scale_shift, float* mean_invstd, void* workspace, int64_t ws_bytes,
                                  hkp_stream_t stream) {
    HKP_CHECK_ARG(scale_shift, "hkp_bn_finalize_ws: null tensor");
    return fin_two("hkp_bn_finalize_ws", c, count, tiles, tile_rows, partials, gamma, beta, momentum, eps,
                   running_mean, running_var, num_batches_tracked, scale_shift, mean_invstd, nullptr, workspace,
                   ws_bytes, stream);
}

extern "C" int hkp_bn_stats(int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                            double* stats, void* workspace, int64_t ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(stats, "hkp_bn_stats: null tensor");
    if (workspace)
        return fin_two("hkp_bn_stats", c, count, tiles, tile_rows, partials, nullptr, nullptr, 0.f, 0.f, nullptr,
                       nullptr, nullptr, nullptr, nullptr, stats, workspace, ws_bytes, stream);
    return fin_one("hkp_bn_stats", c, count, tiles, tile_rows, partials, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr,
                   nullptr, nullptr, nullptr, stats, stream);
}

extern "C" int hkp_bn_finalize_ranks(int32_t c, int32_t nranks, const double* stats, const float* gamma,
                                     const float* beta, float momentum, float eps, float* running_mean,
                                     float* running_var, int64_t* num_batches_tracked, float* scale_shift,
                                     float* mean_invstd, hkp_stream_t stream) {
    HKP_CHECK_ARG(c > 0 && nranks > 0, "hkp_bn_finalize_ranks: bad sizes");
    HKP_CHECK_ARG(stats && scale_shift, "hkp_bn_finalize_ranks: null tensor");
    HKP_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr), "hkp_bn_finalize_ranks: running stats pair");
    hipLaunchKernelGGL(bn_fin_ranks_kernel, dim3((c + 255) / 256), dim3(256), 0, as_stream(stream), c, nranks, stats,
                       gamma, beta, momentum, eps, running_mean, running_var, num_batches_tracked, scale_shift,
                       mean_invstd);
    HKP_LAUNCH_CHECK("hkp_bn_finalize_ranks");
    return HKP_OK;
}

extern "C" int hkp_bn_eval_params(int32_t c, const float* gamma, const float* beta, const float* running_mean,
                                  const float* running_var, float eps, float* scale_shift, float* mean_invstd,
                                  hkp_stream_t stream) {
    HKP_CHECK_ARG(c > 0 && running_mean && running_var && scale_shift, "hkp_bn_eval_params: bad args");
    hipLaunchKernelGGL(bn_eval_kernel, dim3((c + 255) / 256), dim3(256), 0, as_stream(stream), c, gamma, beta,
                       running_mean, running_var, eps, scale_shift, mean_invstd);
    HKP_LAUNCH_CHECK("hkp_bn_eval_params");
    return HKP_OK;
}

extern "C" int hkp_bn_apply(int64_t m, int32_t c, const float* y, const float* scale_shift, const float* res,
                            const float* res_scale_shift, const uint16_t* res_split, int32_t relu, float* out,
                            uint16_t* out_split, int32_t split_passes, hkp_stream_t stream) {
    HKP_CHECK_ARG(m > 0 && c > 0 && c % 4 == 0, "hkp_bn_apply: need m>0 and c%%4==0 (c=%d)", c);
    HKP_CHECK_ARG(y && scale_shift && (out || out_split), "hkp_bn_apply: null tensor");
    HKP_CHECK_ARG(!out_split || ((split_passes == 1 || split_passes == 3) && c % 32 == 0),
                  "hkp_bn_apply: split output needs split_passes 1|3 and c%%32==0");
    HKP_CHECK_ARG(res_scale_shift == nullptr || res != nullptr, "hkp_bn_apply: res_scale_shift without res");
    HKP_CHECK_ARG(res_split == nullptr || (res == nullptr && c % 32 == 0),
                  "hkp_bn_apply: res_split excludes res and needs c%%32==0");
    const long n4 = m * (long)c / 4;
    const int C4 = c / 4;
    const f32x4 *Y = (const f32x4*)y, *SC = (const f32x4*)scale_shift, *SH = (const f32x4*)(scale_shift + c);
    const f32x4* R = (const f32x4*)res;
    const f32x4* RSC = res_scale_shift ? (const f32x4*)res_scale_shift : nullptr;
    const f32x4* RSH = res_scale_shift ? (const f32x4*)(res_scale_shift + c) : nullptr;
    f32x4* O = (f32x4*)out;
    const int g = grid_for(n4);
    hipStream_t st = as_stream(stream);
    const bool fix = ((long)g * 256) % C4 == 0;
#define HKP_APPLY(RES, RL)                                                                                         \
    if (fix)                                                                                                       \
        hipLaunchKernelGGL((bn_apply_kernel<RES, RL, true>), dim3(g), dim3(256), 0, st, n4, C4, Y, SC, SH, R, RSC, \
                           RSH, (const _Float16*)res_split, O, (_Float16*)out_split, split_passes);               \
    else                                                                                                           \
        hipLaunchKernelGGL((bn_apply_kernel<RES, RL, false>), dim3(g), dim3(256), 0, st, n4, C4, Y, SC, SH, R,     \
                           RSC, RSH, (const _Float16*)res_split, O, (_Float16*)out_split, split_passes)
    if (res_split) {
        if (relu) HKP_APPLY(3, true); else HKP_APPLY(3, false);
    } else if (!res) {
        if (relu) HKP_APPLY(0, true); else HKP_APPLY(0, false);
    } else if (!res_scale_shift) {
        if (relu) HKP_APPLY(1, true); else HKP_APPLY(1, false);
    } else {
        if (relu) HKP_APPLY(2, true); else HKP_APPLY(2, false);
    }
#undef HKP_APPLY
    HKP_LAUNCH_CHECK("hkp_bn_apply");
    return HKP_OK;
}

extern "C" int hkp_bn_relu_maxpool(int32_t n, int32_t h, int32_t w, int32_t c, const float* y,
                                   const float* scale_shift, float* out, uint16_t* out_split,
                                   int32_t split_passes, uint8_t* route, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0, "hkp_bn_relu_maxpool: bad sizes");
    HKP_CHECK_ARG(y && scale_shift && (out || out_split), "hkp_bn_relu_maxpool: null tensor");
    HKP_CHECK_ARG(!out_split || ((split_passes == 1 || split_passes == 3) && c % 32 == 0),
                  "hkp_bn_relu_maxpool: split output needs split_passes 1|3 and c%%32==0");
    const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
    const long work = (long)n * ho * wo * (c / 4);
    const bool idx32 = work * 4 < (1L << 31) && (long)n * h * w * c < (1L << 31);
    if (idx32)
        hipLaunchKernelGGL(bn_relu_maxpool_kernel<unsigned>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), n,
                           h, w, c, ho, wo, y, scale_shift, out, (_Float16*)out_split, split_passes, (uchar4*)route);
    else
        hipLaunchKernelGGL(bn_relu_maxpool_kernel<long>, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), n, h,
                           w, c, ho, wo, y, scale_shift, out, (_Float16*)out_split, split_passes, (uchar4*)route);
    HKP_LAUNCH_CHECK("hkp_bn_relu_maxpool");
    return HKP_OK;
}

extern "C" int hkp_bn_apply_f16(int64_t m, int32_t c, const uint16_t* y, const float* scale_shift, const uint16_t* res,
                                const float* res_scale_shift, int32_t relu, uint16_t* out, float* out32,
                                hkp_stream_t stream) {
    HKP_CHECK_ARG(m > 0 && c > 0 && c % 8 == 0, "hkp_bn_apply_f16: need m>0 and c%%8==0 (c=%d)", c);
    HKP_CHECK_ARG(y && scale_shift && out, "hkp_bn_apply_f16: null tensor");
    HKP_CHECK_ARG(res_scale_shift == nullptr || res != nullptr, "hkp_bn_apply_f16: res_scale_shift without res");
    const long n8 = m * (long)c / 8;
    // two 4-wave blocks per CU, streaming loads/stores: the fp16 tensors here
    // (0.3-2.5 GB at C4) stream through once; 16 blocks per CU and cached
    // accesses ran 5.0-5.1 TB/s vs 6.1 on the same 2-read-1-write stream
    // (tools/apply_bw.hip), C4 +3.5 % end to end
    const int g = grid_for(n8, 256, 512);
    hipStream_t st = as_stream(stream);
    const h16x8 *Y = (const h16x8*)y, *R = (const h16x8*)res;
    h16x8* O = (h16x8*)out;
    const bool fix = ((long)g * 256) % (c / 8) == 0;
#define HKP_APPLY16(RES, RL)                                                                                       \
    if (fix)                                                                                                       \
        hipLaunchKernelGGL((bn_apply_f16_kernel<RES, RL, true>), dim3(g), dim3(256), 0, st, n8, c / 8, Y,          \
                           scale_shift, R, res_scale_shift, O, (f32x4*)out32);                                     \
    else                                                                                                           \
        hipLaunchKernelGGL((bn_apply_f16_kernel<RES, RL, false>), dim3(g), dim3(256), 0, st, n8, c / 8, Y,         \
                           scale_shift, R, res_scale_shift, O, (f32x4*)out32)
    if (!res) {
        if (relu) HKP_APPLY16(0, true); else HKP_APPLY16(0, false);
    } else if (!res_scale_shift) {
        if (relu) HKP_APPLY16(1, true); else HKP_APPLY16(1, false);
    } else {
        if (relu) HKP_APPLY16(2, true); else HKP_APPLY16(2, false);
    }
#undef HKP_APPLY16
    HKP_LAUNCH_CHECK("hkp_bn_apply_f16");
    return HKP_OK;
}
