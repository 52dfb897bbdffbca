// BatchNorm statistics of a 1x1 conv's output from the second moments of its
// input (BASELINE config C4: R50-8s inference, plain fp16).
//
// For y = W a (a 1x1 conv, no padding, over M pixels) the batch statistics of
// output channel k are exact linear-algebra functions of the input's mean mu and
// covariance Sigma:
//     mean_k = w_k . mu,      var_k = w_k^T Sigma w_k
// so train-mode BN (src/resnet.py:85-87,106-108: bn3 of every Bottleneck) needs
// no pass over y.  Its scale/shift is known BEFORE the conv runs, and the conv
// epilogue applies bn3 + residual + ReLU itself (hkp_conv2d_fwd_f16_bn): the
// fp16 y3 (4*planes wide) is never written nor re-read by a separate apply pass.
// The Gram matrix costs Cin^2/2 MACs per pixel against the conv's Cin*Cout —
// 1/8 of an expanding conv3's (Cout = 4 Cin).
//
//   gram_f16_kernel<TC>   G partials: row splits x upper-triangle TC x TC channel
//                         tiles; both MFMA operands read TRANSPOSED
//                         (ds_read_b64_tr_b16) from one row-major LDS image filled
//                         by LDS-DMA; column sums by one extra MFMA against ones
//   gram_reduce_kernel    mu and the second moments E = a^T a / M: the row splits
//                         summed in fp64 in fixed order
//   bn_from_gram_kernel   per output channel: mean = w.mu, var = w^T E w - mean^2
//                         (fp64) -> bn_fin_store
//                         (the same scale/shift/running-stat formulas as
//                         hkp_bn_finalize)
// Deterministic: every reduction is in a fixed order.
#include "common.h"

namespace hkp {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __attribute__((aligned(256))) uint4 g_gram_zero_line[8];   // 128 B of zeros

struct GramArgs {
    const _Float16* a;   // [M][C] fp16
    float* part;         // [splits][tiles][TC*TC] fp32, accumulator order
    float* psum;         // [splits][nb][TC] fp32 column sums (diagonal tiles)
    long M;
    int C, nb, tiles, splits;
    long rows;           // rows per split (a multiple of 32)
};

__device__ __forceinline__ void gram_glds16(const void* src, char* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <int OFF>
__device__ __forceinline__ s16x4 gram_tr16(unsigned lds_addr) {
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(lds_addr), "i"(OFF));
    return r;
}

__device__ __forceinline__ f16x8 gram_cat(s16x4 lo, s16x4 hi) {
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// upper-triangle tile t -> (ib, jb), ib <= jb
__device__ __forceinline__ void gram_tile(int t, int nb, int* ib, int* jb) {
    int i = 0;
    while (t >= nb - i) {
        t -= nb - i;
        ++i;
    }
    *ib = i;
    *jb = i + t;
}

// Staged row (32 rows per K-step): TC channels of block ib, then TC of block jb,
// fp16, 16-B chunk P of row r holding logical chunk P ^ f(r),
// f(r) = 2 * ((r & 3) | ((r >> 3 & 1) << 2)): the two 16-lane groups of a
// transposed read's 32-lane half touch rows {8g..8g+3} u {8g+8..8g+11} (or the
// +4 rows), eight distinct f, so their eight 8-B pieces of a chunk pair land in
// eight distinct 8-bank groups: conflict-free.
template <int TC>
__global__ __launch_bounds__(256, 2) void gram_f16_kernel(GramArgs g) {
    constexpr int ROWB = 2 * TC * 2;       // bytes per staged row
    constexpr int CPR = ROWB / 16;         // 16-B chunks per row
    constexpr int RPI = 1024 / ROWB;       // rows per DMA wave-instruction
    constexpr int KR = 32;                 // rows per K-step
    constexpr int STAGE = KR * ROWB;
    constexpr int NST = 4;
    constexpr int GL = KR / RPI / 4;       // DMA instructions per wave per stage
    constexpr int WT = TC / 2;             // wave tile (2 x 2 waves)
    constexpr int UT = WT / 16;            // 16x16 sub-tiles per wave dimension
    __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];

    const int b = xcd_remap(blockIdx.x, gridDim.x);          // a split's tiles on one XCD
    const int s = b / g.tiles, t = b - s * g.tiles;
    int ib, jb;
    gram_tile(t, g.nb, &ib, &jb);
    const bool diag = ib == jb;
    const long r_begin = (long)s * g.rows;
    const long r_end = min(g.M, r_begin + g.rows);
    const int nsteps = r_end > r_begin ? (int)((r_end - r_begin + KR - 1) / KR) : 0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 1, wn = w & 1;

    // ---- DMA sources: instruction i of this wave fills rows RPI*(w*GL+i) .. +RPI-1 ----
    const _Float16* src[GL];
    int srow[GL];
#pragma unroll
    for (int i = 0; i < GL; ++i) {
        const int r = RPI * (w * GL + i) + lane / CPR;
        const int P = lane % CPR;
        const int f = 2 * ((r & 3) | (((r >> 3) & 1) << 2));
        const int L = P ^ f;
        const int ch = L < TC / 8 ? ib * TC + 8 * L : jb * TC + 8 * (L - TC / 8);
        srow[i] = r;
        src[i] = g.a + (r_begin + r) * g.C + ch;
    }
    const _Float16* zero = (const _Float16*)g_gram_zero_line;
    auto issue = [&](int step) {
        char* st = smem + (step & (NST - 1)) * STAGE;
        const long rb = r_begin + (long)KR * step;
#pragma unroll
        for (int i = 0; i < GL; ++i) {
            const bool in = rb + srow[i] < r_end;
            gram_glds16(in ? (const void*)(src[i] + (long)KR * step * g.C) : (const void*)zero,
                        st + RPI * (w * GL + i) * ROWB);
        }
    };

    // ---- transposed fragment reads: lane 4q+p of 16-lane group gq supplies row
    // 8gq+q (second read: +4 rows), channels c0+4p..+3 of the sub-tile ----
    const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int r0 = 8 * gq + q;
    const int f0 = 2 * ((r0 & 3) | (((r0 >> 3) & 1) << 2));
    const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)smem;
    unsigned aoff[UT], boff[UT];
#pragma unroll
    for (int u = 0; u < UT; ++u) {
        const int ca = wm * WT + 16 * u, cb = TC + wn * WT + 16 * u;     // logical channel columns in the row
        aoff[u] = lds0 + r0 * ROWB + 16 * (((ca >> 3) + (p >> 1)) ^ f0) + 8 * (p & 1);
        boff[u] = lds0 + r0 * ROWB + 16 * (((cb >> 3) + (p >> 1)) ^ f0) + 8 * (p & 1);
    }

    f32x4 acc[UT][UT];
    f32x4 accs[UT];
#pragma unroll
    for (int i = 0; i < UT; ++i) {
        accs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < UT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const bool sums = diag && wn == 0;                    // wave-uniform
    f16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (_Float16)1.0f;

    if (nsteps > 0) {
#pragma unroll
        for (int u = 0; u < NST - 1; ++u) issue(u);
        for (int step = 0; step < nsteps; ++step) {
            // this wave's DMA of `step` landed (NST-2 younger stages may stay in flight)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * GL) : "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const unsigned so = (unsigned)((step & (NST - 1)) * STAGE);
            f16x8 fa[UT], fb[UT];
#pragma unroll
            for (int u = 0; u < UT; ++u) {
                fa[u] = gram_cat(gram_tr16<0>(aoff[u] + so), gram_tr16<4 * ROWB>(aoff[u] + so));
                fb[u] = gram_cat(gram_tr16<0>(boff[u] + so), gram_tr16<4 * ROWB>(boff[u] + so));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // stage step+NST-1 goes into the buffer stage step-1 used: every wave
            // finished reading it before this step's barrier
            issue(step + NST - 1);
#pragma unroll
            for (int i = 0; i < UT; ++i)
#pragma unroll
                for (int j = 0; j < UT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            if (sums) {
#pragma unroll
                for (int i = 0; i < UT; ++i)
                    accs[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], ones, accs[i], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // the trailing (zero) DMAs
    }

    // ---- partials: accumulator order [s][t][w][i][j][lane][4] (f32x4 stores) ----
    f32x4* out = (f32x4*)g.part + ((long)(s * g.tiles + t) * 4 + w) * (UT * UT * 64);
#pragma unroll
    for (int i = 0; i < UT; ++i)
#pragma unroll
        for (int j = 0; j < UT; ++j) out[(i * UT + j) * 64 + lane] = acc[i][j];
    if (sums && (lane & 15) == 0) {
        float* ps = g.psum + ((long)s * g.nb + ib) * TC + wm * WT + 4 * gq;
#pragma unroll
        for (int i = 0; i < UT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) ps[16 * i + r] = accs[i][r];
    }
}

// One launch reduces the row splits (fp64, fixed split order; loads batched 8 at a
// time): blocks [0, nel/256) the Gram elements — E[i][j] = E[j][i] = sum / M in
// accumulator order of an upper-triangle tile — and the blocks after them the
// column sums, mu[c] = sum / M.  Centring (Sigma = E - mu mu^T) happens in fp64
// where the quadratic forms are taken (bn_from_gram_kernel).
// SG split groups per value: a block is 256/SG consecutive values (coalesced
// loads of each split's slab) x SG groups of the splits, each group summing
// its contiguous split range in order (8 loads in flight), the SG group sums
// added in group order through LDS — fixed order.  SG = 4 for many splits (R50
// layer1's 512 split sums by one thread each were latency-bound at 26 us).
template <int SG>
__global__ __launch_bounds__(256) void gram_reduce_kernel(int C, int TC, int tiles, int splits, long M,
                                                          const float* part, const float* psum, double* mu,
                                                          double* e2) {
    constexpr int NV = 256 / SG;                           // values per block
    __shared__ double red[SG][NV];
    const long per = (long)TC * TC, nel = per * tiles;
    const int v = threadIdx.x % NV, g = threadIdx.x / NV;
    const long gid = (long)blockIdx.x * NV + v;
    const double inv = 1.0 / (double)M;
    const int k_lo = (int)((long)splits * g / SG), k_hi = (int)((long)splits * (g + 1) / SG);
    auto split_sum = [&](const float* p, long st) -> double {
        double s = 0.0;
        int k = k_lo;
        for (; k + 8 <= k_hi; k += 8) {
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = p[(long)(k + u) * st];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)x[u];
        }
        for (; k < k_hi; ++k) s += (double)p[(long)k * st];
        return s;
    };
    // value gid: a second moment (gid < nel) or a column sum (the means)
    const bool is_e = gid < nel, live = gid < nel + C;
    double s = 0.0;
    int ci = 0, cj = 0;
    if (is_e) {
        const int t = (int)(gid / per), x = (int)(gid - (long)t * per);
        // x = ((w * UT + i) * UT + j) * 256 + lane * 4 + r   (UT = TC / 32)
        const int UT = TC / 32;
        const int r = x & 3, fl = (x >> 2) & 63, ij = x >> 8;
        const int j = ij % UT, i = (ij / UT) % UT, w = ij / (UT * UT);
        const int wm = w >> 1, wn = w & 1, WT = TC / 2;
        int ib, jb;
        gram_tile(t, C / TC, &ib, &jb);
        ci = ib * TC + wm * WT + 16 * i + 4 * (fl >> 4) + r;
        cj = jb * TC + wn * WT + 16 * j + (fl & 15);
        s = split_sum(part + (long)t * per + x, (long)tiles * per);
    } else if (live) {
        const long c = gid - nel;
        const int nb = C / TC, ib = (int)(c / TC), cc = (int)(c - (long)ib * TC);
        s = split_sum(psum + (long)ib * TC + cc, (long)nb * TC);
    }
    if constexpr (SG > 1) {
        red[g][v] = s;
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int q = 1; q < SG; ++q) s += red[q][v];
    }
    if (!live) return;
    if (is_e) {
        const double val = s * inv;
        e2[(long)ci * C + cj] = val;
        e2[(long)cj * C + ci] = val;
    } else {
        mu[gid - nel] = s * inv;
    }
}

// Per output channel k of y = W a: mean = w_k . mu and
// var = w_k^T E w_k - mean^2 (E = the raw second moments; fp64 throughout — the
// centring loses only log10(1 + mean^2/var) of fp64's digits), with w_k = the
// fp16 packed weight row x its inverse scale (the weights the conv multiplies
// with; exact in fp32: an fp16 value times a power of two).  Two launches:
//   bn_from_gram_part_kernel  grid (K/16 channel groups) x (C/256 column blocks)
//                             x (C/64 row groups): thread j of a block sums, for
//                             its 16 channels, s_k = sum_{i in the 64 rows}
//                             E[i][j] w_k[i] (coalesced rows of E, 8 in flight,
//                             the next 8 loading while these are used; weight
//                             rows / columns in LDS, read as broadcasts), and
//                             the block sums q_k = sum_j s_k w_k[j] (and, in row
//                             group 0, m_k = sum_j mu_j w_k[j]) over its 256
//                             columns in fixed order (wave shuffles, then the 4
//                             waves in order) → part[jb][rg][k]
//   bn_from_gram_fin_kernel   per k: the partials in (jb, rg) order → mean, var
//                             → bn_fin_store
// (One block per 16 channels over all of E: a thread walked C rows in
// dependent rounds of 8 loads with one wave per SIMD — latency-bound, 158 us
// for R50's layer4; with the rows split over blocks the chip holds 8x the loads
// in flight.)
constexpr int BFG_KB = 16, BFG_JB = 256, BFG_RB = 64;

// Sum of v[0..KP) over a wave's 64 lanes, reduce-scatter form: at offsets 32,
// 16, ... each lane keeps half of its values plus its partner's copy of that
// half until one is left, then the remaining offsets fold it — KP-1 +
// log2(64/KP) fp64 shuffles instead of 6 per value.  Fixed order.
template <int KP>
__device__ __forceinline__ double bfg_reduce_scatter(double (&v)[KP], int lane) {
    int o = 32;
#pragma unroll
    for (int n = KP; n > 1; n >>= 1, o >>= 1) {
        const int half = n >> 1;
        const bool upper = (lane & o) != 0;
#pragma unroll
        for (int i = 0; i < half; ++i) {
            const double send = upper ? v[i] : v[half + i];
            const double keep = upper ? v[half + i] : v[i];
            v[i] = keep + __shfl_xor(send, o);
        }
    }
    double s = v[0];
#pragma unroll
    for (; o > 0; o >>= 1) s += __shfl_xor(s, o);
    return s;
}
template <int KP>
__device__ __forceinline__ int bfg_rs_k(int lane) {
    int k = 0, o = 32;
#pragma unroll
    for (int n = KP; n > 1; n >>= 1, o >>= 1) k += (lane & o) ? (n >> 1) : 0;
    return k;
}

__global__ __launch_bounds__(256) void bn_from_gram_part_kernel(int K, int C, const double* __restrict__ mu,
                                                                const double* __restrict__ e2,
                                                                const _Float16* __restrict__ w16,
                                                                const float* __restrict__ w_inv_scale,
                                                                double* __restrict__ part) {
    constexpr int KB = BFG_KB, JB = BFG_JB, RB = BFG_RB;
    __shared__ __attribute__((aligned(16))) double wr[RB][KB];   // weights of this block's rows i (fp64:
                                                                 // no conversion in the FMA loop)
    __shared__ float wc[JB][KB];                                 // weights of this block's columns j
    __shared__ double red[4][KB][2];
    const int k0 = blockIdx.x * KB, jb = blockIdx.y, rg = blockIdx.z;
    const int i_base = rg * RB, j_base = jb * JB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j = j_base + tid;
    const bool valid = j < C;
    // the first rows of E and every weight this block needs, all in flight at
    // once (the kernel is latency-bound: a few dependent rounds in all)
    constexpr int RR = 8;                                  // rows of E per round
    double ev[RR], en[RR];
#pragma unroll
    for (int di = 0; di < RR; ++di) ev[di] = valid ? e2[(long)(i_base + di) * C + j] : 0.0;
    {
        float vr[KB], vc[KB], sc[KB];
        const int i = i_base + (tid & (RB - 1));
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {                  // coalesced along each weight row
            const int k = k0 + kk;
            sc[kk] = k < K ? w_inv_scale[k] : 0.f;
            vr[kk] = k < K ? (float)w16[(long)k * C + i] : 0.f;
            vc[kk] = (k < K && valid) ? (float)w16[(long)k * C + j] : 0.f;
        }
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
            if (tid < RB) wr[tid][kk] = (double)(vr[kk] * sc[kk]);
            wc[tid][kk] = vc[kk] * sc[kk];
        }
    }
    __syncthreads();
    double s[KB];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) s[kk] = 0.0;
#pragma unroll 1
    for (int r0 = 0; r0 < RB; r0 += RR) {
        if (r0 + RR < RB) {
#pragma unroll
            for (int di = 0; di < RR; ++di) en[di] = valid ? e2[(long)(i_base + r0 + RR + di) * C + j] : 0.0;
        }
#pragma unroll
        for (int di = 0; di < RR; ++di) {
            const double2* wi = (const double2*)&wr[r0 + di][0];
#pragma unroll
            for (int q2 = 0; q2 < KB / 2; ++q2) {
                const double2 w2 = wi[q2];
                s[2 * q2 + 0] += ev[di] * w2.x;
                s[2 * q2 + 1] += ev[di] * w2.y;
            }
        }
        if (r0 + RR < RB) {
#pragma unroll
            for (int di = 0; di < RR; ++di) ev[di] = en[di];
        }
    }
    const double muj = valid && rg == 0 ? mu[j] : 0.0;
    double v[KB], u[KB];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
        const double wj = valid ? (double)wc[tid][kk] : 0.0;
        v[kk] = s[kk] * wj;
        u[kk] = muj * wj;
    }
    // the wave's 64 lanes summed for all KB channels at once (reduce-scatter:
    // 17 shuffles instead of 6 per channel, in a fixed order); lane l holds the
    // total of channel bfg_rs_k(l)
    const double vs = bfg_reduce_scatter<KB>(v, lane);
    const double us = rg == 0 ? bfg_reduce_scatter<KB>(u, lane) : 0.0;     // the mean term: row group 0 only
    if ((lane & (64 / KB - 1)) == 0) {
        const int kk = bfg_rs_k<KB>(lane);
        red[w][kk][0] = vs;
        red[w][kk][1] = us;
    }
    __syncthreads();
    if (tid < KB && k0 + tid < K) {
        double v = 0.0, m = 0.0;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
            v += red[ww][tid][0];
            m += red[ww][tid][1];
        }
        const long slot = (long)jb * gridDim.z + rg;
        part[(slot * K + k0 + tid) * 2 + 0] = v;
        part[(slot * K + k0 + tid) * 2 + 1] = m;
    }
}

__global__ __launch_bounds__(256) void bn_from_gram_fin_kernel(int K, int nslots, long count,
                                                               const double* __restrict__ part, const float* gamma,
                                                               const float* beta, float momentum, float eps,
                                                               float* rmean, float* rvar, int64_t* nbt, float* ss,
                                                               float* mi) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    double v = 0.0, mean = 0.0;
    for (int sl = 0; sl < nslots; ++sl) {
        v += part[((long)sl * K + k) * 2 + 0];
        mean += part[((long)sl * K + k) * 2 + 1];
    }
    double var = v - mean * mean;
    var = var > 0.0 ? var : 0.0;
    bn_fin_store(k, K, count, mean, var * (double)count, gamma, beta, momentum, eps, rmean, rvar, nbt, ss, mi);
}

static int gram_tc(int c) { return c % 128 == 0 ? 128 : 64; }

// rows per split: about two blocks per CU over all tiles, >= 32 rows, <= 16k rows
// (fp32 accumulation inside a split; fp64 across splits)
static void gram_plan(long m, int c, int* tc, int* tiles, int* splits, long* rows) {
    *tc = gram_tc(c);
    const int nb = c / *tc;
    *tiles = nb * (nb + 1) / 2;
    long sp = std::max<long>(1, 512 / *tiles);
    long r = (m + sp - 1) / sp;
    if (r > 16384) r = 16384;
    r = (r + 31) / 32 * 32;
    *rows = r;
    *splits = (int)((m + r - 1) / r);
}

}  // namespace hkp

using namespace hkp;

extern "C" int64_t hkp_gram_f16_workspace_bytes(int64_t m, int32_t c) {
    if (m <= 0 || c <= 0 || c % 64) return -1;
    int tc, tiles, splits;
    long rows;
    gram_plan(m, c, &tc, &tiles, &splits, &rows);
    return (int64_t)splits * tiles * tc * tc * 4 + (int64_t)splits * (c / tc) * tc * 4 + 256;
}

extern "C" int hkp_gram_f16(int64_t m, int32_t c, const uint16_t* a, double* mean, double* second, void* ws,
                            int64_t ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(m > 0 && m < (1L << 40) && c > 0 && c % 64 == 0 && c <= 2048 && a && mean && second && ws,
                  "hkp_gram_f16: bad args (m=%lld c=%d)", (long long)m, c);
    HKP_CHECK_ARG(ws_bytes >= hkp_gram_f16_workspace_bytes(m, c), "hkp_gram_f16: workspace too small");
    int tc, tiles, splits;
    long rows;
    gram_plan(m, c, &tc, &tiles, &splits, &rows);
    GramArgs g;
    g.a = (const _Float16*)a;
    g.part = (float*)ws;
    g.psum = (float*)ws + (long)splits * tiles * tc * tc;
    g.M = m;
    g.C = c;
    g.nb = c / tc;
    g.tiles = tiles;
    g.splits = splits;
    g.rows = rows;
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)(splits * tiles));
    if (tc == 128) hipLaunchKernelGGL(gram_f16_kernel<128>, grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL(gram_f16_kernel<64>, grid, dim3(256), 0, st, g);
    const long nval = (long)tiles * tc * tc + c;          // second moments, then the means
    if (splits >= 64)
        hipLaunchKernelGGL(gram_reduce_kernel<4>, dim3((unsigned)((nval + 63) / 64)), dim3(256), 0, st, c, tc, tiles,
                           splits, (long)m, (const float*)g.part, (const float*)g.psum, mean, second);
    else
        hipLaunchKernelGGL(gram_reduce_kernel<1>, dim3((unsigned)((nval + 255) / 256)), dim3(256), 0, st, c, tc,
                           tiles, splits, (long)m, (const float*)g.part, (const float*)g.psum, mean, second);
    HKP_LAUNCH_CHECK("hkp_gram_f16");
    return HKP_OK;
}

static int bfg_slots(int c) { return ((c + BFG_JB - 1) / BFG_JB) * (c / BFG_RB); }

extern "C" int64_t hkp_bn_from_gram_workspace_bytes(int32_t k, int32_t c) {
    if (k <= 0 || c <= 0 || c % 64) return -1;
    return (int64_t)bfg_slots(c) * k * 2 * (int64_t)sizeof(double);
}

extern "C" int hkp_bn_from_gram(int32_t k, int32_t c, int64_t count, const double* mean, const double* second,
                                const uint16_t* w_f16, const float* w_inv_scale, const float* gamma,
                                const float* beta, float momentum, float eps, float* running_mean,
                                float* running_var, int64_t* num_batches_tracked, float* scale_shift,
                                float* mean_invstd, void* workspace, int64_t ws_bytes, hkp_stream_t stream) {
    HKP_CHECK_ARG(k > 0 && c > 0 && c <= 2048 && c % 64 == 0 && count > 0 && mean && second && w_f16 && w_inv_scale &&
                      scale_shift && workspace,
                  "hkp_bn_from_gram: bad args");
    HKP_CHECK_ARG(ws_bytes >= hkp_bn_from_gram_workspace_bytes(k, c), "hkp_bn_from_gram: workspace %lld < %lld",
                  (long long)ws_bytes, (long long)hkp_bn_from_gram_workspace_bytes(k, c));
    hipStream_t st = as_stream(stream);
    const int njb = (c + BFG_JB - 1) / BFG_JB, nrg = c / BFG_RB;
    hipLaunchKernelGGL(bn_from_gram_part_kernel,
                       dim3((unsigned)((k + BFG_KB - 1) / BFG_KB), (unsigned)njb, (unsigned)nrg), dim3(256), 0, st,
                       k, c, mean, second, (const _Float16*)w_f16, w_inv_scale, (double*)workspace);
    hipLaunchKernelGGL(bn_from_gram_fin_kernel, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, st, k, njb * nrg,
                       (long)count, (const double*)workspace, gamma, beta, momentum, eps, running_mean, running_var,
                       num_batches_tracked, scale_shift, mean_invstd);
    HKP_LAUNCH_CHECK("hkp_bn_from_gram");
    return HKP_OK;
}
