// Implicit-GEMM convolution forward on fp16 MFMA (v_mfma_f32_32x32x16_f16),
// in two precisions selected by PASSES:
//
//   PASSES = 3  "f16x3": fp32-accurate.  Every fp32 operand is split as
//               hi = f16(x), lo = f16((x - hi) * 2^11), and
//               x*w ≈ hi_x*hi_w + 2^-11 (hi_x*lo_w + lo_x*hi_w)
//               (dropped lo*lo term and lo's own rounding: ~2^-22 relative per
//               product, ~4x fp32's unit roundoff).  hi*hi accumulates in one
//               fp32 MFMA accumulator set, the two cross terms in a second; the
//               epilogue adds them.  3 fp16 MFMAs = 3/16 the cycles of the one
//               fp32 MFMA they replace.
//   PASSES = 1  plain fp16 operands, fp32 accumulation (BASELINE config C4).
//
// Activations stay fp32 NHWC in HBM and are split while staging into LDS;
// weights are pre-split once (hkp_weight_split).  Tile 128 x BN x 32 (one filter
// tap x 32 channels per K-chunk), 4 waves as 2x2, LDS double-buffered, rows
// padded to 80 B (conflict-free ds_read_b128), one barrier per chunk, XCD-aware
// tile order.  Epilogue = conv_fwd.hip's (NHWC store + BN tile partials).
//
// Replaces the same cuDNN convs as conv_fwd.hip (src/resnet.py:20-37,77,86,184-188).
#include "common.h"

namespace hkp {

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct SplitArgs {
    const float* x;
    const _Float16* xhi;   // optional pre-converted fp16 input plane (APL path, passes 1)
    const _Float16* whi;
    const _Float16* wlo;
    float* y;
    float* part;
    const unsigned* amax;  // optional: bit pattern of max|x| → x is scaled by a power of two into fp16 range
    const float* add;      // optional addend of the output (dgrad: the residual-branch gradient)
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M, Kreal, nkc, cchunks, n_tiles;
};

constexpr int SBK = 32;         // K chunk (channels of one tap)
constexpr int SLDR = SBK + 8;   // LDS row stride in halves (80 B)
constexpr float LO_SCALE = 2048.f;
constexpr float LO_INV = 1.f / 2048.f;

// APL (PASSES 1): the input arrives as a pre-converted fp16 plane (written by its producer), so
// the A tile is staged exactly like the weight tile — no conversion in the loop.
template <int BM, int BN, int PASSES, bool APL>
__global__ __launch_bounds__(256, 2) void conv_split_kernel(SplitArgs a) {
    constexpr int NT = 256, WM = 2, WN = 2;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    constexpr int PL = PASSES == 3 ? 2 : 1;          // planes (hi[, lo])
    constexpr int AP = APL ? BM * (SBK / 8) / NT     // f16x8 A loads per thread per plane
                           : BM * (SBK / 4) / NT;    // f32x4 A loads per thread
    constexpr int BP = BN * (SBK / 8) / NT;          // f16x8 B loads per thread per plane
    constexpr int STAGE = PL * (BM + BN) * SLDR;     // halves per stage
    __shared__ __attribute__((aligned(16))) _Float16 smem[2 * STAGE];

    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int col4 = tid & 7, rowb = tid >> 3;   // A: 8 threads x f32x4 per row
    const float asc = pow2_scale_for(a.amax);    // exact power of two (1 when no amax)
    const int c8 = tid & 3, browb = tid >> 2;    // B: 4 threads x f16x8 per row

    int a_n[AP], a_hi[AP], a_wi[AP];
#pragma unroll
    for (int i = 0; i < AP; ++i) {
        const int m = m0 + (APL ? browb + 64 * i : rowb + 32 * i);
        if (m < a.M) {
            const int hw = a.Ho * a.Wo;
            const int n = m / hw, rem = m - n * hw;
            const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
            a_n[i] = n;
            a_hi[i] = ho * a.stride - a.pad;
            a_wi[i] = wo * a.stride - a.pad;
        } else {
            a_n[i] = 0;
            a_hi[i] = -(1 << 28);
            a_wi[i] = -(1 << 28);
        }
    }

    f32x4 ra[APL ? 1 : AP];
    f16x8 rah[APL ? AP : 1];
    static_assert(!APL || PASSES == 1, "pre-split f16x3 input goes through conv_x3.hip");
    f16x8 rbh[BP], rbl[BP];

    auto load_chunk = [&](int kc) {
        const int cg = kc / (a.R * a.S);                 // channel-group-major K order (L2 reuse,
        const int tap = kc - cg * (a.R * a.S);           // as conv_x3.hip)
        const int c0 = cg * SBK;
        const int rr = tap / a.S, ss = tap - rr * a.S;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int hi = a_hi[i] + rr * a.dil, wi = a_wi[i] + ss * a.dil;
            const bool in = (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
            const long pix = ((long)a_n[i] * a.H + hi) * a.W + wi;
            if constexpr (APL) {
                const f16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
                rah[i] = in ? *(const f16x8*)(a.xhi + pix * a.C + c0 + c8 * 8) : z;
            } else {
                ra[i] = in ? *(const f32x4*)(a.x + pix * a.C + c0 + col4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            const long off = (long)(n0 + browb + 64 * i) * a.Kreal + tap * a.C + c0 + c8 * 8;
            rbh[i] = *(const f16x8*)(a.whi + off);
            if constexpr (PASSES == 3) rbl[i] = *(const f16x8*)(a.wlo + off);
        }
    };
    auto store_chunk = [&](int buf) {
        _Float16* st = smem + buf * STAGE;
        _Float16* Ah = st;
        _Float16* Bh = st + BM * SLDR;
        _Float16* Al = st + (BM + BN) * SLDR;
        _Float16* Bl = Al + BM * SLDR;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            if constexpr (APL) {
                const int off = (browb + 64 * i) * SLDR + c8 * 8;
                *(f16x8*)(Ah + off) = rah[i];
            } else {
                f16x4 h, l;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = ra[i][e] * asc;
                    const _Float16 hv = (_Float16)v;
                    h[e] = hv;
                    if constexpr (PASSES == 3) l[e] = (_Float16)((v - (float)hv) * LO_SCALE);
                }
                const int off = (rowb + 32 * i) * SLDR + col4 * 4;
                *(f16x4*)(Ah + off) = h;
                if constexpr (PASSES == 3) *(f16x4*)(Al + off) = l;
            }
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            const int off = (browb + 64 * i) * SLDR + c8 * 8;
            *(f16x8*)(Bh + off) = rbh[i];
            if constexpr (PASSES == 3) *(f16x8*)(Bl + off) = rbl[i];
        }
    };

    f32x16 acc[TM][TN], accc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][j][r] = 0.f;
                accc[i][j][r] = 0.f;
            }

    load_chunk(0);
    store_chunk(0);
    __syncthreads();

    const int frow = lane & 31, fk = (lane >> 5) * 8;
    for (int kc = 0; kc < a.nkc; ++kc) {
        const int cur = kc & 1;
        const bool more = kc + 1 < a.nkc;
        if (more) load_chunk(kc + 1);
        const _Float16* st = smem + cur * STAGE;
        const _Float16* Ah = st + (wm * TM * 32 + frow) * SLDR + fk;
        const _Float16* Bh = st + BM * SLDR + (wn * TN * 32 + frow) * SLDR + fk;
        const _Float16* Al = Ah + (BM + BN) * SLDR;
        const _Float16* Bl = Bh + (BM + BN) * SLDR;
#pragma unroll
        for (int s = 0; s < SBK / 16; ++s) {
            f16x8 ah[TM], bh[TN], al[TM], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                ah[i] = *(const f16x8*)(Ah + i * 32 * SLDR + s * 16);
                if constexpr (PASSES == 3) al[i] = *(const f16x8*)(Al + i * 32 * SLDR + s * 16);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                bh[j] = *(const f16x8*)(Bh + j * 32 * SLDR + s * 16);
                if constexpr (PASSES == 3) bl[j] = *(const f16x8*)(Bl + j * 32 * SLDR + s * 16);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    if constexpr (PASSES == 3) {
                        accc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], accc[i][j], 0, 0, 0);
                        accc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], accc[i][j], 0, 0, 0);
                    }
                }
        }
        if (more) store_chunk(cur ^ 1);
        __syncthreads();
    }
    if constexpr (PASSES == 3) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] += accc[i][j][r] * LO_INV;
    }
    if (a.amax) {
        const float inv = 1.f / asc;   // exact (power of two)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] *= inv;
    }

    // ---- epilogue (as conv_fwd.hip): NHWC store + BN tile partials ----
    const int rbase = m0 + wm * TM * 32 + 4 * (lane >> 5);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                if (m < a.M) {
                    const long off = (long)m * a.K + n;
                    a.y[off] = a.add ? acc[i][j][r] + a.add[off] : acc[i][j][r];
                }
            }
        }
    if (a.part == nullptr) return;
    float* red = (float*)smem;   // [WM][BN] floats, then [BN] tile means
    float* tmean = red + WM * BN;
    const int cnt = min(BM, a.M - m0);
    float colsum[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                s += (m < a.M) ? acc[i][j][r] : 0.f;
            }
        s += __shfl_xor(s, 32);
        colsum[j] = s;
    }
    if (lane < 32) {
#pragma unroll
        for (int j = 0; j < TN; ++j) red[wm * BN + wn * TN * 32 + j * 32 + lane] = colsum[j];
    }
    __syncthreads();
    if (tid < BN) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) s += red[w * BN + tid];
        tmean[tid] = s / (float)cnt;
        a.part[((long)mt * a.K + n0 + tid) * 2 + 0] = s;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const float mu = tmean[wn * TN * 32 + j * 32 + (lane & 31)];
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                const float d = acc[i][j][r] - mu;
                q += (m < a.M) ? d * d : 0.f;
            }
        q += __shfl_xor(q, 32);
        colsum[j] = q;
    }
    __syncthreads();
    if (lane < 32) {
#pragma unroll
        for (int j = 0; j < TN; ++j) red[wm * BN + wn * TN * 32 + j * 32 + lane] = colsum[j];
    }
    __syncthreads();
    if (tid < BN) {
        float q = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) q += red[w * BN + tid];
        a.part[((long)mt * a.K + n0 + tid) * 2 + 1] = q;
    }
}

__global__ __launch_bounds__(256) void weight_split_kernel(long n, const float* __restrict__ w,
                                                          _Float16* __restrict__ hi, _Float16* __restrict__ lo) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float v = w[i];
        const _Float16 h = (_Float16)v;
        hi[i] = h;
        if (lo) lo[i] = (_Float16)((v - (float)h) * LO_SCALE);
    }
}

// flipped + split dgrad weight: hi/lo[c][r'][s'][k] from w[k][R-1-r'][S-1-s'][c]
__global__ __launch_bounds__(256) void weight_flip_split_kernel(int K, int R, int S, int C, const float* __restrict__ w,
                                                               _Float16* __restrict__ hi, _Float16* __restrict__ lo) {
    const long total = (long)K * R * S * C;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int k = (int)(i % K);
        long t = i / K;
        const int sp = (int)(t % S);
        t /= S;
        const int rp = (int)(t % R);
        const int c = (int)(t / R);
        const float v = w[(((long)k * R + (R - 1 - rp)) * S + (S - 1 - sp)) * C + c];
        const _Float16 h = (_Float16)v;
        hi[i] = h;
        if (lo) lo[i] = (_Float16)((v - (float)h) * LO_SCALE);
    }
}

// max |x| as an IEEE bit pattern (non-negative floats order like their bits);
// one atomic per block (a per-wave atomic on one word serialises ~14x).
__global__ __launch_bounds__(256) void absmax_kernel(long n4, const f32x4* __restrict__ x, unsigned* __restrict__ out) {
    __shared__ unsigned red[4];
    const long stride = (long)gridDim.x * blockDim.x;
    unsigned m = 0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const f32x4 v = x[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const unsigned b = __float_as_uint(v[e]) & 0x7FFFFFFFu;
            m = b > m ? b : m;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned t = __shfl_xor(m, o);
        m = t > m ? t : m;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned a = red[0] > red[1] ? red[0] : red[1], b = red[2] > red[3] ? red[2] : red[3];
        atomicMax(out, a > b ? a : b);
    }
}

// ---------------------------------------------------------------------------
// f16x3 backward-filter: dW[k][j] = sum_m dy[m][k] * X[m][j], j = (tap, c).
// K dimension of the MFMA = pixels; both operands are pixel-major in HBM, so the
// loader reads 4 pixels x 4 channels, splits, transposes in registers and writes
// [channel][pixel] rows with ds_write_b64 — the same LDS image (80-B rows) the
// forward split kernel consumes.  Split-K over pixels (gridDim.y) into slabs.
struct WgSplitArgs {
    const float* x;
    const float* dy;
    const unsigned* amax;  // max|dy| bits (power-of-two scaling of dy), nullable
    float* ws;             // [splits][K][Kreal]
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M, Kreal, j_tiles, m_per_split;
};

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void wgrad_split_kernel(WgSplitArgs a) {
    constexpr int NT = 256, WM = 2, WN = 2;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    constexpr int BKM = 32;                          // pixels per stage
    constexpr int AQ = (BKM / 4) * (BM / 4);         // 4x4 quads of dy per stage
    constexpr int BQ = (BKM / 4) * (BN / 4);         // 4x4 quads of x per stage
    constexpr int AQT = (AQ + NT - 1) / NT, BQT = (BQ + NT - 1) / NT;
    constexpr int STAGE = 2 * (BM + BN) * SLDR;      // hi + lo planes, halves
    __shared__ __attribute__((aligned(16))) _Float16 smem[2 * STAGE];

    const int kt = blockIdx.x / a.j_tiles, jt = blockIdx.x - kt * a.j_tiles;
    const int k0 = kt * BM, j0 = jt * BN;
    const int m_begin = blockIdx.y * a.m_per_split;
    const int m_end = min(a.M, m_begin + a.m_per_split);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int hw = a.Ho * a.Wo;
    const int tap = j0 / a.C, c0 = j0 - (j0 / a.C) * a.C;
    const int tr = tap / a.S, ts = tap - tr * a.S;
    const float asc = pow2_scale_for(a.amax);

    f32x4 ra[AQT][4], rb[BQT][4];
    auto load = [&](int mb) {
#pragma unroll
        for (int qi = 0; qi < AQT; ++qi) {
            const int q = tid + NT * qi;
            if (q < AQ) {
                const int p0 = (q / (BM / 4)) * 4, c4 = q % (BM / 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = mb + p0 + e;
                    ra[qi][e] = m < m_end ? *(const f32x4*)(a.dy + (long)m * a.K + k0 + c4 * 4)
                                          : f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
        }
#pragma unroll
        for (int qi = 0; qi < BQT; ++qi) {
            const int q = tid + NT * qi;
            if (q < BQ) {
                const int p0 = (q / (BN / 4)) * 4, c4 = q % (BN / 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = mb + p0 + e;
                    f32x4 v = {0.f, 0.f, 0.f, 0.f};
                    if (m < m_end) {
                        const int n = m / hw, rem = m - n * hw;
                        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
                        const int hi = ho * a.stride - a.pad + tr * a.dil;
                        const int wi = wo * a.stride - a.pad + ts * a.dil;
                        if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
                            v = *(const f32x4*)(a.x + (((long)n * a.H + hi) * a.W + wi) * a.C + c0 + c4 * 4);
                    }
                    rb[qi][e] = v;
                }
            }
        }
    };
    // split + 4x4 transpose: row = channel, 4 consecutive pixels per ds_write_b64
    auto put = [&](_Float16* Th, _Float16* Tl, const f32x4 (&v)[4], int p0, int c4, float sc) {
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
            f16x4 h, l;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = v[e][ch] * sc;
                const _Float16 hv = (_Float16)x;
                h[e] = hv;
                l[e] = (_Float16)((x - (float)hv) * LO_SCALE);
            }
            const int off = (c4 * 4 + ch) * SLDR + p0;
            *(f16x4*)(Th + off) = h;
            *(f16x4*)(Tl + off) = l;
        }
    };
    auto store = [&](int buf) {
        _Float16* st = smem + buf * STAGE;
        _Float16* Ah = st;
        _Float16* Bh = st + BM * SLDR;
        _Float16* Al = st + (BM + BN) * SLDR;
        _Float16* Bl = Al + BM * SLDR;
#pragma unroll
        for (int qi = 0; qi < AQT; ++qi) {
            const int q = tid + NT * qi;
            if (q < AQ) put(Ah, Al, ra[qi], (q / (BM / 4)) * 4, q % (BM / 4), asc);
        }
#pragma unroll
        for (int qi = 0; qi < BQT; ++qi) {
            const int q = tid + NT * qi;
            if (q < BQ) put(Bh, Bl, rb[qi], (q / (BN / 4)) * 4, q % (BN / 4), 1.f);
        }
    };

    f32x16 acc[TM][TN], accc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][j][r] = 0.f;
                accc[i][j][r] = 0.f;
            }
    const int nst = (m_end - m_begin + BKM - 1) / BKM;
    if (nst > 0) {
        load(m_begin);
        store(0);
    }
    __syncthreads();
    const int frow = lane & 31, fk = (lane >> 5) * 8;
    for (int stp = 0; stp < nst; ++stp) {
        const int cur = stp & 1;
        const bool more = stp + 1 < nst;
        if (more) load(m_begin + (stp + 1) * BKM);
        const _Float16* st = smem + cur * STAGE;
        const _Float16* Ah = st + (wm * TM * 32 + frow) * SLDR + fk;
        const _Float16* Bh = st + BM * SLDR + (wn * TN * 32 + frow) * SLDR + fk;
        const _Float16* Al = Ah + (BM + BN) * SLDR;
        const _Float16* Bl = Bh + (BM + BN) * SLDR;
#pragma unroll
        for (int s = 0; s < BKM / 16; ++s) {
            f16x8 ah[TM], bh[TN], al[TM], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                ah[i] = *(const f16x8*)(Ah + i * 32 * SLDR + s * 16);
                al[i] = *(const f16x8*)(Al + i * 32 * SLDR + s * 16);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                bh[j] = *(const f16x8*)(Bh + j * 32 * SLDR + s * 16);
                bl[j] = *(const f16x8*)(Bl + j * 32 * SLDR + s * 16);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    accc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], accc[i][j], 0, 0, 0);
                    accc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], accc[i][j], 0, 0, 0);
                }
        }
        if (more) store(cur ^ 1);
        __syncthreads();
    }
    const float inv = 1.f / asc;
    float* out = a.ws + (long)blockIdx.y * a.K * a.Kreal;
    const int half = lane >> 5, col = lane & 31;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int jj = j0 + wn * TN * 32 + j * 32 + col;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = k0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                out[(long)k * a.Kreal + jj] = (acc[i][j][r] + accc[i][j][r] * LO_INV) * inv;
            }
        }
}

__global__ __launch_bounds__(256) void wg_split_reduce_kernel(long n, int splits, const float* __restrict__ ws,
                                                             float* __restrict__ out) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float s = 0.f;
        for (int k = 0; k < splits; ++k) s += ws[(long)k * n + i];
        out[i] = s;
    }
}

template <int BN, int PASSES, bool APL = false>
static int launch_split(const SplitArgs& a, int m_tiles, hipStream_t st) {
    hipLaunchKernelGGL((conv_split_kernel<128, BN, PASSES, APL>), dim3(m_tiles * a.n_tiles), dim3(256), 0, st, a);
    HKP_LAUNCH_CHECK("hkp_conv2d_fwd_split");
    return HKP_OK;
}

}  // namespace hkp

using namespace hkp;

extern "C" int hkp_weight_split(int64_t n, const float* w, uint16_t* w_hi, uint16_t* w_lo, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && w && w_hi, "hkp_weight_split: bad args");
    long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(weight_split_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), (long)n, w,
                       (_Float16*)w_hi, (_Float16*)w_lo);
    HKP_LAUNCH_CHECK("hkp_weight_split");
    return HKP_OK;
}

extern "C" int hkp_conv2d_fwd_split(const hkp_conv_desc* d, const float* x, const uint16_t* x_hi,
                                    const uint16_t* w_hi, const uint16_t* w_lo, int32_t passes,
                                    float* y, float* stat_partials, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG((x || x_hi) && w_hi && y, "hkp_conv2d_fwd_split: null tensor");
    HKP_CHECK_ARG(!x_hi || passes == 1, "hkp_conv2d_fwd_split: x_hi plane is for passes 1 (passes 3: hkp_conv2d_fwd_x3)");
    HKP_CHECK_ARG(passes == 1 || (passes == 3 && w_lo), "hkp_conv2d_fwd_split: passes must be 1 or 3 (3 needs w_lo)");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv2d_fwd_split: NHWC only");
    HKP_CHECK_ARG(d->c % 32 == 0 && d->k % 64 == 0, "hkp_conv2d_fwd_split: need Cin%%32==0, Cout%%64==0");
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31) && (long)d->n * d->h * d->w < (1L << 31), "hkp_conv2d_fwd_split: too large");
    SplitArgs a;
    a.x = x; a.whi = (const _Float16*)w_hi; a.wlo = (const _Float16*)w_lo; a.y = y; a.part = stat_partials;
    a.xhi = (const _Float16*)x_hi;
    a.amax = nullptr; a.add = nullptr;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = d->pad; a.dil = d->dilation; a.Ho = ho; a.Wo = wo;
    a.M = (int)M;
    a.Kreal = d->r * d->s * d->c;
    a.cchunks = d->c / SBK;
    a.nkc = d->r * d->s * a.cchunks;
    const bool bn128 = d->k % 128 == 0;
    a.n_tiles = d->k / (bn128 ? 128 : 64);
    const int m_tiles = (int)((M + 127) / 128);
    hipStream_t st = as_stream(stream);
    if (x_hi) return bn128 ? launch_split<128, 1, true>(a, m_tiles, st) : launch_split<64, 1, true>(a, m_tiles, st);
    if (passes == 3)
        return bn128 ? launch_split<128, 3>(a, m_tiles, st) : launch_split<64, 3>(a, m_tiles, st);
    return bn128 ? launch_split<128, 1>(a, m_tiles, st) : launch_split<64, 1>(a, m_tiles, st);
}

extern "C" int hkp_absmax(int64_t n, const float* x, uint32_t* amax_bits, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && n % 4 == 0 && x && amax_bits, "hkp_absmax: need n%%4==0 and non-null tensors");
    hipStream_t st = as_stream(stream);
    hipError_t e = hipMemsetAsync(amax_bits, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) {
        set_error("hkp_absmax: memset: %s", hipGetErrorString(e));
        return (int)e;
    }
    long g = (n / 4 + 255) / 256;
    if (g > 512) g = 512;          // one same-address atomicMax per block: keep them few
    hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)g), dim3(256), 0, st, (long)(n / 4), (const f32x4*)x,
                       (unsigned*)amax_bits);
    HKP_LAUNCH_CHECK("hkp_absmax");
    return HKP_OK;
}

extern "C" int hkp_conv_weight_flip_split(const hkp_conv_desc* d, const float* w, uint16_t* hi, uint16_t* lo,
                                          hkp_stream_t stream) {
    HKP_CHECK_ARG(d && w && hi, "hkp_conv_weight_flip_split: null argument");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv_weight_flip_split: KRSC weights only");
    const long total = (long)d->k * d->r * d->s * d->c;
    long g = (total + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(weight_flip_split_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), d->k, d->r,
                       d->s, d->c, w, (_Float16*)hi, (_Float16*)lo);
    HKP_LAUNCH_CHECK("hkp_conv_weight_flip_split");
    return HKP_OK;
}

extern "C" int hkp_conv2d_bwd_data_split(const hkp_conv_desc* d, const float* dy, const uint16_t* wf_hi,
                                         const uint16_t* wf_lo, const uint32_t* dy_amax_bits, const float* add,
                                         float* dx, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(dy && wf_hi && wf_lo && dx, "hkp_conv2d_bwd_data_split: null tensor");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC && d->stride == 1,
                  "hkp_conv2d_bwd_data_split: stride-1 NHWC convs only (strided ones use hkp_conv2d_bwd_data)");
    HKP_CHECK_ARG(d->c % 64 == 0 && d->k % 32 == 0, "hkp_conv2d_bwd_data_split: need Cin%%64==0, Cout%%32==0");
    const int padp = d->dilation * (d->r - 1) - d->pad;
    HKP_CHECK_ARG(padp >= 0 && d->dilation * (d->s - 1) - d->pad == padp, "hkp_conv2d_bwd_data_split: padding");
    const long M = (long)d->n * d->h * d->w;
    HKP_CHECK_ARG(M < (1L << 31), "hkp_conv2d_bwd_data_split: too large");
    SplitArgs a;
    a.x = dy; a.whi = (const _Float16*)wf_hi; a.wlo = (const _Float16*)wf_lo; a.y = dx; a.part = nullptr;
    a.xhi = nullptr;
    a.amax = dy_amax_bits; a.add = add;
    a.N = d->n; a.H = ho; a.W = wo; a.C = d->k; a.K = d->c; a.R = d->r; a.S = d->s;
    a.stride = 1; a.pad = padp; a.dil = d->dilation; a.Ho = d->h; a.Wo = d->w;
    a.M = (int)M;
    a.Kreal = d->r * d->s * d->k;
    a.cchunks = d->k / SBK;
    a.nkc = d->r * d->s * a.cchunks;
    const bool bn128 = d->c % 128 == 0;
    a.n_tiles = d->c / (bn128 ? 128 : 64);
    const int m_tiles = (int)((M + 127) / 128);
    hipStream_t st = as_stream(stream);
    return bn128 ? launch_split<128, 3>(a, m_tiles, st) : launch_split<64, 3>(a, m_tiles, st);
}

static void wg_split_plan(const hkp_conv_desc* d, long M, int* splits, int* mps, int* bm, int* bn) {
    *bm = d->k % 128 == 0 ? 128 : 64;
    *bn = d->c % 128 == 0 ? 128 : 64;
    const long tiles = (long)(d->k / *bm) * ((long)d->r * d->s * d->c / *bn);
    long sp = (2048 + tiles - 1) / tiles;
    const long max_sp = (M + 255) / 256;
    if (sp > max_sp) sp = max_sp;
    if (sp < 1) sp = 1;
    long m = (M + sp - 1) / sp;
    m = (m + 31) / 32 * 32;
    *splits = (int)((M + m - 1) / m);
    *mps = (int)m;
}

extern "C" int64_t hkp_conv_bwd_filter_split_workspace(const hkp_conv_desc* d) {
    int ho, wo;
    if (hkp_conv_out_hw(d, &ho, &wo) != HKP_OK) return -1;
    int sp, mps, bm, bn;
    wg_split_plan(d, (long)d->n * ho * wo, &sp, &mps, &bm, &bn);
    return (int64_t)sp * d->k * d->r * d->s * d->c * (int64_t)sizeof(float);
}

extern "C" int hkp_conv2d_bwd_filter_split(const hkp_conv_desc* d, const float* x, const float* dy,
                                           const uint32_t* dy_amax_bits, float* dw, void* workspace,
                                           int64_t ws_bytes, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(x && dy && dw && workspace, "hkp_conv2d_bwd_filter_split: null tensor");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv2d_bwd_filter_split: NHWC convs only");
    HKP_CHECK_ARG(d->k % 64 == 0 && d->c % 64 == 0, "hkp_conv2d_bwd_filter_split: need Cout%%64==0, Cin%%64==0");
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31), "hkp_conv2d_bwd_filter_split: too large");
    int sp, mps, bm, bn;
    wg_split_plan(d, M, &sp, &mps, &bm, &bn);
    const long need = (long)sp * d->k * d->r * d->s * d->c * (long)sizeof(float);
    HKP_CHECK_ARG(ws_bytes >= need, "hkp_conv2d_bwd_filter_split: workspace %ld < %ld", (long)ws_bytes, need);
    WgSplitArgs a;
    a.x = x; a.dy = dy; a.amax = dy_amax_bits; a.ws = (float*)workspace;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = d->pad; a.dil = d->dilation; a.Ho = ho; a.Wo = wo;
    a.M = (int)M;
    a.Kreal = d->r * d->s * d->c;
    a.j_tiles = a.Kreal / bn;
    a.m_per_split = mps;
    dim3 grid((d->k / bm) * a.j_tiles, sp);
    hipStream_t st = as_stream(stream);
    if (bm == 128 && bn == 128)
        hipLaunchKernelGGL((wgrad_split_kernel<128, 128>), grid, dim3(256), 0, st, a);
    else if (bm == 128)
        hipLaunchKernelGGL((wgrad_split_kernel<128, 64>), grid, dim3(256), 0, st, a);
    else if (bn == 128)
        hipLaunchKernelGGL((wgrad_split_kernel<64, 128>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((wgrad_split_kernel<64, 64>), grid, dim3(256), 0, st, a);
    HKP_LAUNCH_CHECK("hkp_conv2d_bwd_filter_split");
    const long n = (long)d->k * a.Kreal;
    long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(wg_split_reduce_kernel, dim3((unsigned)g), dim3(256), 0, st, n, sp, a.ws, dw);
    HKP_LAUNCH_CHECK("hkp_conv2d_bwd_filter_split(reduce)");
    return HKP_OK;
}
