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
    const _Float16* whi;
    const _Float16* wlo;
    float* y;
    float* part;
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M, Kreal, nkc, cchunks, n_tiles;
};

constexpr int SBK = 32;         // K chunk (channels of one tap)
constexpr int SLDR = SBK + 8;   // LDS row stride in halves (80 B)
constexpr float LO_SCALE = 2048.f;
constexpr float LO_INV = 1.f / 2048.f;

template <int BM, int BN, int PASSES>
__global__ __launch_bounds__(256, 2) void conv_split_kernel(SplitArgs a) {
    constexpr int NT = 256, WM = 2, WN = 2;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    constexpr int PL = PASSES == 3 ? 2 : 1;          // planes (hi[, lo])
    constexpr int AP = BM * (SBK / 4) / NT;          // f32x4 A loads per thread
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
    const int c8 = tid & 3, browb = tid >> 2;    // B: 4 threads x f16x8 per row

    int a_n[AP], a_hi[AP], a_wi[AP];
#pragma unroll
    for (int i = 0; i < AP; ++i) {
        const int m = m0 + rowb + 32 * i;
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

    f32x4 ra[AP];
    f16x8 rbh[BP], rbl[BP];

    auto load_chunk = [&](int kc) {
        const int tap = kc / a.cchunks;
        const int c0 = (kc - tap * a.cchunks) * SBK;
        const int rr = tap / a.S, ss = tap - rr * a.S;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int hi = a_hi[i] + rr * a.dil, wi = a_wi[i] + ss * a.dil;
            if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W) {
                const long pix = ((long)a_n[i] * a.H + hi) * a.W + wi;
                ra[i] = *(const f32x4*)(a.x + pix * a.C + c0 + col4 * 4);
            } else {
                ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            const long off = (long)(n0 + browb + 64 * i) * a.Kreal + kc * SBK + c8 * 8;
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
            f16x4 h, l;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float v = ra[i][e];
                const _Float16 hv = (_Float16)v;
                h[e] = hv;
                if constexpr (PASSES == 3) l[e] = (_Float16)((v - (float)hv) * LO_SCALE);
            }
            const int off = (rowb + 32 * i) * SLDR + col4 * 4;
            *(f16x4*)(Ah + off) = h;
            if constexpr (PASSES == 3) *(f16x4*)(Al + off) = l;
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
                if (m < a.M) a.y[(long)m * a.K + n] = acc[i][j][r];
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

template <int BN, int PASSES>
static int launch_split(const SplitArgs& a, int m_tiles, hipStream_t st) {
    hipLaunchKernelGGL((conv_split_kernel<128, BN, PASSES>), dim3(m_tiles * a.n_tiles), dim3(256), 0, st, a);
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

extern "C" int hkp_conv2d_fwd_split(const hkp_conv_desc* d, const float* x, const uint16_t* w_hi,
                                    const uint16_t* w_lo, int32_t passes, float* y, float* stat_partials,
                                    hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(x && w_hi && y, "hkp_conv2d_fwd_split: null tensor");
    HKP_CHECK_ARG(passes == 1 || (passes == 3 && w_lo), "hkp_conv2d_fwd_split: passes must be 1 or 3 (3 needs w_lo)");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv2d_fwd_split: NHWC only");
    HKP_CHECK_ARG(d->c % 32 == 0 && d->k % 64 == 0, "hkp_conv2d_fwd_split: need Cin%%32==0, Cout%%64==0");
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31) && (long)d->n * d->h * d->w < (1L << 31), "hkp_conv2d_fwd_split: too large");
    SplitArgs a;
    a.x = x; a.whi = (const _Float16*)w_hi; a.wlo = (const _Float16*)w_lo; a.y = y; a.part = stat_partials;
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
    if (passes == 3)
        return bn128 ? launch_split<128, 3>(a, m_tiles, st) : launch_split<64, 3>(a, m_tiles, st);
    return bn128 ? launch_split<128, 1>(a, m_tiles, st) : launch_split<64, 1>(a, m_tiles, st);
}
