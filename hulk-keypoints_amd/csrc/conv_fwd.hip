// Implicit-GEMM convolution forward on fp32 MFMA (gfx950).
//
// GEMM view: M = N*Ho*Wo output pixels (rows), N = Cout (cols), K = R*S*Cin.
// Activations NHWC, weights KRSC, so a K-chunk of 32 is one filter tap x 32
// contiguous input channels — every A and B row segment is a 128-B coalesced
// load.  Tiles are staged global→registers→LDS (double buffered, one barrier
// per K-chunk) and consumed by v_mfma_f32_32x32x2_f32 (exact fp32, 64
// FLOP/clk/SIMD).  Each lane reads 4 consecutive k of its row with one
// ds_read_b128; the K order inside a chunk is permuted identically for A and B
// (lane half h takes k = 8*kk + 4*h + s at MFMA step s), which leaves the dot
// product unchanged.  Rows are padded to 36 floats: conflict-free b128 reads.
//
// Replaces the cuDNN convs the reference calls implicitly:
//   conv3x3 (padding = dilation)   src/resnet.py:20-37
//   Bottleneck 1x1 convs           src/resnet.py:77,86
//   downsample 1x1 (stride)        src/resnet.py:184-188
//   stem 7x7/s2/p3 (NCHW, C=3)     src/resnet.py:137
//
// Epilogue (optional): per-tile, per-channel (sum, M2) BatchNorm partials —
// M2 is taken around the TILE mean from the fp32 accumulators still in
// registers, so the fp64 Chan merge in bn.hip never suffers E[x^2]-E[x]^2
// cancellation.
#include <stdarg.h>

#include "common.h"

namespace hkp {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

struct ConvArgs {
    const float* x;
    const float* w;
    float* y;
    float* part;
    const float* add;  // optional addend of the output (dgrad: the residual-branch gradient)
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M;        // N*Ho*Wo
    int Kreal;    // R*S*C
    int nkc;      // K-chunks of 32
    int cchunks;  // C/32 (NHWC)
    int n_tiles;  // Cout / BN
};

constexpr int BK = 32;
constexpr int LDR = BK + 4;  // padded LDS row (floats)
constexpr int CONV_BM = 128;

// MODE_FWD: NHWC forward; MODE_STEM: NCHW image + OIHW weight gather;
// MODE_DGRAD: transposed conv (backward-data of a strided conv): the "input" is
// dy, rows are dx pixels, and tap (r,s) reads dy[(h - pad' + r*dil)/stride] only
// where that division is exact (weights pre-flipped by hkp_conv_weight_flip).
enum { MODE_FWD = 0, MODE_STEM = 1, MODE_DGRAD = 2 };

template <int BM, int BN, int MODE>
__global__ __launch_bounds__(256, 2) void conv_fwd_kernel(ConvArgs a) {
    constexpr bool STEM = MODE == MODE_STEM;
    constexpr int NT = 256, WM = 2, WN = 2;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    constexpr int AP = BM * (BK / 4) / NT;  // float4 A loads per thread
    constexpr int BP = BN * (BK / 4) / NT;  // float4 B loads per thread
    __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDR];
    float* As = smem;
    float* Bs = smem + 2 * BM * LDR;

    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int col4 = tid & 7, rowb = tid >> 3;

    // per-thread A-row geometry (fixed across the K loop)
    int a_n[AP], a_hi[AP], a_wi[AP];
#pragma unroll
    for (int i = 0; i < AP; ++i) {
        const int m = m0 + rowb + 32 * i;
        if (m < a.M) {
            const int hw = a.Ho * a.Wo;
            const int n = m / hw, rem = m - n * hw;
            const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
            a_n[i] = n;
            a_hi[i] = MODE == MODE_DGRAD ? ho - a.pad : ho * a.stride - a.pad;
            a_wi[i] = MODE == MODE_DGRAD ? wo - a.pad : wo * a.stride - a.pad;
        } else {
            a_n[i] = 0;
            a_hi[i] = -(1 << 28);  // never in bounds
            a_wi[i] = -(1 << 28);
        }
    }

    f32x4 ra[AP], rb[BP];

    auto load_chunk = [&](int kc) {
        if constexpr (!STEM) {
            const int tap = kc / a.cchunks;
            const int c0 = (kc - tap * a.cchunks) * BK + col4 * 4;
            const int rr = tap / a.S, ss = tap - rr * a.S;
#pragma unroll
            for (int i = 0; i < AP; ++i) {
                int hi = a_hi[i] + rr * a.dil, wi = a_wi[i] + ss * a.dil;
                if constexpr (MODE == MODE_DGRAD) {
                    const bool exact = hi >= 0 && wi >= 0 && hi % a.stride == 0 && wi % a.stride == 0;
                    hi = exact ? hi / a.stride : -1;
                    wi = exact ? wi / a.stride : -1;
                }
                if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W) {
                    const long pix = ((long)a_n[i] * a.H + hi) * a.W + wi;
                    ra[i] = *(const f32x4*)(a.x + pix * a.C + c0);
                } else {
                    ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
#pragma unroll
            for (int i = 0; i < BP; ++i) {
                const int row = rowb + 32 * i;
                rb[i] = *(const f32x4*)(a.w + (long)(n0 + row) * a.Kreal + kc * BK + col4 * 4);
            }
        } else {
            // stem: NCHW input, OIHW weight, k = c*R*S + r*S + s (the weight's own flattening)
            const int RS = a.R * a.S;
#pragma unroll
            for (int i = 0; i < AP; ++i) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = kc * BK + col4 * 4 + e;
                    float v = 0.f;
                    if (k < a.Kreal) {
                        const int c = k / RS, t = k - c * RS;
                        const int rr = t / a.S, ss = t - rr * a.S;
                        const int hi = a_hi[i] + rr * a.dil, wi = a_wi[i] + ss * a.dil;
                        if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
                            v = a.x[(((long)a_n[i] * a.C + c) * a.H + hi) * a.W + wi];
                    }
                    ra[i][e] = v;
                }
            }
#pragma unroll
            for (int i = 0; i < BP; ++i) {
                const int row = rowb + 32 * i;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = kc * BK + col4 * 4 + e;
                    rb[i][e] = k < a.Kreal ? a.w[(long)(n0 + row) * a.Kreal + k] : 0.f;
                }
            }
        }
    };
    auto store_chunk = [&](int buf) {
        float* A = As + buf * BM * LDR;
        float* B = Bs + buf * BN * LDR;
#pragma unroll
        for (int i = 0; i < AP; ++i) *(f32x4*)(A + (rowb + 32 * i) * LDR + col4 * 4) = ra[i];
#pragma unroll
        for (int i = 0; i < BP; ++i) *(f32x4*)(B + (rowb + 32 * i) * LDR + col4 * 4) = rb[i];
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    load_chunk(0);
    store_chunk(0);
    __syncthreads();

    const int frow = lane & 31, fk = (lane >> 5) * 4;
    for (int kc = 0; kc < a.nkc; ++kc) {
        const int cur = kc & 1;
        const bool more = kc + 1 < a.nkc;
        if (more) load_chunk(kc + 1);
        const float* A = As + cur * BM * LDR + (wm * TM * 32 + frow) * LDR + fk;
        const float* B = Bs + cur * BN * LDR + (wn * TN * 32 + frow) * LDR + fk;
#pragma unroll
        for (int kk = 0; kk < BK / 8; ++kk) {
            f32x4 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = *(const f32x4*)(A + i * 32 * LDR + kk * 8);
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = *(const f32x4*)(B + j * 32 * LDR + kk * 8);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
        }
        if (more) store_chunk(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: store y (NHWC) ----
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

    // ---- epilogue: BN partials (sum, M2 about the tile mean) ----
    float* red = smem;               // [WM][BN]
    float* tmean = smem + WM * BN;   // [BN]
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

template <int BM, int BN, int MODE>
static int launch_conv(const ConvArgs& a, int m_tiles, hipStream_t st) {
    const int grid = m_tiles * a.n_tiles;
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, MODE>), dim3(grid), dim3(256), 0, st, a);
    HKP_LAUNCH_CHECK("hkp_conv2d_fwd");
    return HKP_OK;
}

static int conv_geometry(const hkp_conv_desc* d, int* ho, int* wo) {
    HKP_CHECK_ARG(d != nullptr, "conv: null descriptor");
    HKP_CHECK_ARG(d->n > 0 && d->h > 0 && d->w > 0 && d->c > 0 && d->k > 0 && d->r > 0 && d->s > 0,
                  "conv: non-positive size");
    HKP_CHECK_ARG(d->stride > 0 && d->dilation > 0 && d->pad >= 0, "conv: bad stride/dilation/pad");
    *ho = (d->h + 2 * d->pad - d->dilation * (d->r - 1) - 1) / d->stride + 1;
    *wo = (d->w + 2 * d->pad - d->dilation * (d->s - 1) - 1) / d->stride + 1;
    HKP_CHECK_ARG(*ho > 0 && *wo > 0, "conv: empty output");
    return HKP_OK;
}

}  // namespace hkp

using namespace hkp;

extern "C" const char* hkp_last_error(void) { return g_err; }
extern "C" const char* hkp_version(void) { return "hulkkp 0.1.0 gfx950"; }

extern "C" int hkp_conv_out_hw(const hkp_conv_desc* d, int32_t* ho, int32_t* wo) {
    int h = 0, w = 0;
    int rc = conv_geometry(d, &h, &w);
    if (rc) return rc;
    if (ho) *ho = h;
    if (wo) *wo = w;
    return HKP_OK;
}

extern "C" int64_t hkp_conv_stat_tiles(const hkp_conv_desc* d) {
    int ho, wo;
    if (conv_geometry(d, &ho, &wo)) return -1;
    const long M = (long)d->n * ho * wo;
    return (M + CONV_BM - 1) / CONV_BM;
}

extern "C" int hkp_conv2d_fwd(const hkp_conv_desc* d, const float* x, const float* w, float* y,
                              float* stat_partials, hkp_stream_t stream) {
    int ho, wo;
    int rc = conv_geometry(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(x && w && y, "hkp_conv2d_fwd: null tensor");
    HKP_CHECK_ARG(d->k % 64 == 0, "hkp_conv2d_fwd: Cout=%d must be a multiple of 64", d->k);
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31) && (long)d->n * d->h * d->w < (1L << 31), "hkp_conv2d_fwd: tensor too large");
    ConvArgs a;
    a.x = x; a.w = w; a.y = y; a.part = stat_partials; a.add = nullptr;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = d->pad; a.dil = d->dilation; a.Ho = ho; a.Wo = wo;
    a.M = (int)M;
    a.Kreal = d->r * d->s * d->c;
    const int m_tiles = (int)((M + CONV_BM - 1) / CONV_BM);
    const bool bn128 = d->k % 128 == 0;
    a.n_tiles = d->k / (bn128 ? 128 : 64);
    hipStream_t st = as_stream(stream);
    if (d->in_layout == HKP_LAYOUT_NHWC) {
        HKP_CHECK_ARG(d->c % 32 == 0, "hkp_conv2d_fwd: NHWC Cin=%d must be a multiple of 32", d->c);
        a.cchunks = d->c / 32;
        a.nkc = d->r * d->s * a.cchunks;
        return bn128 ? launch_conv<CONV_BM, 128, MODE_FWD>(a, m_tiles, st)
                      : launch_conv<CONV_BM, 64, MODE_FWD>(a, m_tiles, st);
    }
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NCHW, "hkp_conv2d_fwd: bad layout %d", d->in_layout);
    HKP_CHECK_ARG(d->c <= 8, "hkp_conv2d_fwd: NCHW path is the stem (Cin<=8), got %d", d->c);
    a.cchunks = 0;
    a.nkc = (a.Kreal + BK - 1) / BK;
    return bn128 ? launch_conv<CONV_BM, 128, MODE_STEM>(a, m_tiles, st)
                  : launch_conv<CONV_BM, 64, MODE_STEM>(a, m_tiles, st);
}

// ---------------------------------------------------------------- dgrad ----
extern "C" int hkp_conv2d_bwd_data(const hkp_conv_desc* d, const float* dy, const float* w_flip, const float* add, float* dx,
                                   hkp_stream_t stream) {
    int ho, wo;
    int rc = conv_geometry(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(dy && w_flip && dx, "hkp_conv2d_bwd_data: null tensor");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv2d_bwd_data: NHWC convs only (the stem needs no dgrad)");
    HKP_CHECK_ARG(d->c % 64 == 0 && d->k % 32 == 0, "hkp_conv2d_bwd_data: need Cin%%64==0 and Cout%%32==0");
    const long M = (long)d->n * d->h * d->w;  // dx pixels
    HKP_CHECK_ARG(M < (1L << 31), "hkp_conv2d_bwd_data: tensor too large");
    // dx = conv(dy, flip(w)) with pad' = dil*(R-1) - pad; strided convs use the transposed loader
    const int padp = d->dilation * (d->r - 1) - d->pad;
    HKP_CHECK_ARG(padp >= 0 && d->dilation * (d->s - 1) - d->pad == padp, "hkp_conv2d_bwd_data: asymmetric padding");
    ConvArgs a;
    a.x = dy; a.w = w_flip; a.y = dx; a.part = nullptr; a.add = add;
    a.N = d->n; a.H = ho; a.W = wo; a.C = d->k; a.K = d->c; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = padp; a.dil = d->dilation; a.Ho = d->h; a.Wo = d->w;
    a.M = (int)M;
    a.Kreal = d->r * d->s * d->k;
    a.cchunks = d->k / 32;
    a.nkc = d->r * d->s * a.cchunks;
    const bool bn128 = d->c % 128 == 0;
    a.n_tiles = d->c / (bn128 ? 128 : 64);
    const int m_tiles = (int)((M + CONV_BM - 1) / CONV_BM);
    hipStream_t st = as_stream(stream);
    if (d->stride == 1)
        return bn128 ? launch_conv<CONV_BM, 128, MODE_FWD>(a, m_tiles, st)
                     : launch_conv<CONV_BM, 64, MODE_FWD>(a, m_tiles, st);
    return bn128 ? launch_conv<CONV_BM, 128, MODE_DGRAD>(a, m_tiles, st)
                 : launch_conv<CONV_BM, 64, MODE_DGRAD>(a, m_tiles, st);
}
