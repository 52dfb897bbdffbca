// Convolution backward: weight flip (for dgrad through the forward template)
// and backward-filter (wgrad) on fp32 MFMA.
//
// wgrad GEMM: dW[k][j] = sum_m dy[m][k] * X[m][j] with j = (tap, c) (NHWC,
// KRSC weight) or j = (c, r, s) (stem: NCHW image, OIHW weight) and
// X[m][j] the input pixel that tap reads for output pixel m.  The reduction
// dimension (N*Ho*Wo pixels) is split over gridDim.y; each split writes its
// [K][Kreal] partial to a workspace slab and hkp_conv2d_bwd_filter's second
// kernel sums the slabs in fixed order — deterministic, no float atomics.
//
// Replaces the implicit cuDNN backward-filter / backward-data of every conv
// in src/resnet.py (conv3x3 :20-37, 1x1 :77,86, downsample :184-188, stem :137)
// that the reference's loss.backward() (train.py:35) runs.
#include "common.h"

namespace hkp {

// w'[c][r'][s'][k] = w[k][R-1-r'][S-1-s'][c]   (KRSC → flipped CRSK)
__global__ __launch_bounds__(256) void weight_flip_kernel(int K, int R, int S, int C, const float* __restrict__ w,
                                                         float* __restrict__ wf) {
    const long total = (long)K * R * S * C;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        // i indexes the OUTPUT (c, r', s', k) so the writes are coalesced
        const int k = (int)(i % K);
        long t = i / K;
        const int sp = (int)(t % S);
        t /= S;
        const int rp = (int)(t % R);
        const int c = (int)(t / R);
        wf[i] = w[(((long)k * R + (R - 1 - rp)) * S + (S - 1 - sp)) * C + c];
    }
}

struct WgArgs {
    const float* x;   // NHWC input (or NCHW image for the stem)
    const float* dy;  // NHWC [M][K]
    float* ws;        // [splits][K][Kreal]
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M, Kreal;
    int k_tiles, j_tiles;
    int m_per_split;  // multiple of 32
};

constexpr int WG_BKM = 32;  // pixels per LDS stage

template <int BM, int BN, bool STEM>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(WgArgs a) {
    constexpr int NT = 256;
    constexpr int WM = 2, WN = 2;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    constexpr int AP = WG_BKM * BM / 4 / NT;  // float4 of dy per thread per stage
    constexpr int BPV = WG_BKM * BN / 4 / NT;  // float4 of x per thread per stage
    constexpr int APR = BM / 4, BPR = BN / 4;  // float4 per LDS row
    __shared__ __attribute__((aligned(16))) float smem[2 * WG_BKM * (BM + BN)];
    float* As = smem;                       // [2][BKM][BM]   dy tile, row = pixel
    float* Bs = smem + 2 * WG_BKM * BM;     // [2][BKM][BN]   gathered x tile, row = pixel

    const int tile = blockIdx.x;
    const int kt = tile / a.j_tiles, jt = tile - kt * a.j_tiles;
    const int k0 = kt * BM, j0 = jt * BN;
    const int m_begin = blockIdx.y * a.m_per_split;
    const int m_end = min(a.M, m_begin + a.m_per_split);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
    const int hw = a.Ho * a.Wo;

    // NHWC: the j tile lies inside one filter tap (C % BN == 0)
    int tap_r = 0, tap_s = 0, c0 = 0;
    if constexpr (!STEM) {
        const int tap = j0 / a.C;
        c0 = j0 - tap * a.C;
        tap_r = tap / a.S;
        tap_s = tap - tap_r * a.S;
    }

    f32x4 ra[AP], rb[BPV];
    auto load = [&](int mb) {
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int idx = tid + NT * i;
            const int p = idx / APR, c4 = idx - p * APR;
            const int m = mb + p;
            ra[i] = m < m_end ? *(const f32x4*)(a.dy + (long)m * a.K + k0 + c4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < BPV; ++i) {
            const int idx = tid + NT * i;
            const int p = idx / BPR, c4 = idx - p * BPR;
            const int m = mb + p;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (m < m_end) {
                const int n = m / hw, rem = m - n * hw;
                const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
                if constexpr (!STEM) {
                    const int hi = ho * a.stride - a.pad + tap_r * a.dil;
                    const int wi = wo * a.stride - a.pad + tap_s * a.dil;
                    if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
                        v = *(const f32x4*)(a.x + (((long)n * a.H + hi) * a.W + wi) * a.C + c0 + c4 * 4);
                } else {
                    const int RS = a.R * a.S;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int j = j0 + c4 * 4 + e;
                        if (j < a.Kreal) {
                            const int c = j / RS, t = j - c * RS;
                            const int rr = t / a.S, ss = t - rr * a.S;
                            const int hi = ho * a.stride - a.pad + rr * a.dil;
                            const int wi = wo * a.stride - a.pad + ss * a.dil;
                            if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
                                v[e] = a.x[(((long)n * a.C + c) * a.H + hi) * a.W + wi];
                        }
                    }
                }
            }
            rb[i] = v;
        }
    };
    auto store = [&](int buf) {
        float* A = As + buf * WG_BKM * BM;
        float* B = Bs + buf * WG_BKM * BN;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int idx = tid + NT * i;
            *(f32x4*)(A + (idx / APR) * BM + (idx % APR) * 4) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BPV; ++i) {
            const int idx = tid + NT * i;
            *(f32x4*)(B + (idx / BPR) * BN + (idx % BPR) * 4) = rb[i];
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nst = (m_end - m_begin + WG_BKM - 1) / WG_BKM;
    if (nst > 0) {
        load(m_begin);
        store(0);
    }
    __syncthreads();
    const int half = lane >> 5, col = lane & 31;
    for (int st = 0; st < nst; ++st) {
        const int cur = st & 1;
        const bool more = st + 1 < nst;
        if (more) load(m_begin + (st + 1) * WG_BKM);
        const float* A = As + cur * WG_BKM * BM + half * BM + wm * TM * 32 + col;
        const float* B = Bs + cur * WG_BKM * BN + half * BN + wn * TN * 32 + col;
#pragma unroll
        for (int kk = 0; kk < WG_BKM; kk += 2) {
            float af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = A[kk * BM + i * 32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = B[kk * BN + j * 32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (more) store(cur ^ 1);
        __syncthreads();
    }

    float* out = a.ws + (long)blockIdx.y * a.K * a.Kreal;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int jj = j0 + wn * TN * 32 + j * 32 + col;
            if (jj >= a.Kreal) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = k0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                out[(long)k * a.Kreal + jj] = acc[i][j][r];
            }
        }
}

// dw[i] = sum_s ws[s][i] in a fixed order: 4 lanes per element each sum every
// 4th split (many loads in flight per thread), then the 4 lane sums pairwise
__global__ __launch_bounds__(256) void split_reduce_kernel(long n, int splits, const float* __restrict__ ws,
                                                          float* __restrict__ out, int accumulate) {
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
    if (q == 0 && i < n) {
        const float t = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
        out[i] = accumulate ? out[i] + t : t;
    }
}

static int wgrad_plan(const hkp_conv_desc* d, int ho, int wo, int* splits, int* m_per_split, int* bm, int* bn) {
    const long M = (long)d->n * ho * wo;
    const int Kreal = d->r * d->s * d->c;
    *bm = d->k % 128 == 0 ? 128 : 64;
    if (d->in_layout == HKP_LAYOUT_NHWC)
        *bn = d->c % 128 == 0 ? 128 : 64;
    else
        *bn = 64;
    const long tiles = (long)(d->k / *bm) * ((Kreal + *bn - 1) / *bn);
    long sp = (2048 + tiles - 1) / tiles;
    const long max_sp = (M + 255) / 256;  // at least 256 pixels per split
    if (sp > max_sp) sp = max_sp;
    if (sp < 1) sp = 1;
    long mps = (M + sp - 1) / sp;
    mps = (mps + WG_BKM - 1) / WG_BKM * WG_BKM;
    sp = (M + mps - 1) / mps;
    *splits = (int)sp;
    *m_per_split = (int)mps;
    return HKP_OK;
}

}  // namespace hkp

using namespace hkp;

extern "C" int hkp_conv_weight_flip(const hkp_conv_desc* d, const float* w, float* w_flip, hkp_stream_t stream) {
    HKP_CHECK_ARG(d && w && w_flip, "hkp_conv_weight_flip: null argument");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv_weight_flip: KRSC weights only");
    const long total = (long)d->k * d->r * d->s * d->c;
    long g = (total + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(weight_flip_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), d->k, d->r, d->s, d->c,
                       w, w_flip);
    HKP_LAUNCH_CHECK("hkp_conv_weight_flip");
    return HKP_OK;
}

extern "C" int64_t hkp_conv_bwd_filter_workspace(const hkp_conv_desc* d) {
    int ho, wo;
    if (hkp_conv_out_hw(d, &ho, &wo) != HKP_OK) return -1;
    int sp, mps, bm, bn;
    wgrad_plan(d, ho, wo, &sp, &mps, &bm, &bn);
    return (int64_t)sp * d->k * d->r * d->s * d->c * (int64_t)sizeof(float);
}

extern "C" int hkp_conv2d_bwd_filter(const hkp_conv_desc* d, const float* x, const float* dy, float* dw,
                                     int32_t accumulate, void* workspace, int64_t ws_bytes, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(x && dy && dw && workspace, "hkp_conv2d_bwd_filter: null tensor");
    HKP_CHECK_ARG(d->k % 64 == 0, "hkp_conv2d_bwd_filter: Cout=%d must be a multiple of 64", d->k);
    if (d->in_layout == HKP_LAYOUT_NHWC)
        HKP_CHECK_ARG(d->c % 64 == 0, "hkp_conv2d_bwd_filter: NHWC Cin=%d must be a multiple of 64", d->c);
    else
        HKP_CHECK_ARG(d->c <= 8, "hkp_conv2d_bwd_filter: NCHW path is the stem (Cin<=8)");
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31), "hkp_conv2d_bwd_filter: tensor too large");
    int sp, mps, bm, bn;
    wgrad_plan(d, ho, wo, &sp, &mps, &bm, &bn);
    const long need = (long)sp * d->k * d->r * d->s * d->c * (long)sizeof(float);
    HKP_CHECK_ARG(ws_bytes >= need, "hkp_conv2d_bwd_filter: workspace %ld < %ld bytes", (long)ws_bytes, need);
    WgArgs a;
    a.x = x; a.dy = dy; a.ws = (float*)workspace;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = d->pad; a.dil = d->dilation; a.Ho = ho; a.Wo = wo;
    a.M = (int)M;
    a.Kreal = d->r * d->s * d->c;
    a.k_tiles = d->k / bm;
    a.j_tiles = (a.Kreal + bn - 1) / bn;
    a.m_per_split = mps;
    dim3 grid(a.k_tiles * a.j_tiles, sp);
    hipStream_t st = as_stream(stream);
    if (d->in_layout == HKP_LAYOUT_NHWC) {
        if (bm == 128 && bn == 128)
            hipLaunchKernelGGL((conv_wgrad_kernel<128, 128, false>), grid, dim3(256), 0, st, a);
        else if (bm == 128)
            hipLaunchKernelGGL((conv_wgrad_kernel<128, 64, false>), grid, dim3(256), 0, st, a);
        else if (bn == 128)
            hipLaunchKernelGGL((conv_wgrad_kernel<64, 128, false>), grid, dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL((conv_wgrad_kernel<64, 64, false>), grid, dim3(256), 0, st, a);
    } else {
        if (bm == 128)
            hipLaunchKernelGGL((conv_wgrad_kernel<128, 64, true>), grid, dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL((conv_wgrad_kernel<64, 64, true>), grid, dim3(256), 0, st, a);
    }
    HKP_LAUNCH_CHECK("hkp_conv2d_bwd_filter");
    const long n = (long)d->k * a.Kreal;
    hipLaunchKernelGGL(split_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, n, sp, a.ws, dw,
                       accumulate);
    HKP_LAUNCH_CHECK("hkp_conv2d_bwd_filter(reduce)");
    return HKP_OK;
}
