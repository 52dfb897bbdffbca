// f16x3 implicit-GEMM convolution forward, deep-pipelined (the main-path conv of
// the f16x3 precision; arithmetic identical to conv_f16.hip's PASSES=3 kernel).
//
// Operands arrive PRE-SPLIT in the "packed split" layout written by their
// producers (bn_apply / bn_relu_maxpool with split_passes=3; weights by
// hkp_weight_pack_x3):
//
//     xs[pixel][C/32][ hi(32 ch) | lo(32 ch) ]        fp16, 128 B per (pixel, group)
//     ws[k][tap][C/32][ hi(32 ch) | lo(32 ch) ]
//
// so one K-step (one filter tap x 32 channels) of one GEMM row is exactly one
// 128-B cache line holding both planes.  The same bytes as the fp32 tensor.
//
// Tile 256 (pixels) x BN (output channels) x 32 channels, 8 waves as 4x2.
// Staging is LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no
// ds_write) into a 3-stage LDS ring, two K-steps in flight ahead of the
// compute, retired by a counted s_waitcnt vmcnt + raw s_barrier (never
// __syncthreads inside the loop: its fence would drain the DMA queue).
// LDS rows are 128 B and unpadded (the DMA writes lane-linear 1 KiB pieces);
// bank conflicts of the fragment reads are removed by an XOR swizzle of the
// 16-B chunk index with (row>>1)&7, applied to the per-lane SOURCE address of
// the DMA and to the ds_read address.  Out-of-image taps / rows past M load a
// zero line.  Epilogue: NHWC fp32 store + BN tile partials per 128-row tile
// (the same partials format as every other conv here).
//
// Replaces the same cuDNN convs as conv_fwd.hip (src/resnet.py:20-37,77,86,184-188).
#include "common.h"

namespace hkp {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __attribute__((aligned(256))) uint4 g_x3_zero_line[8];   // 128 B of zeros (static, zero-initialised)

struct X3Args {
    const _Float16* xs;
    const _Float16* ws;
    float* y;
    float* part;
    int N, H, W, C, K, R, S, stride, pad, dil, Ho, Wo;
    int M, nks, cch, n_tiles;
};

constexpr float X3_LO_INV = 1.f / 2048.f;

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <int BN>
__global__ __launch_bounds__(512, 1) void conv_x3_kernel(X3Args a) {
    constexpr int BM = 256, WM = 4, WN = 2;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    constexpr int ROW = 128;                       // bytes per LDS row
    constexpr int STAGE = (BM + BN) * ROW;
    constexpr int GA = BM / 64, GB = BN / 64;      // DMA instructions per thread per stage
    constexpr int GL = GA + GB;
    static_assert(TN >= 1 && GB >= 1, "BN must be a multiple of 64");
    __shared__ __attribute__((aligned(1024))) char smem[3 * STAGE];

    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mt = tile / a.n_tiles, nt = tile - mt * a.n_tiles;
    const int m0 = mt * BM, n0 = nt * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w % WN;

    // ---- DMA source bookkeeping (rows this lane feeds) ----
    const int cstride = a.cch * 64;                // halves per pixel
    // per row: image-space origin (hb, wb) of its receptive field and the base
    // pointer of that (possibly padded-out) origin pixel; a tap adds a
    // wave-uniform offset.  Rows past M get an origin that is never in-bounds.
    int a_hb[GA], a_wb[GA];
    const _Float16* a_p[GA];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int row = 8 * (w * GA + i) + (lane >> 3);
        const int L = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
        const int m = m0 + row;
        if (m < a.M) {
            const int hw = a.Ho * a.Wo;
            const int n = m / hw, rem = m - n * hw;
            const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
            a_hb[i] = ho * a.stride - a.pad;
            a_wb[i] = wo * a.stride - a.pad;
            a_p[i] = a.xs + (((long)n * a.H + a_hb[i]) * a.W + a_wb[i]) * cstride + L;
        } else {
            a_hb[i] = -(1 << 28);
            a_wb[i] = -(1 << 28);
            a_p[i] = a.xs;
        }
    }
    const _Float16* b_src[GB];
#pragma unroll
    for (int j = 0; j < GB; ++j) {
        const int row = 8 * (w * GB + j) + (lane >> 3);
        const int L = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
        b_src[j] = a.ws + (long)(n0 + row) * a.nks * 64 + L;
    }
    const _Float16* zero = (const _Float16*)g_x3_zero_line;

    auto issue = [&](int t) {
        char* st = smem + (t % 3) * STAGE;
        const int tap = t / a.cch;
        const int cc = t - tap * a.cch;
        const int rr = tap / a.S, ss = tap - rr * a.S;
        const int dh = rr * a.dil, dw = ss * a.dil;
        const long toff = ((long)dh * a.W + dw) * cstride + cc * 64;
#pragma unroll
        for (int i = 0; i < GA; ++i) {
            const bool in = (unsigned)(a_hb[i] + dh) < (unsigned)a.H && (unsigned)(a_wb[i] + dw) < (unsigned)a.W;
            glds16(in ? a_p[i] + toff : zero, st + (8 * (w * GA + i)) * ROW);
        }
#pragma unroll
        for (int j = 0; j < GB; ++j) glds16(b_src[j] + (long)t * 64, st + (BM + 8 * (w * GB + j)) * ROW);
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

    // fragment read offsets: lane reads row (lane&31) of each 32-row tile, logical
    // chunk 4*plane + 2*s + (lane>>5), stored at chunk ^ ((row>>1)&7)
    const int frow = lane & 31, sw = (frow >> 1) & 7, kh = lane >> 5;
    int foff[2][2];
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int s = 0; s < 2; ++s) foff[pl][s] = frow * ROW + (((4 * pl + 2 * s + kh) ^ sw) << 4);
    const int a_base = (wm * TM * 32) * ROW, b_base = (BM + wn * TN * 32) * ROW;

    const int nks = a.nks;
    issue(0);
    if (nks > 1) issue(1);
    for (int t = 0; t < nks; ++t) {
        if (t + 1 < nks) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();      // stage t landed for every wave; stage t-1 fully read
        if (t + 2 < nks) issue(t + 2);
        const char* st = smem + (t % 3) * STAGE;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            f16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                ah[i] = *(const f16x8*)(st + a_base + i * 32 * ROW + foff[0][s]);
                al[i] = *(const f16x8*)(st + a_base + i * 32 * ROW + foff[1][s]);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                bh[j] = *(const f16x8*)(st + b_base + j * 32 * ROW + foff[0][s]);
                bl[j] = *(const f16x8*)(st + b_base + j * 32 * ROW + foff[1][s]);
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
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] += accc[i][j][r] * X3_LO_INV;

    // ---- epilogue: NHWC store + BN partials per 128-row tile ----
    const int rbase = m0 + wm * TM * 32 + 4 * kh;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * TN * 32 + j * 32 + frow;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                if (m < a.M) a.y[(long)m * a.K + n] = acc[i][j][r];
            }
        }
    if (a.part == nullptr) return;
    __syncthreads();                       // every wave done reading the ring
    float* red = (float*)smem;             // [WM][BN] column sums, then [2][BN] half-tile means
    float* tmean = red + WM * BN;
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
    const long tile128 = (long)(m0 >> 7);
    if (tid < 2 * BN) {
        const int h = tid / BN, c = tid - h * BN;
        const int cnt = min(128, a.M - (m0 + 128 * h));
        if (cnt > 0) {
            const float s = red[(2 * h) * BN + c] + red[(2 * h + 1) * BN + c];
            tmean[h * BN + c] = s / (float)cnt;
            a.part[((tile128 + h) * a.K + n0 + c) * 2 + 0] = s;
        }
    }
    __syncthreads();
    const float* mu_h = tmean + (wm >> 1) * BN;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const float mu = mu_h[wn * TN * 32 + j * 32 + frow];
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
    if (tid < 2 * BN) {
        const int h = tid / BN, c = tid - h * BN;
        if (a.M - (m0 + 128 * h) > 0)
            a.part[((tile128 + h) * a.K + n0 + c) * 2 + 1] = red[(2 * h) * BN + c] + red[(2 * h + 1) * BN + c];
    }
}

// w[k][tap][c] fp32 (KRSC) → ws[k][tap][c/32][hi32|lo32]; element e → 2e - (c&31) (+32 for lo)
__global__ __launch_bounds__(256) void weight_pack_x3_kernel(long n, const float* __restrict__ w,
                                                            _Float16* __restrict__ ws) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const float v = w[e];
        const _Float16 h = (_Float16)v;
        const long o = 2 * e - (e & 31);
        ws[o] = h;
        ws[o + 32] = (_Float16)((v - (float)h) * SPLIT_LO_SCALE);
    }
}

}  // namespace hkp

using namespace hkp;

extern "C" int hkp_weight_pack_x3(int64_t n, int32_t c, const float* w, uint16_t* w_split, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && c > 0 && c % 32 == 0 && n % c == 0 && w && w_split, "hkp_weight_pack_x3: bad args");
    long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(weight_pack_x3_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), (long)n, w,
                       (_Float16*)w_split);
    HKP_LAUNCH_CHECK("hkp_weight_pack_x3");
    return HKP_OK;
}

extern "C" int hkp_conv2d_fwd_x3(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* w_split, float* y,
                                 float* stat_partials, hkp_stream_t stream) {
    int ho, wo;
    int rc = hkp_conv_out_hw(d, &ho, &wo);
    if (rc) return rc;
    HKP_CHECK_ARG(x_split && w_split && y, "hkp_conv2d_fwd_x3: null tensor");
    HKP_CHECK_ARG(d->in_layout == HKP_LAYOUT_NHWC, "hkp_conv2d_fwd_x3: NHWC only");
    HKP_CHECK_ARG(d->c % 32 == 0 && d->k % 64 == 0, "hkp_conv2d_fwd_x3: need Cin%%32==0, Cout%%64==0 (c=%d k=%d)",
                  d->c, d->k);
    const long M = (long)d->n * ho * wo;
    HKP_CHECK_ARG(M < (1L << 31) && (long)d->n * d->h * d->w * d->c < (1L << 40), "hkp_conv2d_fwd_x3: too large");
    X3Args a;
    a.xs = (const _Float16*)x_split; a.ws = (const _Float16*)w_split; a.y = y; a.part = stat_partials;
    a.N = d->n; a.H = d->h; a.W = d->w; a.C = d->c; a.K = d->k; a.R = d->r; a.S = d->s;
    a.stride = d->stride; a.pad = d->pad; a.dil = d->dilation; a.Ho = ho; a.Wo = wo;
    a.M = (int)M; a.cch = d->c / 32; a.nks = d->r * d->s * a.cch;
    const int bn = d->k % 128 == 0 ? 128 : 64;
    a.n_tiles = d->k / bn;
    const long m_tiles = (M + 255) / 256;
    hipStream_t st = as_stream(stream);
    if (bn == 128) hipLaunchKernelGGL(conv_x3_kernel<128>, dim3(m_tiles * a.n_tiles), dim3(512), 0, st, a);
    else hipLaunchKernelGGL(conv_x3_kernel<64>, dim3(m_tiles * a.n_tiles), dim3(512), 0, st, a);
    HKP_LAUNCH_CHECK("hkp_conv2d_fwd_x3");
    return HKP_OK;
}
