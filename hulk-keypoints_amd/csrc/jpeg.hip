// Device half of the hybrid JPEG decode (include/hkp_jpeg.h): the entropy-decoded
// coefficients of a batch of same-geometry images → uint8 [n][H][W][3] BGR, the
// image cv2.imread gives (/root/reference/src/dataset.py:71).
//
// Integer arithmetic of libjpeg-turbo's default decode (oracle/jpeg_ref.py
// restates it and cites the IJG sources): jidctint.c's islow IDCT, jdsample.c's
// fancy (triangle) upsampling, jdcolor.c's YCbCr → RGB tables.  Bit-exact by
// construction; tests/test_gpu_jpeg.py compares with Pillow's libjpeg-turbo.
//
// Two launches, both HBM-light (a 640x480 4:2:0 image is 0.9 MB of coefficients
// and 0.9 MB of output):
//   jpeg_idct_kernel   8 lanes per 8x8 block: lane j dequantises and transforms
//                      column j, the column results meet in LDS, lane j then
//                      transforms row j and stores its 8 samples (one 8-B store)
//                      into the component plane [bh*8][bw*8]
//   jpeg_color_kernel  one lane per 4 output pixels: upsamples each component at
//                      those pixels from the planes (L2-resident), converts, and
//                      writes 12 bytes of BGR
#include "common.h"
#include "../../include/hkp_jpeg.h"

namespace hkp {

namespace {

constexpr int CONST_BITS = 13, PASS1_BITS = 2;

struct JpegGeomDev {
    int width, height, ncomp;
    int fh[3], fv[3];              // upsampling factor of each component (1 or 2)
    int bw[3], bh[3], dw[3], dh[3];
    long blk_off[3];
    long nblocks;
    long plane_off[3];             // byte offset of each component plane within an image's planes
    long plane_bytes;              // all planes of one image
};

__device__ __forceinline__ long descale(long x, int n) { return (x + (1L << (n - 1))) >> n; }

// jidctint.c's 1-D kernel (even part from s0, s2, s4, s6; odd part from s1, s3,
// s5, s7); outputs before descaling
__device__ __forceinline__ void idct_1d(const long s[8], long o[8]) {
    long z1 = (s[2] + s[6]) * 4433;                      // FIX_0_541196100
    const long tmp2 = z1 + s[6] * (-15137);              // - FIX_1_847759065
    const long tmp3 = z1 + s[2] * 6270;                  // FIX_0_765366865
    const long tmp0 = (s[0] + s[4]) << CONST_BITS;
    const long tmp1 = (s[0] - s[4]) << CONST_BITS;
    const long tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    long t0 = s[7], t1 = s[5], t2 = s[3], t3 = s[1];
    z1 = t0 + t3;
    long z2 = t1 + t2, z3 = t0 + t2, z4 = t1 + t3;
    const long z5 = (z3 + z4) * 9633;                    // FIX_1_175875602
    t0 *= 2446;                                          // FIX_0_298631336
    t1 *= 16819;                                         // FIX_2_053119869
    t2 *= 25172;                                         // FIX_3_072711026
    t3 *= 12299;                                         // FIX_1_501321110
    z1 *= -7373;                                         // - FIX_0_899976223
    z2 *= -20995;                                        // - FIX_2_562915447
    z3 = z3 * -16069 + z5;                               // - FIX_1_961570560
    z4 = z4 * -3196 + z5;                                // - FIX_0_390180644
    t0 += z1 + z3;
    t1 += z2 + z4;
    t2 += z2 + z3;
    t3 += z1 + z4;
    o[0] = tmp10 + t3;
    o[7] = tmp10 - t3;
    o[1] = tmp11 + t2;
    o[6] = tmp11 - t2;
    o[2] = tmp12 + t1;
    o[5] = tmp12 - t1;
    o[3] = tmp13 + t0;
    o[4] = tmp13 - t0;
}

// jdmaster.c's post-IDCT range-limit table, indexed by v & 1023
__device__ __forceinline__ unsigned range_limit_idct(long v) {
    const int i = (int)(v & 1023);
    return i < 128 ? i + 128 : i < 512 ? 255 : i < 896 ? 0 : i - 896;
}

constexpr int IDCT_BLOCKS = 32;                          // 8x8 blocks per 256-lane workgroup

__global__ __launch_bounds__(256) void jpeg_idct_kernel(JpegGeomDev g, long total, const short* __restrict__ coefs,
                                                        const unsigned short* __restrict__ qt,
                                                        unsigned char* __restrict__ planes) {
    __shared__ int ws[IDCT_BLOCKS][8][9];                // [block][row][col], padded
    const int jb = threadIdx.x >> 3, j = threadIdx.x & 7;
    const long b = (long)blockIdx.x * IDCT_BLOCKS + jb;
    const bool live = b < total;
    const long img = live ? b / g.nblocks : 0;
    const long lb = live ? b - img * g.nblocks : 0;
    const int c = lb >= g.blk_off[2] && g.ncomp > 2 ? 2 : lb >= g.blk_off[1] && g.ncomp > 1 ? 1 : 0;
    const short* in = coefs + b * 64;
    const unsigned short* q = qt + (img * g.ncomp + c) * 64;
    if (live) {
        // pass 1: column j, results scaled by 2^PASS1_BITS
        long s[8], o[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) s[r] = (long)in[r * 8 + j] * (long)q[r * 8 + j];
        idct_1d(s, o);
#pragma unroll
        for (int r = 0; r < 8; ++r) ws[jb][r][j] = (int)descale(o[r], CONST_BITS - PASS1_BITS);
    }
    __syncthreads();
    if (!live) return;
    // pass 2: row j
    long s[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = ws[jb][j][k];
    idct_1d(s, o);
    unsigned lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        lo |= range_limit_idct(descale(o[k], CONST_BITS + PASS1_BITS + 3)) << (8 * k);
        hi |= range_limit_idct(descale(o[k + 4], CONST_BITS + PASS1_BITS + 3)) << (8 * k);
    }
    const long k0 = lb - g.blk_off[c];
    const long by = k0 / g.bw[c], bx = k0 - by * g.bw[c];
    unsigned char* dst = planes + img * g.plane_bytes + g.plane_off[c] + (by * 8 + j) * (long)g.bw[c] * 8 + bx * 8;
    *(uint2*)dst = make_uint2(lo, hi);
}

// one component's sample at full-resolution pixel (x, y): jdsample.c
__device__ __forceinline__ int up_sample(const unsigned char* p, int pitch, int dw, int dh, int fh, int fv, int x,
                                         int y) {
    if (fh == 1) return p[(long)y * pitch + x];
    const int cx = x >> 1, px = x & 1;
    if (dw <= 2) return p[(long)(y / fv) * pitch + cx];    // box upsampling
    if (fv == 1) {                                       // h2v1_fancy_upsample
        const unsigned char* r = p + (long)y * pitch;
        const int v3 = 3 * r[cx];
        if (px == 0) return cx == 0 ? r[0] : (v3 + r[cx - 1] + 1) >> 2;
        return cx == dw - 1 ? r[cx] : (v3 + r[cx + 1] + 2) >> 2;
    }
    // h2v2_fancy_upsample: column sums with the row above (even y) / below (odd y)
    const int cy = y >> 1;
    const int ny = (y & 1) ? min(cy + 1, dh - 1) : max(cy - 1, 0);
    const unsigned char* r0 = p + (long)cy * pitch;
    const unsigned char* r1 = p + (long)ny * pitch;
    const int cs = 3 * r0[cx] + r1[cx];
    if (px == 0) return cx == 0 ? (4 * cs + 8) >> 4 : (3 * cs + 3 * r0[cx - 1] + r1[cx - 1] + 8) >> 4;
    return cx == dw - 1 ? (4 * cs + 7) >> 4 : (3 * cs + 3 * r0[cx + 1] + r1[cx + 1] + 7) >> 4;
}

__device__ __forceinline__ unsigned char clamp255(int v) { return (unsigned char)min(max(v, 0), 255); }

__global__ __launch_bounds__(256) void jpeg_color_kernel(JpegGeomDev g, int n, const unsigned char* __restrict__ planes,
                                                         unsigned char* __restrict__ out) {
    const int qw = (g.width + 3) / 4;                   // pixel quads per row
    const long quads = (long)n * g.height * qw;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < quads; t += stride) {
        const long img = t / ((long)g.height * qw);
        const long rem = t - img * g.height * qw;
        const int y = (int)(rem / qw), x0 = (int)(rem - (long)y * qw) * 4;
        const unsigned char* base = planes + img * g.plane_bytes;
        unsigned char* o = out + ((img * g.height + y) * (long)g.width + x0) * 3;
        const int nx = min(4, g.width - x0);
        for (int k = 0; k < nx; ++k) {
            const int x = x0 + k;
            const int Y = up_sample(base + g.plane_off[0], g.bw[0] * 8, g.dw[0], g.dh[0], g.fh[0], g.fv[0], x, y);
            if (g.ncomp == 1) {
                o[3 * k] = o[3 * k + 1] = o[3 * k + 2] = (unsigned char)Y;
                continue;
            }
            const int cb = up_sample(base + g.plane_off[1], g.bw[1] * 8, g.dw[1], g.dh[1], g.fh[1], g.fv[1], x, y) - 128;
            const int cr = up_sample(base + g.plane_off[2], g.bw[2] * 8, g.dw[2], g.dh[2], g.fh[2], g.fv[2], x, y) - 128;
            // jdcolor.c ycc_rgb_convert: SCALEBITS 16, ONE_HALF rounding
            const int r = Y + ((91881 * cr + 32768) >> 16);
            const int gg = Y + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
            const int b = Y + ((116130 * cb + 32768) >> 16);
            o[3 * k] = clamp255(b);
            o[3 * k + 1] = clamp255(gg);
            o[3 * k + 2] = clamp255(r);
        }
    }
}

bool geom_dev(const hkpj_geom* g, JpegGeomDev* d) {
    if (g->ncomp != 1 && g->ncomp != 3) return false;
    d->width = g->width;
    d->height = g->height;
    d->ncomp = g->ncomp;
    d->nblocks = g->nblocks;
    long off = 0;
    for (int c = 0; c < 3; ++c) {
        if (c >= g->ncomp) {
            d->fh[c] = d->fv[c] = 1;
            d->bw[c] = d->bh[c] = d->dw[c] = d->dh[c] = 0;
            d->blk_off[c] = g->nblocks;
            d->plane_off[c] = off;
            continue;
        }
        if (g->hs[c] < 1 || g->vs[c] < 1 || g->hmax % g->hs[c] || g->vmax % g->vs[c]) return false;
        d->fh[c] = g->hmax / g->hs[c];
        d->fv[c] = g->vmax / g->vs[c];
        if (d->fh[c] > 2 || d->fv[c] > d->fh[c]) return false;
        d->bw[c] = g->bw[c];
        d->bh[c] = g->bh[c];
        d->dw[c] = g->dw[c];
        d->dh[c] = g->dh[c];
        if ((long)g->bw[c] * 8 < g->dw[c] || (long)g->bh[c] * 8 < g->dh[c] || g->dw[c] * d->fh[c] < g->width ||
            g->dh[c] * d->fv[c] < g->height)
            return false;
        d->blk_off[c] = g->blk_off[c];
        d->plane_off[c] = off;
        off += (long)g->bw[c] * 8 * g->bh[c] * 8;
    }
    d->plane_bytes = off;
    return g->blk_off[0] == 0 &&
           (g->ncomp == 1 || (g->blk_off[1] == (long)g->bw[0] * g->bh[0] &&
                              g->blk_off[2] == g->blk_off[1] + (long)g->bw[1] * g->bh[1])) &&
           g->nblocks == d->plane_bytes / 64;
}

}  // namespace

}  // namespace hkp

using namespace hkp;

extern "C" int64_t hkp_jpeg_planes_bytes(const hkpj_geom* g) {
    JpegGeomDev d;
    if (!g || !geom_dev(g, &d)) return -1;
    return d.plane_bytes;
}

extern "C" int hkp_jpeg_reconstruct(int32_t n, const hkpj_geom* g, const int16_t* coefs, const uint16_t* qt,
                                    uint8_t* planes, int64_t planes_bytes, uint8_t* out_bgr, hkp_stream_t stream) {
    HKP_CHECK_ARG(g && coefs && qt && planes && out_bgr && n > 0, "hkp_jpeg_reconstruct: null argument");
    JpegGeomDev d;
    HKP_CHECK_ARG(geom_dev(g, &d), "hkp_jpeg_reconstruct: unsupported or inconsistent geometry");
    HKP_CHECK_ARG(planes_bytes >= (int64_t)n * d.plane_bytes, "hkp_jpeg_reconstruct: planes workspace %ld < %ld",
                  (long)planes_bytes, (long)n * d.plane_bytes);
    hipStream_t st = as_stream(stream);
    const long total = (long)n * d.nblocks;
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((total + IDCT_BLOCKS - 1) / IDCT_BLOCKS)), dim3(256), 0, st, d,
                       total, (const short*)coefs, (const unsigned short*)qt, (unsigned char*)planes);
    HKP_LAUNCH_CHECK("hkp_jpeg_reconstruct (idct)");
    const long quads = (long)n * d.height * ((d.width + 3) / 4);
    const long grid = std::min<long>((quads + 255) / 256, 8192);
    hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)grid), dim3(256), 0, st, d, (int)n,
                       (const unsigned char*)planes, (unsigned char*)out_bgr);
    HKP_LAUNCH_CHECK("hkp_jpeg_reconstruct (color)");
    return HKP_OK;
}
