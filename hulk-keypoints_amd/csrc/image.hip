// Image-side kernels around the heatmap path:
//   * ToTensor on the device (dataset.py:16,71): uint8 HWC BGR → fp32 NCHW / 255;
//   * the keypoint visualisation of Prediction.plot (prediction.py:40-66) —
//     per-heatmap min-max normalisation to uint8 (cv2.normalize NORM_MINMAX),
//     JET colour map, 0.65·image + 0.35·map blend, a dot at the argmax, tiled
//     into the reference's two-column grid — so no [B,K,H,W] heatmap crosses PCIe
//     for plotting.  Arithmetic is the package's numpy restatement of plot()
//     (src/prediction.py, used when OpenCV is absent), step for step in fp32 with
//     truncating uint8 casts, so the two agree bit for bit.
#include "common.h"

namespace hkp {

__global__ __launch_bounds__(256) void u8_to_nchw_kernel(long total, int C, int HW, const uint8_t* __restrict__ img,
                                                        float* __restrict__ x) {
    // one thread per output element of x [n][c][h*w]; reads are C-strided bytes
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const long p = i % HW, nc = i / HW;
        const int c = (int)(nc % C);
        const long n = nc / C;
        x[i] = __fdiv_rn((float)img[(n * HW + p) * C + c], 255.f);
    }
}

// per-plane (min, max) of heat [planes][HW]; one block per plane
__global__ __launch_bounds__(256) void plane_minmax_kernel(long HW, const float* __restrict__ heat,
                                                          float* __restrict__ mm) {
    __shared__ float rmin[4], rmax[4];
    const float* h = heat + (long)blockIdx.x * HW;
    float lo = INFINITY, hi = -INFINITY;
    for (long i = threadIdx.x; i < HW; i += 256) {
        const float v = h[i];
        lo = fminf(lo, v);
        hi = fmaxf(hi, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, o));
        hi = fmaxf(hi, __shfl_xor(hi, o));
    }
    if ((threadIdx.x & 63) == 0) {
        rmin[threadIdx.x >> 6] = lo;
        rmax[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        mm[2 * blockIdx.x] = fminf(fminf(rmin[0], rmin[1]), fminf(rmin[2], rmin[3]));
        mm[2 * blockIdx.x + 1] = fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]));
    }
}

__device__ __forceinline__ uint8_t jet_channel(float x, float centre) {
    // clip(1.5 - |4x - centre|, 0, 1) * 255, truncated
    const float t = fminf(fmaxf(__fsub_rn(1.5f, fabsf(__fsub_rn(__fmul_rn(4.f, x), centre))), 0.f), 1.f);
    return (uint8_t)__fmul_rn(t, 255.f);
}

// Half-width of row |d| of a filled circle of radius r as OpenCV's cv::circle
// draws it (thickness -1, LINE_8, no shift → the midpoint "Circle" rasteriser of
// imgproc/drawing.cpp: per step (dx, dy) rows ±dy span ±dx and rows ±dx span ±dy)
// — prediction.py:52 cv2.circle(overlay, (x, y), 4, (0, 0, 0), -1).  -1: outside.
__host__ __device__ inline int disc_halfwidth(int r, int d) {
    if (d < 0) d = -d;
    int hw = -1, err = 0, dx = r, dy = 0, plus = 1, minus = (r << 1) - 1;
    while (dx >= dy) {
        if (d == dy && dx > hw) hw = dx;
        if (d == dx && dy > hw) hw = dy;
        ++dy;
        err += plus;
        plus += 2;
        const int mask = (err <= 0) - 1;
        err -= minus & mask;
        dx += mask;
        minus -= mask & 2;
    }
    return hw;
}

// out [n][rows][cols][3]: keypoint plane k sits in column k / half (half = K/2;
// K == 1: one column), row block k % half.  Per pixel, as prediction.py:47-52:
//   u   = uint8(float(v * s + t)) with s = 255 / (max - min), t = -min * s in
//         double (cv2.normalize NORM_MINMAX into float32, then .astype(uint8));
//   vis = JET(u) (BGR; the analytic JET — cv2's LUT is not available here);
//   out = round(0.65 * img + 0.35 * vis) saturated (cv2.addWeighted);
//   the filled radius-4 disc at the argmax (cv2.circle) is black.
__global__ __launch_bounds__(256) void heat_overlay_kernel(int N, int K, int H, int W, int half,
                                                          const float* __restrict__ heat,
                                                          const uint8_t* __restrict__ img,
                                                          const int32_t* __restrict__ yx,
                                                          const float* __restrict__ mm, uint8_t* __restrict__ out) {
    const int cols = K == 1 ? 1 : 2;
    const long total = (long)N * K * H * W;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int x = (int)(i % W);
        long t = i / W;
        const int y = (int)(t % H);
        t /= H;
        const int k = (int)(t % K);
        const int n = (int)(t / K);
        const long plane = (long)n * K + k;
        const double mn = mm[2 * plane], mx = mm[2 * plane + 1];
        const double sc = mx - mn > 2.220446049250313e-16 ? 255.0 / (mx - mn) : 0.0;
        const double sh = 0.0 - mn * sc;
        const float v = heat[(plane * H + y) * W + x];
        const float nv = (float)((double)v * sc + sh);
        const uint8_t u = (uint8_t)fminf(fmaxf(nv, 0.f), 255.f);
        const float xn = __fdiv_rn((float)u, 255.f);
        const uint8_t vis[3] = {jet_channel(xn, 1.f), jet_channel(xn, 2.f), jet_channel(xn, 3.f)};   // B, G, R
        const int py = yx[2 * plane], px = yx[2 * plane + 1];
        const int hw = abs(y - py) <= 4 ? disc_halfwidth(4, y - py) : -1;
        const bool dot = hw >= 0 && abs(x - px) <= hw;
        const int col = K == 1 ? 0 : k / half, rb = K == 1 ? 0 : k % half;
        uint8_t* o = out + ((((long)n * (H * (K == 1 ? 1 : half)) + rb * H + y) * (cols * W)) + col * W + x) * 3;
        const uint8_t* im = img + (((long)n * H + y) * W + x) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float b = rintf(__fadd_rn(__fmul_rn(0.65f, (float)im[c]), __fmul_rn(0.35f, (float)vis[c])));
            o[c] = dot ? 0 : (uint8_t)fminf(fmaxf(b, 0.f), 255.f);
        }
    }
}

// Soft-argmax of each heatmap plane with the reference's index mapping FIXED
// (prediction.py:31-38 builds x from i % width over d.T.ravel(), i.e. mixes the
// axes, and its result is discarded at :45): p = softmax(beta * h) over the
// plane, out = (sum p * x, sum p * y) in fp64, fixed-order block reduction
// (deterministic).  One block per plane.
__global__ __launch_bounds__(256) void soft_argmax_kernel(int H, int W, float beta, const float* __restrict__ heat,
                                                         float* __restrict__ out_xy) {
    __shared__ double red[4][3];
    __shared__ float mxs[4];
    const long HW = (long)H * W;
    const float* h = heat + (long)blockIdx.x * HW;
    float m = -INFINITY;
    for (long i = threadIdx.x; i < HW; i += 256) m = fmaxf(m, beta * h[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) mxs[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(mxs[0], mxs[1]), fmaxf(mxs[2], mxs[3]));
    double s = 0.0, sx = 0.0, sy = 0.0;
    for (long i = threadIdx.x; i < HW; i += 256) {
        const double e = exp((double)(beta * h[i] - m));
        s += e;
        sx += e * (double)(i % W);
        sy += e * (double)(i / W);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        sx += __shfl_xor(sx, o);
        sy += __shfl_xor(sy, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = s;
        red[threadIdx.x >> 6][1] = sx;
        red[threadIdx.x >> 6][2] = sy;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double S = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
        out_xy[2 * blockIdx.x] = (float)(((red[0][1] + red[1][1]) + (red[2][1] + red[3][1])) / S);
        out_xy[2 * blockIdx.x + 1] = (float)(((red[0][2] + red[1][2]) + (red[2][2] + red[3][2])) / S);
    }
}

static inline unsigned grid_of(long work) {
    long g = (work + 255) / 256;
    return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace hkp

using namespace hkp;

extern "C" int hkp_images_u8_to_nchw(int32_t n, int32_t h, int32_t w, int32_t c, const uint8_t* img_nhwc,
                                     float* x_nchw, hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && h > 0 && w > 0 && c > 0 && img_nhwc && x_nchw, "hkp_images_u8_to_nchw: bad args");
    const long total = (long)n * c * h * w;
    hipLaunchKernelGGL(u8_to_nchw_kernel, dim3(grid_of(total)), dim3(256), 0, as_stream(stream), total, c, h * w,
                       img_nhwc, x_nchw);
    HKP_LAUNCH_CHECK("hkp_images_u8_to_nchw");
    return HKP_OK;
}

extern "C" int hkp_heat_overlay(int32_t n, int32_t k, int32_t H, int32_t W, const float* heat,
                                const uint8_t* img_nhwc, const int32_t* argmax_yx, float* minmax_ws, uint8_t* out,
                                hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && k > 0 && H > 0 && W > 0, "hkp_heat_overlay: bad sizes");
    HKP_CHECK_ARG(k == 1 || k % 2 == 0, "hkp_heat_overlay: K must be 1 or even (two equal columns, k=%d)", k);
    HKP_CHECK_ARG(heat && img_nhwc && argmax_yx && minmax_ws && out, "hkp_heat_overlay: null tensor");
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(plane_minmax_kernel, dim3((unsigned)(n * k)), dim3(256), 0, st, (long)H * W, heat, minmax_ws);
    HKP_LAUNCH_CHECK("hkp_heat_overlay(minmax)");
    const long total = (long)n * k * H * W;
    hipLaunchKernelGGL(heat_overlay_kernel, dim3(grid_of(total)), dim3(256), 0, st, n, k, H, W, k == 1 ? 1 : k / 2,
                       heat, img_nhwc, argmax_yx, minmax_ws, out);
    HKP_LAUNCH_CHECK("hkp_heat_overlay");
    return HKP_OK;
}

extern "C" int hkp_soft_argmax(int32_t n, int32_t k, int32_t H, int32_t W, float beta, const float* heat, float* out_xy,
                               hkp_stream_t stream) {
    HKP_CHECK_ARG(n > 0 && k > 0 && H > 0 && W > 0 && heat && out_xy, "hkp_soft_argmax: bad args");
    hipLaunchKernelGGL(soft_argmax_kernel, dim3((unsigned)(n * k)), dim3(256), 0, as_stream(stream), H, W, beta, heat,
                       out_xy);
    HKP_LAUNCH_CHECK("hkp_soft_argmax");
    return HKP_OK;
}
