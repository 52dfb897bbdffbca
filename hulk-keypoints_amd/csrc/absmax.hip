// max |x| (hkp_absmax): the power-of-two gradient scale source of the f16x3
// backward convs when no BN-backward bound is at hand (include/hulkkp.h).
#include "common.h"

namespace hkp {

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

}  // namespace hkp

using namespace hkp;

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
