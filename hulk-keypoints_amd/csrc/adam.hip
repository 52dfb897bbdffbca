// Fused multi-tensor Adam (L2 weight decay) — SURVEY §8(f2): the optimizer step of
// train.py:36 (optim.Adam(lr=1e-4, weight_decay=1e-4), train.py:79) as one pass
// over every parameter: read p, g, m, v; write p, m, v (28 B per element, HBM-bound)
// in a handful of launches instead of torch's ~10 foreach kernels per tensor group.
//
// Per element, the operation sequence of torch.optim.Adam's multi-tensor path
// (torch/optim/adam.py _multi_tensor_adam, amsgrad=False, maximize=False):
//     g  = g + wd * p                      _foreach_add(grads, params, alpha=wd)
//     m  = m + (1 - b1) * (g - m)          _foreach_lerp_(exp_avgs, grads, 1 - b1)
//     v  = v * b2 + (1 - b2) * g * g       _foreach_mul_ / _foreach_addcmul_
//     d  = sqrt(v) / sqrt(bc2) + eps       _foreach_sqrt / _foreach_div_ / _foreach_add_
//     p  = p + (-lr / bc1) * m / d         _foreach_addcdiv_
// with 1 - b1, 1 - b2, bc1 = 1 - b1^step, bc2 = 1 - b2^step computed on the host
// in double (as torch does: its scalars are Python floats) and passed as fp32.
#include "common.h"

namespace hkp {

constexpr int ADAM_MAXT = 48;
constexpr int ADAM_UNIT = 4096;   // elements per block (256 threads x 4 float4)

struct AdamT {
    float* p;
    const float* g;
    float* m;
    float* v;
    long n;
};

struct AdamTable {
    AdamT t[ADAM_MAXT];
    int ubeg[ADAM_MAXT + 1];
    int n;
    float b2, omb1, omb2, eps, wd, neg_step, bc2_sqrt;   // omb = 1 - beta (host double → fp32)
};

// a + s*b as one rounding where ATen's CUDA functors contract (a + scalar*x →
// fma): the weight-decay add, the lerp, addcmul and addcdiv
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamTable& a) {
    g = __fmaf_rn(a.wd, p, g);
    m = __fmaf_rn(a.omb1, __fsub_rn(g, m), m);
    v = __fmaf_rn(a.omb2, __fmul_rn(g, g), __fmul_rn(v, a.b2));
    const float d = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), a.bc2_sqrt), a.eps);
    p = __fmaf_rn(a.neg_step, __fdiv_rn(m, d), p);
}

__global__ __launch_bounds__(256) void adam_kernel(const AdamTable a) {
    int j = 0;
    while (j + 1 < a.n && (int)blockIdx.x >= a.ubeg[j + 1]) ++j;
    const AdamT& T = a.t[j];
    const long base = (long)(blockIdx.x - a.ubeg[j]) * ADAM_UNIT;
    const bool vec = ((T.n & 3) == 0) && ((((uintptr_t)T.p | (uintptr_t)T.g | (uintptr_t)T.m | (uintptr_t)T.v) & 15) == 0);
    if (vec) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const long i = base + 4L * (threadIdx.x + 256 * q);
            if (i >= T.n) break;
            f32x4 p = *(const f32x4*)(T.p + i), g = *(const f32x4*)(T.g + i);
            f32x4 m = *(const f32x4*)(T.m + i), v = *(const f32x4*)(T.v + i);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float pe = p[e], me = m[e], ve = v[e];
                adam_elem(pe, g[e], me, ve, a);
                p[e] = pe;
                m[e] = me;
                v[e] = ve;
            }
            *(f32x4*)(T.p + i) = p;
            *(f32x4*)(T.m + i) = m;
            *(f32x4*)(T.v + i) = v;
        }
    } else {
        for (long i = base + threadIdx.x; i < base + ADAM_UNIT && i < T.n; i += 256) {
            float p = T.p[i], m = T.m[i], v = T.v[i];
            adam_elem(p, T.g[i], m, v, a);
            T.p[i] = p;
            T.m[i] = m;
            T.v[i] = v;
        }
    }
}

}  // namespace hkp

using namespace hkp;

extern "C" int hkp_adam_step(int32_t ntensors, const hkp_adam_tensor* tensors, float beta2, float one_minus_beta1,
                             float one_minus_beta2, float eps, float weight_decay, float neg_step_size,
                             float bias_correction2_sqrt, hkp_stream_t stream) {
    HKP_CHECK_ARG(ntensors >= 0 && (ntensors == 0 || tensors), "hkp_adam_step: bad tensor list");
    HKP_CHECK_ARG(bias_correction2_sqrt > 0.f, "hkp_adam_step: bias_correction2_sqrt must be > 0");
    for (int i = 0; i < ntensors; ++i) {
        const hkp_adam_tensor& t = tensors[i];
        HKP_CHECK_ARG(t.n >= 0 && (t.n == 0 || (t.param && t.grad && t.exp_avg && t.exp_avg_sq)),
                      "hkp_adam_step: tensor %d: null pointer", i);
        HKP_CHECK_ARG((t.n + ADAM_UNIT - 1) / ADAM_UNIT < (1L << 30), "hkp_adam_step: tensor %d too large", i);
    }
    hipStream_t st = as_stream(stream);
    for (int i0 = 0; i0 < ntensors; i0 += ADAM_MAXT) {
        AdamTable a;
        a.n = 0;
        a.b2 = beta2; a.omb1 = one_minus_beta1; a.omb2 = one_minus_beta2; a.eps = eps; a.wd = weight_decay;
        a.neg_step = neg_step_size; a.bc2_sqrt = bias_correction2_sqrt;
        long units = 0;
        for (int i = i0; i < ntensors && i < i0 + ADAM_MAXT; ++i) {
            const hkp_adam_tensor& s = tensors[i];
            if (s.n == 0) continue;
            AdamT& d = a.t[a.n];
            d.p = s.param; d.g = s.grad; d.m = s.exp_avg; d.v = s.exp_avg_sq; d.n = s.n;
            a.ubeg[a.n++] = (int)units;
            units += (s.n + ADAM_UNIT - 1) / ADAM_UNIT;
        }
        if (units == 0) continue;
        HKP_CHECK_ARG(units < (1L << 31), "hkp_adam_step: too many elements in one launch");
        a.ubeg[a.n] = (int)units;
        hipLaunchKernelGGL(adam_kernel, dim3((unsigned)units), dim3(256), 0, st, a);
        HKP_LAUNCH_CHECK("hkp_adam_step");
    }
    return HKP_OK;
}
