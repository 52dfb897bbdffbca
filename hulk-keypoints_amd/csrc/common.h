// Shared helpers for the libhulkkp HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include "../../include/hulkkp.h"
#ifdef HKP_AB_KNOBS
#include "../../include/hulkkp_ab.h"
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace hkp {

// A/B instruments (tools/ only): the process-global knobs and their hkp_debug_*
// setters (include/hulkkp_ab.h) exist only in the -DHKP_AB_KNOBS build (`make ab`
// -> tools/ab_lib/libhulkkp_ab.so); the product library compiles each knob as a
// constant at its default, so it keeps no process-global switches
#ifdef HKP_AB_KNOBS
#define HKP_AB_KNOB(T, name, dflt) static T name = dflt
#else
#define HKP_AB_KNOB(T, name, dflt) static constexpr T name = dflt
#endif

// thread-local last-error message (hkp_last_error)
void set_error(const char* fmt, ...);

#define HKP_CHECK_ARG(cond, ...)                  \
    do {                                          \
        if (!(cond)) {                            \
            ::hkp::set_error(__VA_ARGS__);        \
            return HKP_ERR_BAD_ARG;               \
        }                                         \
    } while (0)

#define HKP_LAUNCH_CHECK(what)                                                      \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) {                                                     \
            ::hkp::set_error("%s: launch failed: %s", what, hipGetErrorString(e_)); \
            return (int)e_;                                                         \
        }                                                                           \
    } while (0)

static inline hipStream_t as_stream(hkp_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// XCD-aware bijective remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD (one L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));

// Operand split of 4 consecutive channels (element index e4*4, C % 32 == 0) for
// the next conv: passes 1 → hi plane [P][C]; passes 3 → packed split layout
// [P][C/32][hi32|lo32] (element e → 2e - (e&31), lo 32 halves later) with
// hi = f16(v), lo = f16(v - hi) — the operand format of conv_x3.hip.
__device__ __forceinline__ void store_split4(const f32x4& v, long e4, _Float16* __restrict__ out, int passes) {
    h16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const _Float16 hv = (_Float16)v[e];
        h[e] = hv;
        l[e] = (_Float16)(v[e] - (float)hv);
    }
    if (passes == 1) {
        ((h16x4*)out)[e4] = h;
    } else {
        const long e = e4 * 4, o = 2 * e - (e & 31);
        *(h16x4*)(out + o) = h;
        *(h16x4*)(out + o + 32) = l;
    }
}

// 2^e with e chosen so that amax * 2^e lands in [2^13, 2^14): exact scaling that
// keeps hi inside fp16's range and the (unscaled) lo of large elements normal
__device__ __forceinline__ float pow2_scale_for(const unsigned* amax_bits) {
    if (amax_bits == nullptr) return 1.f;
    const float m = __uint_as_float(*amax_bits);
    if (!(m > 0.f) || !(m < INFINITY)) return 1.f;
    int e;
    frexpf(m, &e);               // m = f * 2^e, f in [0.5, 1)
    e = 14 - e;
    e = e < -100 ? -100 : (e > 100 ? 100 : e);
    return ldexpf(1.f, e);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Per-channel reductions over [tiles][C][2] partials: a block covers CPB
// channels x (256/CPB) tile lanes, so the CPB channels of one tile row are one
// contiguous load (8*CPB bytes) instead of CPB separate sectors; lane sums are
// combined in a fixed order.  CPB chosen so that C/CPB blocks still fill the chip.
static inline int partials_cpb(int C) { return C >= 1024 ? 8 : C >= 512 ? 4 : C >= 256 ? 2 : 1; }
// (the BN finalize kernels take 1024-thread blocks for >= 4096 tiles)

// NW = waves per block (4: the 256-thread finalize; 16: the 1024-thread one for
// long tile lists); the per-wave sums are combined pairwise in a fixed order
template <int CPB, int NW = 4>
__device__ __forceinline__ double lanes_sum_d(double v, double (*red)[8]) {
#pragma unroll
    for (int o = CPB; o < 64; o <<= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, cl = threadIdx.x % CPB;
    __syncthreads();
    if (lane < CPB) red[wid][lane] = v;
    __syncthreads();
    double a[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) a[i] = red[i][cl];
#pragma unroll
    for (int w = NW / 2; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) a[i] = a[2 * i] + a[2 * i + 1];
    return a[0];
}

template <int CPB, int NW = 4>
__device__ __forceinline__ double lanes_max_d(double v, double (*red)[8]) {
#pragma unroll
    for (int o = CPB; o < 64; o <<= 1) v = fmax(v, __shfl_xor(v, o));
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, cl = threadIdx.x % CPB;
    __syncthreads();
    if (lane < CPB) red[wid][lane] = v;
    __syncthreads();
    double m = red[0][cl];
#pragma unroll
    for (int i = 1; i < NW; ++i) m = fmax(m, red[i][cl]);
    return m;
}

// scale/shift, mean/invstd and running statistics of channel c from the merged
// fp64 mean and M2 (sum of squared deviations over all `count` rows)
__device__ __forceinline__ void bn_fin_store(int c, int C, long count, double mean, double m2, const float* gamma,
                                             const float* beta, float momentum, float eps, float* rmean, float* rvar,
                                             int64_t* nbt, float* ss, float* mi) {
    const double var = m2 / (double)count;
    const double invstd = 1.0 / sqrt(var + (double)eps);
    const float inv_f = (float)invstd, mean_f = (float)mean;
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    const float alpha = __fmul_rn(inv_f, g);
    ss[c] = alpha;
    ss[C + c] = __fsub_rn(b, __fmul_rn(mean_f, alpha));
    if (mi) {
        mi[c] = mean_f;
        mi[C + c] = inv_f;
    }
    if (rmean) {
        const double unbiased = count > 1 ? m2 / (double)(count - 1) : var;
        rmean[c] = (float)((double)momentum * mean + (1.0 - (double)momentum) * (double)rmean[c]);
        rvar[c] = (float)((double)momentum * unbiased + (1.0 - (double)momentum) * (double)rvar[c]);
    }
    if (nbt && c == 0) nbt[0] += 1;
}

}  // namespace hkp
