// Compute-only MFMA ceiling on this part (make the "practically
// reachable MFMA rate" claim reproducible).  Every CU runs 8 waves (2 per SIMD,
// the conv kernels' occupancy), each issuing v_mfma_f32_16x16x32_f16 back to
// back into a 64x128 wave tile (32 independent 16x16 accumulators — the
// 256x256 conv body's wave tile), on random fp16 operands (the DVFS give-back
// of MI355X_MICROARCH.md depends on the data: zeros clock higher) and on zeros.
// Variant "lds": the operand fragments are re-read from LDS every k-step as the
// conv body does (24 ds_read_b128 per 96 MFMAs).  After a >= 2 s warm-up of
// back-to-back launches, the median of timed launches is reported as fp16
// TFLOP/s, and as a fraction of the 2.5 PF dense spec.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_peak.hip -o tools/bin/mfma_peak
//   tools/bin/mfma_peak            (prints one JSON object per variant)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int UM = 4, UN = 8;   // 64 x 128 wave tile of 16x16 blocks

template <bool LDS>
__global__ __launch_bounds__(512, 1) void mfma_loop(const f16x8* __restrict__ in, float* __restrict__ out, int iters) {
    __shared__ f16x8 lds[512 * 3];
    const int tid = threadIdx.x;
    f16x8 a[UM], b[UN];
#pragma unroll
    for (int i = 0; i < UM; ++i) a[i] = in[(blockIdx.x * 512 + tid) * 12 % 65536 + i];
#pragma unroll
    for (int j = 0; j < UN; ++j) b[j] = in[(blockIdx.x * 512 + tid) * 12 % 65536 + UM + j];
    if (LDS) {
        for (int i = tid; i < 512 * 3; i += 512) lds[i] = in[(blockIdx.x * 7 + i) % 65536];
        __syncthreads();
    }
    f32x4 acc[UM][UN];
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int lane = tid & 63;
    for (int it = 0; it < iters; ++it) {
        if (LDS) {   // the conv body's operand traffic: 8 A + 16 B fragment reads per 96 MFMAs
#pragma unroll
            for (int i = 0; i < UM; ++i) a[i] = lds[(lane + 64 * i + it) % 1536];
#pragma unroll
            for (int j = 0; j < UN; ++j) b[j] = lds[(lane + 64 * (UM + j) + it) % 1536];
        }
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int i = 0; i < UM; ++i)
#pragma unroll
                for (int j = 0; j < UN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < UM; ++i)
#pragma unroll
        for (int j = 0; j < UN; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 512 + tid] = s;
}

template <bool LDS>
static void run(const char* name, const f16x8* in, float* out, int cus) {
    const int blocks = cus * 4, iters = 4096;
    // FLOPs: blocks * 8 waves * iters * 3 * UM * UN MFMAs * (16*16*32*2)
    const double flops = (double)blocks * 8 * iters * 3 * UM * UN * 16.0 * 16 * 32 * 2;
    hipEvent_t s, e;
    CHECK(hipEventCreate(&s));
    CHECK(hipEventCreate(&e));
    float ms = 0.f, warm = 0.f;
    while (warm < 2000.f) {   // >= 2 s of back-to-back launches: the clock settles
        CHECK(hipEventRecord(s));
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(mfma_loop<LDS>, dim3(blocks), dim3(512), 0, 0, in, out, iters);
        CHECK(hipEventRecord(e));
        CHECK(hipEventSynchronize(e));
        CHECK(hipEventElapsedTime(&ms, s, e));
        warm += ms;
    }
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) {
        CHECK(hipEventRecord(s));
        hipLaunchKernelGGL(mfma_loop<LDS>, dim3(blocks), dim3(512), 0, 0, in, out, iters);
        CHECK(hipEventRecord(e));
        CHECK(hipEventSynchronize(e));
        CHECK(hipEventElapsedTime(&ms, s, e));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double tf = flops / (t[t.size() / 2] * 1e-3) / 1e12;
    printf("{\"variant\": \"%s\", \"mfma\": \"v_mfma_f32_16x16x32_f16\", \"waves_per_simd\": 2, \"median_ms\": %.4f, "
           "\"tflops\": %.1f, \"frac_of_2500\": %.3f}\n", name, t[t.size() / 2], tf, tf / 2500.0);
    fflush(stdout);
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t n = 65536 + 64;
    std::vector<_Float16> h(n * 8);
    srand(1);
    for (auto& v : h) v = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
    f16x8 *rnd, *zero;
    float* out;
    CHECK(hipMalloc(&rnd, n * sizeof(f16x8)));
    CHECK(hipMalloc(&zero, n * sizeof(f16x8)));
    CHECK(hipMalloc(&out, (size_t)cus * 4 * 512 * sizeof(float)));
    CHECK(hipMemcpy(rnd, h.data(), n * sizeof(f16x8), hipMemcpyHostToDevice));
    CHECK(hipMemset(zero, 0, n * sizeof(f16x8)));
    run<false>("registers_random", rnd, out, cus);
    run<false>("registers_zeros", zero, out, cus);
    run<true>("lds_operands_random", rnd, out, cus);
    CHECK(hipFree(rnd));
    CHECK(hipFree(zero));
    CHECK(hipFree(out));
    return 0;
}
