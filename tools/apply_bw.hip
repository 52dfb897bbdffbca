// Streaming-rate probe for the fp16 BN apply shape (out = relu(y*a+b + res),
// 2 reads + 1 write of 16-B vectors over 1.26 GB tensors — C4 layer3 block
// output): the product kernel's loop form beside variants, plus a plain copy.
//   hipcc -O3 --offload-arch=gfx950 tools/apply_bw.hip -o tools/bin/apply_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void apply_res(long n8, int C8, const h16x8* __restrict__ y,
                                                 const float* __restrict__ ss, const h16x8* __restrict__ res,
                                                 h16x8* __restrict__ out) {
    const int C = C8 * 8;
    const long stride = (long)gridDim.x * blockDim.x;
    const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
    float a[8], b[8];
    const int c0 = (int)(i0 % C8) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        a[e] = ss[c0 + e];
        b[e] = ss[C + c0 + e];
    }
    for (long i = i0; i < n8; i += U * stride) {
        h16x8 v[U], r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + u * stride;
            if (k < n8) {
                v[u] = NT ? __builtin_nontemporal_load(&y[k]) : y[k];
                r[u] = NT ? __builtin_nontemporal_load(&res[k]) : res[k];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + u * stride;
            if (k >= n8) break;
            h16x8 h;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float o = (float)v[u][e] * a[e] + b[e] + (float)r[u][e];
                h[e] = (_Float16)(o > 0.f ? o : 0.f);
            }
            if (NT) __builtin_nontemporal_store(h, &out[k]);
            else out[k] = h;
        }
    }
}

__global__ __launch_bounds__(256) void copy16(long n8, const h16x8* __restrict__ y, h16x8* __restrict__ out) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) out[i] = y[i];
}

int main() {
    const long m = 614400L * 128 / 128 * 1;   // pixels of C4 layer3 (128 x 60 x 80)
    const int C = 1024;
    const long n8 = m * C / 8;
    h16x8 *y, *r, *o;
    float* ss;
    hipMalloc(&y, n8 * 16);
    hipMalloc(&r, n8 * 16);
    hipMalloc(&o, n8 * 16);
    hipMalloc(&ss, 2 * C * 4);
    hipMemset(y, 0x3c, n8 * 16);
    hipMemset(r, 0x3c, n8 * 16);
    hipMemset(ss, 0, 2 * C * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        const int it = 10;
        for (int w = 0; w < it; ++w) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        printf("%-40s %8.3f ms  %6.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    const double b3 = 3.0 * n8 * 16, b2 = 2.0 * n8 * 16;
    const int C8 = C / 8;
    for (int rep = 0; rep < 2; ++rep)
    for (int g : {4096, 2048, 1536, 1024, 768, 512}) {
        char nm[64];
        snprintf(nm, 64, "apply U2 grid %d", g);
        timeit(nm, b3, [&] { hipLaunchKernelGGL((apply_res<2, false>), dim3(g), dim3(256), 0, 0, n8, C8, y, ss, r, o); });
        snprintf(nm, 64, "apply U2 nt grid %d", g);
        timeit(nm, b3, [&] { hipLaunchKernelGGL((apply_res<2, true>), dim3(g), dim3(256), 0, 0, n8, C8, y, ss, r, o); });
        snprintf(nm, 64, "apply U1 grid %d", g);
        timeit(nm, b3, [&] { hipLaunchKernelGGL((apply_res<1, false>), dim3(g), dim3(256), 0, 0, n8, C8, y, ss, r, o); });
        snprintf(nm, 64, "apply U1 nt grid %d", g);
        timeit(nm, b3, [&] { hipLaunchKernelGGL((apply_res<1, true>), dim3(g), dim3(256), 0, 0, n8, C8, y, ss, r, o); });
    }
    timeit("copy grid 4096", b2, [&] { hipLaunchKernelGGL(copy16, dim3(4096), dim3(256), 0, 0, n8, y, o); });
    timeit("copy grid 2048", b2, [&] { hipLaunchKernelGGL(copy16, dim3(2048), dim3(256), 0, 0, n8, y, o); });
    timeit("hipMemcpy d2d", b2, [&] { hipMemcpyAsync(o, y, n8 * 16, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
