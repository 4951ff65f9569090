// Launch-overhead probe: per-launch device time of a no-work kernel (reads one flag and
// exits) vs grid size and dynamic LDS, back to back on one stream. Guides how the
// follow-up (active-set / repair) kernels are launched.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64, 2) void probe(const int *flag, double *out)
{
    extern __shared__ double sm[];
    if (*flag == 0) return;
    sm[threadIdx.x] = threadIdx.x;
    __syncthreads();
    out[blockIdx.x * 64 + threadIdx.x] = sm[63 - threadIdx.x];
}

__global__ __launch_bounds__(64, 2) void busy(double *out, int iters)
{
    double v = threadIdx.x;
    for (int k = 0; k < iters; ++k) v = fma(v, 0.999, 1.0);
    out[blockIdx.x * 64 + threadIdx.x] = v;
}

int main()
{
    int *flag;
    double *out;
    hipMalloc(&flag, 4);
    hipMemset(flag, 0, 4);
    hipMalloc(&out, 8 * 64 * 4096);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grids[] = {1, 64, 256, 1024, 2048};
    const int ldss[] = {0, 20480};
    for (int lds : ldss) {
        hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
        for (int g : grids) {
            for (int w = 0; w < 50; ++w) hipLaunchKernelGGL(probe, dim3(g), dim3(64), lds, s, flag, out);
            hipStreamSynchronize(s);
            const int N = 2000;
            hipEventRecord(e0, s);
            for (int k = 0; k < N; ++k) hipLaunchKernelGGL(probe, dim3(g), dim3(64), lds, s, flag, out);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            std::printf("probe grid=%5d lds=%6d  %.3f us/launch (back to back)\n", g, lds, 1e3 * ms / N);
        }
    }
    // a ~30 us kernel followed by 0, 1, 2 no-work kernels: incremental wall cost
    for (int extra = 0; extra <= 2; ++extra) {
        const int N = 500;
        for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
        hipStreamSynchronize(s);
        hipEventRecord(e0, s);
        for (int k = 0; k < N; ++k) {
            hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
            for (int x = 0; x < extra; ++x) hipLaunchKernelGGL(probe, dim3(2048), dim3(64), 20480, s, flag, out);
        }
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("busy + %d no-work kernels (grid 2048, 20 KB): %.3f us/iter\n", extra, 1e3 * ms / N);
    }
    for (int extra = 1; extra <= 2; ++extra) {
        const int N = 500;
        hipEventRecord(e0, s);
        for (int k = 0; k < N; ++k) {
            hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
            for (int x = 0; x < extra; ++x) hipLaunchKernelGGL(probe, dim3(256), dim3(64), 20480, s, flag, out);
        }
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("busy + %d no-work kernels (grid 256, 20 KB): %.3f us/iter\n", extra, 1e3 * ms / N);
    }
    return 0;
}
