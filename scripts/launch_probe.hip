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

// same, but the (never taken) work path needs ~1 KB of scratch per lane, like the repair kernel
__global__ __launch_bounds__(64, 2) void probe_scratch(const int *flag, double *out, int k)
{
    if (*flag == 0) return;
    volatile double buf[128];
    for (int j = 0; j < 128; ++j) buf[j] = j * out[j];
    out[blockIdx.x * 64 + threadIdx.x] = buf[(threadIdx.x + k) & 127];
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
    // the same with a scratch-using no-work kernel, and as a hipGraph
    for (int g : {256, 512, 2048}) {
        const int N = 500;
        hipEventRecord(e0, s);
        for (int k = 0; k < N; ++k) {
            hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
            hipLaunchKernelGGL(probe_scratch, dim3(g), dim3(64), 20480, s, flag, out, k);
        }
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("busy + 1 scratch no-work kernel (grid %d, 20 KB): %.3f us/iter\n", g, 1e3 * ms / N);
    }
    {
        hipGraph_t gr;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
        hipLaunchKernelGGL(probe_scratch, dim3(512), dim3(64), 20480, s, flag, out, 1);
        hipStreamEndCapture(s, &gr);
        hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        for (int w = 0; w < 20; ++w) hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        const int N = 500;
        hipEventRecord(e0, s);
        for (int k = 0; k < N; ++k) hipGraphLaunch(ge, s);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("graph(busy + scratch no-work grid 512): %.3f us/iter\n", 1e3 * ms / N);
    }
    {
        const int N = 500;
        hipEventRecord(e0, s);
        for (int k = 0; k < N; ++k) hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("busy alone: %.3f us/iter\n", 1e3 * ms / N);
    }
    return 0;
}
