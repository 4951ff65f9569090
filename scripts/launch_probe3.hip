// Launch-overhead probe 3: does the ~5 us empty follow-up launch come from cold misses? A busy
// kernel that streams 64 MB (evicting L2, like the fast kernel's inputs) is followed by a no-work
// kernel that reads a counter (kernarg -> counter chain); variants: the busy kernel's waves touch
// the counter line at their end (the line in every XCD's L2), a 512-byte kernel argument.
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big {
    const int *flag;
    double pad[40];
};

__global__ __launch_bounds__(64, 2) void stream_busy(const double *in, double *out, long n, const int *touch)
{
    double s = 0.0;
    for (long k = (long)blockIdx.x * 64 + threadIdx.x; k < n; k += (long)gridDim.x * 64) s += in[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (touch && threadIdx.x == 0) out[blockIdx.x * 64] += (double)touch[0];
}

__global__ __launch_bounds__(64, 1) void probe(const int *flag, double *out)
{
    if (*flag == 0) return;
    out[blockIdx.x * 64 + threadIdx.x] = 1.0;
}

__global__ __launch_bounds__(64, 1) void probe_big(const Big b, double *out)
{
    if (*b.flag == 0) return;
    out[blockIdx.x * 64 + threadIdx.x] = b.pad[threadIdx.x & 31];
}

int main()
{
    int *flag;
    double *in, *out;
    const long n = 8L << 20; // 64 MB
    hipMalloc(&flag, 256);
    hipMemset(flag, 0, 256);
    hipMalloc(&in, n * 8);
    hipMemset(in, 0, n * 8);
    hipMalloc(&out, 8 * 64 * 4096);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    Big big{};
    big.flag = flag;
    auto run = [&](const char *name, auto launch) {
        const int N = 300;
        for (int w = 0; w < 10; ++w) launch();
        hipStreamSynchronize(s);
        hipEventRecord(e0, s);
        for (int k = 0; k < N; ++k) launch();
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("%-52s %8.3f us/iter\n", name, 1e3 * ms / N);
    };
    run("stream 64 MB alone", [&] { hipLaunchKernelGGL(stream_busy, dim3(2048), dim3(64), 0, s, in, out, n, nullptr); });
    run("stream + empty (cold counter)", [&] {
        hipLaunchKernelGGL(stream_busy, dim3(2048), dim3(64), 0, s, in, out, n, nullptr);
        hipLaunchKernelGGL(probe, dim3(16), dim3(64), 0, s, flag, out);
    });
    run("stream (touches counter) + empty", [&] {
        hipLaunchKernelGGL(stream_busy, dim3(2048), dim3(64), 0, s, in, out, n, flag);
        hipLaunchKernelGGL(probe, dim3(16), dim3(64), 0, s, flag, out);
    });
    run("stream + empty, 336-byte kernarg", [&] {
        hipLaunchKernelGGL(stream_busy, dim3(2048), dim3(64), 0, s, in, out, n, nullptr);
        hipLaunchKernelGGL(probe_big, dim3(16), dim3(64), 0, s, big, out);
    });
    run("stream (touches) + empty, 336-byte kernarg", [&] {
        hipLaunchKernelGGL(stream_busy, dim3(2048), dim3(64), 0, s, in, out, n, flag);
        hipLaunchKernelGGL(probe_big, dim3(16), dim3(64), 0, s, big, out);
    });
    return 0;
}
