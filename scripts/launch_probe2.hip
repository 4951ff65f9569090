// Launch-overhead probe 2: what makes an empty follow-up launch cost ~5 us after a busy kernel
// (the QPPVM repair kernel with an empty work list, rocprofv3 r03)? Same no-work body, one
// resource at a time: 512 registers (VGPR + AGPR), a block-0 store, 40 KB dynamic LDS, scratch.
#include <hip/hip_runtime.h>
#include <cstdio>

#define BODY                                                         \
    if (*flag == 0) {                                                \
        if (STORE && blockIdx.x == 0 && threadIdx.x == 0) cnt[0] = 0; \
        return;                                                      \
    }                                                                \
    out[blockIdx.x * 64 + threadIdx.x] = 1.0;

template <bool STORE>
__global__ __launch_bounds__(64, 1) void p_plain(const int *flag, int *cnt, double *out) { BODY }

template <bool STORE>
__global__ __launch_bounds__(64, 1) void p_regs(const int *flag, int *cnt, double *out)
{
    asm volatile("" ::: "v255", "a127");
    BODY
}

template <bool STORE>
__global__ __launch_bounds__(64, 1) void p_scratch(const int *flag, int *cnt, double *out, int k)
{
    if (*flag == 0) {
        if (STORE && blockIdx.x == 0 && threadIdx.x == 0) cnt[0] = 0;
        return;
    }
    volatile double buf[8];
    for (int j = 0; j < 8; ++j) buf[j] = j * out[j];
    out[blockIdx.x * 64 + threadIdx.x] = buf[(threadIdx.x + k) & 7];
}

__global__ __launch_bounds__(64, 2) void busy(double *out, int iters)
{
    double v = threadIdx.x;
    for (int k = 0; k < iters; ++k) v = fma(v, 0.999, 1.0);
    out[blockIdx.x * 64 + threadIdx.x] = v;
}

int main()
{
    int *flag, *cnt;
    double *out;
    hipMalloc(&flag, 4);
    hipMemset(flag, 0, 4);
    hipMalloc(&cnt, 16);
    hipMalloc(&out, 8 * 64 * 4096);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto f : {(const void *)p_plain<false>, (const void *)p_plain<true>, (const void *)p_regs<false>,
                   (const void *)p_regs<true>, (const void *)p_scratch<false>, (const void *)p_scratch<true>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    auto run = [&](const char *name, auto launch) {
        const int N = 400;
        for (int w = 0; w < 20; ++w) {
            hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
            launch();
        }
        hipStreamSynchronize(s);
        hipEventRecord(e0, s);
        for (int k = 0; k < N; ++k) {
            hipLaunchKernelGGL(busy, dim3(2048), dim3(64), 0, s, out, 20000);
            launch();
        }
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::printf("%-44s %8.3f us/iter\n", name, 1e3 * ms / N);
    };
    run("busy alone", [] {});
    for (int lds : {0, 40960}) {
        for (int g : {16, 2048}) {
            char nm[128];
#define V(K, ST, ...)                                                                           \
    std::snprintf(nm, sizeof nm, "+ %s store=%d lds=%d grid=%d", #K, ST, lds, g);             \
    run(nm, [&] { hipLaunchKernelGGL(K<ST>, dim3(g), dim3(64), lds, s, flag, cnt, out __VA_ARGS__); });
            V(p_plain, false)
            V(p_plain, true)
            V(p_regs, false)
            V(p_regs, true)
            V(p_scratch, false, , 1)
            V(p_scratch, true, , 1)
        }
    }
    return 0;
}
