// Stage probe: how fast can the QPPVM fast kernel's input burst arrive? B = 4096 instances of the
// config-1 layout (n = 30: M [B][30][30], J [B][2][6][30], poses, q, qd, qref, h; 11.6 KB each),
// two instances per wave64 (lane i <-> joint i), 2 waves per SIMD (2,048 blocks, one round), each
// wave loads its instances and writes one checksum per lane. Variants:
//   dx2      the product's pattern: one 8-byte buffer load per lane per M row / J row (lane = column)
//   dx4lds   M and J as 16-byte loads of contiguous chunks into LDS, then each lane reads its column
//   dx2_1w   dx2 with one instance per wave (4,096 blocks of 32 lanes... as 64 with half idle)
// Time per launch (events, back to back) and the bytes it moves -> GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int N = 30, NP = 32, T = 2;
constexpr int PER = N * N + T * 6 * N + 2 * T * 12 + 4 * N; // doubles per instance in the probe

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const double *p, long elems)
{
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, (int)(elems * 8 < 0x7fffffffL ? elems * 8 : 0x7fffffffL),
                                             0x00020000);
}
__device__ __forceinline__ double bl(__amdgpu_buffer_rsrc_t r, int v, int s)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, v, s, 0));
}

__global__ __launch_bounds__(64, 2) void dx2(const double *M, const double *J, const double *P, const double *V,
                                               double *out, int B)
{
    const int sub = threadIdx.x / NP, i = threadIdx.x % NP, ic = i < N ? i : N - 1;
    const long b0 = (long)blockIdx.x * 2, b = b0 + sub;
    const int lb = (int)(b - b0);
    const auto Mr = rs(M + b0 * N * N, (B - b0) * N * N), Jr = rs(J + b0 * T * 6 * N, (B - b0) * T * 6 * N);
    const auto Pr = rs(P + b0 * T * 24, (B - b0) * T * 24), Vr = rs(V + b0 * 4 * N, (B - b0) * 4 * N);
    double acc = 0.0;
    double v[4], jv[T * 6], m[NP], p[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = bl(Vr, 8 * (lb * 4 * N + k * N + ic), 0);
#pragma unroll
    for (int r = 0; r < T * 6; ++r) jv[r] = bl(Jr, 8 * (lb * T * 6 * N + ic), 8 * r * N);
#pragma unroll
    for (int k = 0; k < 2; ++k) p[k] = bl(Pr, 8 * (lb * T * 24 + (k * NP + i < T * 24 ? k * NP + i : 0)), 0);
#pragma unroll
    for (int r = 0; r < NP; ++r) m[r] = bl(Mr, 8 * (lb * N * N + ic), 8 * (r < N ? r : N - 1) * N);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += v[k];
#pragma unroll
    for (int r = 0; r < T * 6; ++r) acc += jv[r];
    acc += p[0] + p[1];
#pragma unroll
    for (int r = 0; r < NP; ++r) acc += m[r];
    out[b * NP + i] = acc;
}

// 16-byte loads of each wave's contiguous M / J blocks into LDS (global_load_lds_dwordx4 when the
// compiler uses it; else through VGPRs), then lane i reads its column
__global__ __launch_bounds__(64, 2) void dx4lds(const double *M, const double *J, const double *P, const double *V,
                                                  double *out, int B)
{
    __shared__ __attribute__((aligned(16))) double sm[2 * (N * N + T * 6 * N)];
    const int sub = threadIdx.x / NP, i = threadIdx.x % NP, ic = i < N ? i : N - 1;
    const long b0 = (long)blockIdx.x * 2, b = b0 + sub;
    const int lb = (int)(b - b0);
    const auto Pr = rs(P + b0 * T * 24, (B - b0) * T * 24), Vr = rs(V + b0 * 4 * N, (B - b0) * 4 * N);
    // M block of the two instances: 2 * 900 doubles = 900 double2 -> 64 lanes x 15 (14.06) rounds
    const double2 *M2 = reinterpret_cast<const double2 *>(M + b0 * N * N);
    const double2 *J2 = reinterpret_cast<const double2 *>(J + b0 * T * 6 * N);
    double2 *s2 = reinterpret_cast<double2 *>(sm);
    constexpr int MC = N * N, JC = T * 6 * N; // per instance, both even
    double2 t[15], u[6];
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        const int e = k * 64 + threadIdx.x;
        t[k] = e < MC ? M2[e] : make_double2(0, 0);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int e = k * 64 + threadIdx.x;
        u[k] = e < JC ? J2[e] : make_double2(0, 0);
    }
    double v[4], p[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = bl(Vr, 8 * (lb * 4 * N + k * N + ic), 0);
#pragma unroll
    for (int k = 0; k < 2; ++k) p[k] = bl(Pr, 8 * (lb * T * 24 + (k * NP + i < T * 24 ? k * NP + i : 0)), 0);
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        const int e = k * 64 + threadIdx.x;
        if (e < MC) s2[e] = t[k];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int e = k * 64 + threadIdx.x;
        if (e < JC) s2[MC + e] = u[k];
    }
    __syncthreads();
    double acc = 0.0;
    const double *Ms = sm + sub * N * N, *Js = sm + 2 * MC + sub * JC;
#pragma unroll
    for (int r = 0; r < NP; ++r) acc += Ms[(r < N ? r : N - 1) * N + ic];
#pragma unroll
    for (int r = 0; r < T * 6; ++r) acc += Js[r * N + ic];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += v[k];
    acc += p[0] + p[1];
    out[b * NP + i] = acc;
}

int main()
{
    const int B = 4096;
    double *M, *J, *P, *V, *out;
    hipMalloc(&M, (size_t)B * N * N * 8);
    hipMalloc(&J, (size_t)B * T * 6 * N * 8);
    hipMalloc(&P, (size_t)B * T * 24 * 8);
    hipMalloc(&V, (size_t)B * 4 * N * 8);
    hipMalloc(&out, (size_t)B * NP * 8);
    hipMemset(M, 0, (size_t)B * N * N * 8);
    hipMemset(J, 0, (size_t)B * T * 6 * N * 8);
    hipMemset(P, 0, (size_t)B * T * 24 * 8);
    hipMemset(V, 0, (size_t)B * 4 * N * 8);
    const double bytes = (double)B * PER * 8 + (double)B * NP * 8;
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, auto k) {
        for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k, dim3(B / 2), dim3(64), 0, s, M, J, P, V, out, B);
        hipStreamSynchronize(s);
        const int R = 200;
        hipEventRecord(e0, s);
        for (int w = 0; w < R; ++w) hipLaunchKernelGGL(k, dim3(B / 2), dim3(64), 0, s, M, J, P, V, out, B);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / R;
        std::printf("%-10s %8.2f us/launch  %7.0f GB/s (%.1f MB)\n", name, us, bytes / us * 1e-3, bytes * 1e-6);
    };
    run("dx2", dx2);
    run("dx4lds", dx4lds);
    run("dx2", dx2);
    run("dx4lds", dx4lds);
    return 0;
}
