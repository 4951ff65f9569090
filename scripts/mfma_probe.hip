// MFMA f64 layout probe: one wave runs v_mfma_f64_16x16x4f64 on lane-indexed operands and
// dumps A, B (one double per lane) and D (4 doubles per lane); scripts check the layout
// hypotheses on the host:
//   A: lane l holds A[l % 16][l / 16]      B: lane l holds B[l / 16][l % 16]
//   D: lane l, register v holds D[4 v + l / 16][l % 16]   (CK: group_size 1, 4 groups per block)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef double double4_t __attribute__((ext_vector_type(4)));

__global__ void probe(double *out)
{
    const int l = threadIdx.x;
    const double a = 1.0 + 0.37 * l + 0.011 * l * l;
    const double b = 2.0 - 0.23 * l + 0.007 * l * l;
    double4_t c = {0.0, 0.0, 0.0, 0.0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    out[l * 6 + 0] = a;
    out[l * 6 + 1] = b;
    for (int v = 0; v < 4; ++v) out[l * 6 + 2 + v] = c[v];
}

int main()
{
    double *d, h[64 * 6];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    double A[16][4], B[4][16];
    for (int l = 0; l < 64; ++l) {
        A[l % 16][l / 16] = h[l * 6];
        B[l / 16][l % 16] = h[l * 6 + 1];
    }
    double e1 = 0.0, e2 = 0.0;
    for (int l = 0; l < 64; ++l)
        for (int v = 0; v < 4; ++v) {
            const int j = l % 16;
            const int i1 = 4 * v + l / 16, i2 = 4 * (l / 16) + v;
            double d1 = 0.0, d2 = 0.0;
            for (int k = 0; k < 4; ++k) {
                d1 += A[i1][k] * B[k][j];
                d2 += A[i2][k] * B[k][j];
            }
            e1 = fmax(e1, fabs(d1 - h[l * 6 + 2 + v]));
            e2 = fmax(e2, fabs(d2 - h[l * 6 + 2 + v]));
        }
    std::printf("{\"D_row_4v_plus_lane_div16_err\": %.3e, \"D_row_4lane_div16_plus_v_err\": %.3e}\n", e1, e2);
    return 0;
}
