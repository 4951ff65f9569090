// Gauss-Jordan probe: the QPPVM fast kernel's stage + elimination in isolation, config-1 shape (B =
// 4096, n = 30, two instances per wave64, 2 waves per SIMD, one wave round). Variants:
//   right  the product's order: every M row loaded, Y = M G^T, then block_gj (wbq_device.h), right-looking
//   left   left-looking: column block kb is brought up to date by the stored steps p < kb when its
//          loads arrive (vmcnt retires in order), Y accumulated block by block, so the elimination
//          runs while later columns of M are still in flight
// Both apply every step to every column in the same order with the same operations, so their outputs
// are compared bit for bit. Time per launch from events around back-to-back launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I qppvm_amd/csrc scripts/gj_probe.hip -o scripts/gj_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "wbq_device.h"

#ifndef PROBE_Y
#define PROBE_Y 0 // Y = M G^T in the probe (1) or the elimination alone (0)
#endif

using namespace wbq;

constexpr int N = 30, NP = 32, NC = 32, M0 = 6, NR = 3, BS = kGjBS, NB = NC / BS;

#define NOSTAMP(k) do {} while (0)
#define STAMP_UNUSED(k)                                                                                         \
    do {                                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                      \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        if (threadIdx.x == 0) a.st[blockIdx.x * 16 + (k)] = t_;                                          \
    } while (0)

#define CHECK(x)                                                                                         \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) {                                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));               \
            std::exit(1);                                                                                \
        }                                                                                                \
    } while (0)

struct Args {
    const double *M, *G, *R; // [B][N][N], [B][M0][N], [B][NR][N]
    double *X, *Y;           // [B][NR][N] = M^-1 R, [B][M0][N] = (M G^T)^T
    unsigned long long *st;  // [grid][16] s_memtime stamps (lane 0 of every wave)
    const int *row_sel;      // [M0] (identity; a runtime index as in the product's G rows)
    int B;
};

// Block Gauss-Jordan with an explicit pivot-block inverse (candidate for wbq_device.h block_gj): the
// 4 x 4 SPD pivot block D is inverted in closed form through its 2 x 2 Schur complement (two 2 x 2
// inverses by determinants: a dependent chain of ~25 operations instead of the Cholesky + two
// triangular solves' ~55), y = D^-1 a_i is a 4 x 4 matrix-vector product, and one update form serves
// every row: row_i += hh . row_P with hh = -D^-1 a_i outside the block and hh = D^-1 e_ri - e_ri inside
// it (row_i - row_P[ri] + (D^-1 row_P)[ri] = the normalised pivot row): no cc * A multiply per column.
template <int NP, int NR, int RHS, int NC = NP>
__device__ __forceinline__ bool block_gj2(double (&A)[NC], double (&rhs)[NR], int n, int i, double *PN, double *RH)
{
    constexpr int BS = kGjBS;
    static_assert(BS == 4, "block_gj2: 4 x 4 pivot blocks");
    bool notspd = false;
    if (i < NP) {
#pragma unroll
        for (int c = 0; c < BS; ++c) PN[i * BS + c] = A[c];
    }
    if (i < BS) {
#pragma unroll
        for (int m = 0; m < NR; ++m) RH[i * RHS + m] = rhs[m];
    }
#pragma unroll
    for (int kb = 0; kb < NC / BS; ++kb) {
        const int k = kb * BS;
        if (k < n) {
            __syncthreads();
            const double *pn = PN + (kb & 1) * NP * BS;
            const double *rh = RH + (kb & 1) * BS * RHS;
            double *pnn = PN + ((kb + 1) & 1) * NP * BS;
            double *rhn = RH + ((kb + 1) & 1) * BS * RHS;
            // D = [P Q; Q^T R] (symmetric: lower triangle from the panel rows k..k+3)
            const double d00 = pn[k * BS], d10 = pn[(k + 1) * BS], d11 = pn[(k + 1) * BS + 1];
            const double d20 = pn[(k + 2) * BS], d21 = pn[(k + 2) * BS + 1], d22 = pn[(k + 2) * BS + 2];
            const double d30 = pn[(k + 3) * BS], d31 = pn[(k + 3) * BS + 1], d32 = pn[(k + 3) * BS + 2];
            const double d33 = pn[(k + 3) * BS + 3];
            const double detP = fma(d00, d11, -d10 * d10);
            const double iP = frcp(detP);
            const double p00 = d11 * iP, p01 = -d10 * iP, p11 = d00 * iP; // P^-1
            // W = P^-1 Q, Q = [d20 d30; d21 d31]
            const double w00 = fma(p00, d20, p01 * d21), w01 = fma(p00, d30, p01 * d31);
            const double w10 = fma(p01, d20, p11 * d21), w11 = fma(p01, d30, p11 * d31);
            // S = R - Q^T W
            const double s00 = d22 - fma(d20, w00, d21 * w10);
            const double s01 = d32 - fma(d20, w01, d21 * w11);
            const double s11 = d33 - fma(d30, w01, d31 * w11);
            const double detS = fma(s00, s11, -s01 * s01);
            notspd |= !(d00 > 0.0 && detP > 0.0 && s00 > 0.0 && detS > 0.0);
            const double iS = frcp(detS);
            const double t00 = s11 * iS, t01 = -s01 * iS, t11 = s00 * iS; // S^-1
            // -W S^-1 (rows 0..1, columns 2..3 of D^-1)
            const double u00 = -fma(w00, t00, w01 * t01), u01 = -fma(w00, t01, w01 * t11);
            const double u10 = -fma(w10, t00, w11 * t01), u11 = -fma(w10, t01, w11 * t11);
            // P^-1 + W S^-1 W^T = P^-1 - U W^T
            const double v00 = p00 - fma(u00, w00, u01 * w01);
            const double v01 = p01 - fma(u00, w10, u01 * w11);
            const double v11 = p11 - fma(u10, w10, u11 * w11);
            const double Di[4][4] = {{v00, v01, u00, u01}, {v01, v11, u10, u11}, {u00, u10, t00, t01}, {u01, u11, t01, t11}};
            const int ri = i - k;
            const bool inK = ri >= 0 && ri < BS;
            double hh[BS];
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                double y = Di[c][0] * A[k];
#pragma unroll
                for (int q = 1; q < BS; ++q) y = fma(Di[c][q], A[k + q], y);
                double e = 0.0;
#pragma unroll
                for (int q = 0; q < BS; ++q) e = (ri == q) ? Di[c][q] : e;
                hh[c] = inK ? e - (ri == c ? 1.0 : 0.0) : -y;
            }
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                double v = rhs[m];
#pragma unroll
                for (int c = 0; c < BS; ++c) v = fma(hh[c], rh[c * RHS + m], v);
                rhs[m] = v;
            }
#pragma unroll
            for (int j = k + BS; j < k + 2 * BS && j < NC; ++j) {
                double v = A[j];
#pragma unroll
                for (int c = 0; c < BS; ++c) v = fma(hh[c], pn[j * BS + c], v);
                A[j] = v;
            }
            if (k + BS < n) {
                if (i < NP) {
#pragma unroll
                    for (int c = 0; c < BS; ++c)
                        if (k + BS + c < NC) pnn[i * BS + c] = A[(k + BS + c) < NC ? k + BS + c : NC - 1];
                }
                const int rn = i - (k + BS);
                if (rn >= 0 && rn < BS) {
#pragma unroll
                    for (int m = 0; m < NR; ++m) rhn[rn * RHS + m] = rhs[m];
                }
            }
#pragma unroll
            for (int j = k + 2 * BS; j < NC; ++j) {
                double v = A[j];
#pragma unroll
                for (int c = 0; c < BS; ++c) v = fma(hh[c], pn[j * BS + c], v);
                A[j] = v;
            }
        }
    }
    return notspd;
}

// block_gj with the trailing update's panel reads issued a chunk ahead (the compiler's own schedule kept
// one ds_read_b128 in flight and waited for each: the elimination ran at the LDS latency, not at its
// bandwidth or the FP64 rate). CH columns per chunk, two chunks in registers. UNI: one update form for
// every row (hh = D^-1 e_ri - e_ri inside the pivot block), no cc * A multiply per column.
template <int NP, int NR, int RHS, int NC, int CH, bool UNI>
__device__ __forceinline__ bool block_gj3(double (&A)[NC], double (&rhs)[NR], int n, int i, double *PN, double *RH)
{
    static_assert(NC % kGjBS == 0 && NC <= NP, "block_gj3: NC");
    constexpr int BS = kGjBS;
    bool notspd = false;
    if (i < NP) {
#pragma unroll
        for (int c = 0; c < BS; ++c) PN[i * BS + c] = A[c];
    }
    if (i < BS) {
#pragma unroll
        for (int m = 0; m < NR; ++m) RH[i * RHS + m] = rhs[m];
    }
#pragma unroll
    for (int kb = 0; kb < NC / BS; ++kb) {
        const int k = kb * BS;
        if (k < n) {
            __syncthreads();
            const double *pn = PN + (kb & 1) * NP * BS;
            const double *rh = RH + (kb & 1) * BS * RHS;
            double *pnn = PN + ((kb + 1) & 1) * NP * BS;
            double *rhn = RH + ((kb + 1) & 1) * BS * RHS;
            // the lookahead panel and the first trailing chunk are read with the pivot block
            double la[BS][BS];
#pragma unroll
            for (int u = 0; u < BS; ++u)
#pragma unroll
                for (int c = 0; c < BS; ++c) la[u][c] = (k + BS + u < NC) ? pn[(k + BS + u) * BS + c] : 0.0;
            constexpr int J0 = 0; (void)J0;
            double d[BS][BS];
#pragma unroll
            for (int r = 0; r < BS; ++r)
#pragma unroll
                for (int c = 0; c <= r; ++c) d[r][c] = pn[(k + r) * BS + c];
            double rv[BS][NR];
#pragma unroll
            for (int c = 0; c < BS; ++c)
#pragma unroll
                for (int m = 0; m < NR; ++m) rv[c][m] = rh[c * RHS + m];
            double il[BS];
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                double dd = d[c][c];
#pragma unroll
                for (int q_ = 0; q_ < c; ++q_) dd = fma(-d[c][q_], d[c][q_], dd);
                notspd |= !(dd > 0.0);
                il[c] = frsq(dd);
#pragma unroll
                for (int r = c + 1; r < BS; ++r) {
                    double t = d[r][c];
#pragma unroll
                    for (int q_ = 0; q_ < c; ++q_) t = fma(-d[r][q_], d[c][q_], t);
                    d[r][c] = t * il[c];
                }
            }
            const int ri = i - k;
            const bool inK = ri >= 0 && ri < BS;
            double y[BS];
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                double v = inK ? (ri == c ? 1.0 : 0.0) : A[k + c];
#pragma unroll
                for (int q_ = 0; q_ < c; ++q_) v = fma(-d[c][q_], y[q_], v);
                y[c] = v * il[c];
            }
#pragma unroll
            for (int c = BS - 1; c >= 0; --c) {
                double v = y[c];
#pragma unroll
                for (int q_ = c + 1; q_ < BS; ++q_) v = fma(-d[q_][c], y[q_], v);
                y[c] = v * il[c];
            }
            const double cc = inK ? 0.0 : 1.0;
            double hh[BS];
#pragma unroll
            for (int c = 0; c < BS; ++c) hh[c] = UNI ? (inK ? y[c] - (ri == c ? 1.0 : 0.0) : -y[c]) : (inK ? y[c] : -y[c]);
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                double v = UNI ? rhs[m] : cc * rhs[m];
#pragma unroll
                for (int c = 0; c < BS; ++c) v = fma(hh[c], rv[c][m], v);
                rhs[m] = v;
            }
#pragma unroll
            for (int u = 0; u < BS; ++u) {
                const int j = k + BS + u;
                if (j < NC) {
                    double v = UNI ? A[j] : cc * A[j];
#pragma unroll
                    for (int c = 0; c < BS; ++c) v = fma(hh[c], la[u][c], v);
                    A[j] = v;
                }
            }
            if (k + BS < n) {
                if (i < NP) {
#pragma unroll
                    for (int c = 0; c < BS; ++c)
                        if (k + BS + c < NC) pnn[i * BS + c] = A[(k + BS + c) < NC ? k + BS + c : NC - 1];
                }
                const int rn = i - (k + BS);
                if (rn >= 0 && rn < BS) {
#pragma unroll
                    for (int m = 0; m < NR; ++m) rhn[rn * RHS + m] = rhs[m];
                }
            }
            // trailing columns in chunks of CH, the next chunk's reads issued before this chunk's FMAs
            constexpr int NCH = (NC + CH - 1) / CH;
            double pv[2][CH][BS];
#pragma unroll
            for (int ch = 0; ch <= NCH; ++ch) {
                const int j0 = k + 2 * BS + ch * CH;
                if (ch < NCH && j0 < NC) {
#pragma unroll
                    for (int u = 0; u < CH; ++u)
#pragma unroll
                        for (int c = 0; c < BS; ++c) pv[ch & 1][u][c] = (j0 + u < NC) ? pn[(j0 + u) * BS + c] : 0.0;
                }
                __builtin_amdgcn_sched_barrier(0);
                const int jp = j0 - CH;
                if (ch > 0 && jp < NC) {
#pragma unroll
                    for (int u = 0; u < CH; ++u) {
                        const int j = jp + u;
                        if (j < NC) {
                            double v = UNI ? A[j] : cc * A[j];
#pragma unroll
                            for (int c = 0; c < BS; ++c) v = fma(hh[c], pv[(ch - 1) & 1][u][c], v);
                            A[j] = v;
                        }
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    return notspd;
}

// LDS per instance: G rows [M0][NP], panels [NB][NP][BS] (left) or [2][NP][BS] (right), RHS [2][BS][8]
constexpr int kG = 0, kPN = M0 * NP, kPNsize = NB * NP * BS, kRH = kPN + kPNsize, kSIZE = kRH + 2 * BS * 8;

template <int MODE>
__global__ __launch_bounds__(64, 2) void gj_kernel(const Args a)
{
    constexpr bool LEFT = MODE == 1 || MODE == 3, SYN = MODE == 2 || MODE == 3 || MODE == 6;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int sub = threadIdx.x / NP, i = threadIdx.x - sub * NP;
    const long b0 = (long)blockIdx.x * 2, b = b0 + sub;
    const int ic = i < N ? i : N - 1;
    const bool row = i < N;
    double *S = smem + sub * kSIZE;
    const long B = a.B;
    const __amdgpu_buffer_rsrc_t Grs = rsrc_at(a.G, b0, B, (long)M0 * N), Rrs = rsrc_at(a.R, b0, B, (long)NR * N);
    const __amdgpu_buffer_rsrc_t Mrs = rsrc_at(a.M, b0, B, (long)N * N);
    NOSTAMP(0);
    double gv[M0], rhs[NR];
#pragma unroll
    for (int c = 0; c < M0; ++c) gv[c] = bload(Grs, (int)(8 * (sub * M0 * N + ic)), 8 * c * N);
#pragma unroll
    for (int m = 0; m < NR; ++m) rhs[m] = bload(Rrs, (int)(8 * (sub * NR * N + ic)), 8 * m * N);
    __builtin_amdgcn_sched_barrier(0);
    double A[NC];
#pragma unroll
    for (int r = 0; r < NC; ++r) { // issue order pinned: row r before row r + 1 (vmcnt retires in order)
        if constexpr (SYN) // diagonally dominant SPD, no memory traffic
            A[r] = (r == ic ? 40.0 : 1.0 / (1.0 + r + ic)) + 1e-3 * (double)(b & 7);
        else
            A[r] = bload(Mrs, (int)(8 * (sub * N * N + ic)), 8 * (r < N ? r : N - 1) * N);
        if (LEFT) __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (MODE == 4) { // the stage alone
        double acc = rhs[0] + rhs[1] + rhs[2];
#pragma unroll
        for (int c = 0; c < M0; ++c) acc += gv[c];
#pragma unroll
        for (int r = 0; r < NC; ++r) acc += A[r];
        if (row) a.X[(b * NR) * N + i] = acc;
        return;
    }
#pragma unroll
    for (int c = 0; c < M0; ++c) S[kG + c * NP + i] = row ? gv[c] : 0.0;
#pragma unroll
    for (int m = 0; m < NR; ++m) rhs[m] = row ? rhs[m] : 0.0;
    lds_barrier();
    double Y[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) Y[c] = 0.0;
    if constexpr (!LEFT) {
#pragma unroll
        for (int r = 0; r < NC; ++r) A[r] = (row && r < N) ? A[r] : (r == i ? 1.0 : 0.0);
#if PROBE_Y
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            double v = 0.0;
            const int rr = a.row_sel[c];
#pragma unroll
            for (int j = 0; j < NC; ++j) v = fma(A[j], S[kG + rr * NP + j], v);
            Y[c] = v;
        }
#endif
        __syncthreads();
        NOSTAMP(1);
        if constexpr (MODE == 7) (void)block_gj3<NP, NR, 8, NC, 4, false>(A, rhs, N, i, S + kPN, S + kRH);
        else if constexpr (MODE == 8) (void)block_gj3<NP, NR, 8, NC, 4, true>(A, rhs, N, i, S + kPN, S + kRH);
        else if constexpr (MODE == 9) (void)block_gj3<NP, NR, 8, NC, 8, false>(A, rhs, N, i, S + kPN, S + kRH);
        else if constexpr (MODE >= 5) (void)block_gj2<NP, NR, 8, NC>(A, rhs, N, i, S + kPN, S + kRH);
        else (void)block_gj<NP, NR, 8, NC>(A, rhs, N, i, S + kPN, S + kRH);
        NOSTAMP(10);
    } else {
        // left-looking: hh / cc of every step kept per lane
        double hs[NB][BS], cs[NB];
        const double rowf = row ? 1.0 : 0.0;
        double *RH = S + kRH;
#pragma unroll
        for (int kb = 0; kb < NB; ++kb) {
            const int k = kb * BS;
            if (k < N) {
                // this block's columns (their loads are waited for here, in issue order)
                double v[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) // (arithmetic masking: a select here was hoisted into one branch over all blocks)
                    v[c] = k + c < N ? A[k + c] * rowf : (k + c == i ? 1.0 : 0.0); // (lanes i >= N: k + c != i)
#if PROBE_Y
#pragma unroll
                for (int cy = 0; cy < M0; ++cy) {
                    const int rr = a.row_sel[cy];
#pragma unroll
                    for (int c = 0; c < BS; ++c) Y[cy] = fma(v[c], S[kG + rr * NP + k + c], Y[cy]);
                }
#endif
                // steps p < kb in order: v = cc_p v + sum_c hh_p[c] panel_p[j][c] (block_gj's arithmetic)
#pragma unroll
                for (int p = 0; p < kb; ++p) {
                    const double *pn = S + kPN + p * NP * BS;
#pragma unroll
                    for (int c = 0; c < BS; ++c) {
                        double t = cs[p] * v[c];
#pragma unroll
                        for (int q = 0; q < BS; ++q) t = fma(hs[p][q], pn[(k + c) * BS + q], t);
                        v[c] = t;
                    }
                }
                NOSTAMP(1 + kb);
                double *pk = S + kPN + kb * NP * BS;
#pragma unroll
                for (int c = 0; c < BS; ++c) pk[i * BS + c] = v[c];
                const int ri = i - k;
                if (ri >= 0 && ri < BS) {
#pragma unroll
                    for (int m = 0; m < NR; ++m) RH[(kb & 1) * BS * 8 + ri * 8 + m] = rhs[m];
                }
                __syncthreads();
                double d[BS][BS];
#pragma unroll
                for (int r = 0; r < BS; ++r)
#pragma unroll
                    for (int c = 0; c <= r; ++c) d[r][c] = pk[(k + r) * BS + c];
                double il[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    double dd = d[c][c];
#pragma unroll
                    for (int q_ = 0; q_ < c; ++q_) dd = fma(-d[c][q_], d[c][q_], dd);
                    il[c] = frsq(dd);
#pragma unroll
                    for (int r = c + 1; r < BS; ++r) {
                        double t = d[r][c];
#pragma unroll
                        for (int q_ = 0; q_ < c; ++q_) t = fma(-d[r][q_], d[c][q_], t);
                        d[r][c] = t * il[c];
                    }
                }
                const bool inK = ri >= 0 && ri < BS;
                double y[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    double w = inK ? (ri == c ? 1.0 : 0.0) : v[c];
#pragma unroll
                    for (int q_ = 0; q_ < c; ++q_) w = fma(-d[c][q_], y[q_], w);
                    y[c] = w * il[c];
                }
#pragma unroll
                for (int c = BS - 1; c >= 0; --c) {
                    double w = y[c];
#pragma unroll
                    for (int q_ = c + 1; q_ < BS; ++q_) w = fma(-d[q_][c], y[q_], w);
                    y[c] = w * il[c];
                }
                cs[kb] = inK ? 0.0 : 1.0;
#pragma unroll
                for (int c = 0; c < BS; ++c) hs[kb][c] = inK ? y[c] : -y[c];
                const double *rh = RH + (kb & 1) * BS * 8;
#pragma unroll
                for (int m = 0; m < NR; ++m) {
                    double w = cs[kb] * rhs[m];
#pragma unroll
                    for (int c = 0; c < BS; ++c) w = fma(hs[kb][c], rh[c * 8 + m], w);
                    rhs[m] = w;
                }
            }
        }
    }
    if (LEFT) NOSTAMP(10);
    if (row) {
#pragma unroll
        for (int m = 0; m < NR; ++m) a.X[(b * NR + m) * N + i] = rhs[m];
#pragma unroll
        for (int c = 0; c < M0; ++c) a.Y[(b * M0 + c) * N + i] = Y[c];
    }
}

int main(int argc, char **argv)
{
    const int B = 4096, reps = argc > 1 ? std::atoi(argv[1]) : 200;
    std::mt19937_64 rng(1);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(0.5, 5.0);
    std::vector<double> M((size_t)B * N * N), G((size_t)B * M0 * N), R((size_t)B * NR * N);
    {
        // one SPD M = Q diag Q^T, replicated (config 1: identical instances)
        std::vector<double> Q(N * N), Mi(N * N, 0.0);
        for (auto &v : Q) v = nd(rng);
        for (int c = 0; c < N; ++c) { // Gram-Schmidt
            for (int p = 0; p < c; ++p) {
                double s = 0;
                for (int r = 0; r < N; ++r) s += Q[r * N + c] * Q[r * N + p];
                for (int r = 0; r < N; ++r) Q[r * N + c] -= s * Q[r * N + p];
            }
            double s = 0;
            for (int r = 0; r < N; ++r) s += Q[r * N + c] * Q[r * N + c];
            for (int r = 0; r < N; ++r) Q[r * N + c] /= std::sqrt(s);
        }
        std::vector<double> lam(N);
        for (auto &l : lam) l = ud(rng);
        for (int r = 0; r < N; ++r)
            for (int c = 0; c < N; ++c) {
                double s = 0;
                for (int k = 0; k < N; ++k) s += Q[r * N + k] * lam[k] * Q[c * N + k];
                Mi[r * N + c] = s;
            }
        for (int r = 0; r < N; ++r)
            for (int c = 0; c < r; ++c) Mi[c * N + r] = Mi[r * N + c];
        for (int b = 0; b < B; ++b) std::memcpy(&M[(size_t)b * N * N], Mi.data(), sizeof(double) * N * N);
    }
    for (auto &v : G) v = nd(rng);
    for (auto &v : R) v = nd(rng);
    double *dM, *dG, *dR, *dX[6], *dY[2];
    unsigned long long *dst;
    CHECK(hipMalloc(&dst, sizeof(unsigned long long) * 16 * (B / 2)));
    CHECK(hipMemset(dst, 0, sizeof(unsigned long long) * 16 * (B / 2)));
    int *dsel, hsel[M0] = {0, 1, 2, 3, 4, 5};
    CHECK(hipMalloc(&dsel, sizeof(hsel)));
    CHECK(hipMemcpy(dsel, hsel, sizeof(hsel), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&dM, M.size() * 8));
    CHECK(hipMalloc(&dG, G.size() * 8));
    CHECK(hipMalloc(&dR, R.size() * 8));
    for (int v = 2; v < 6; ++v) CHECK(hipMalloc(&dX[v], R.size() * 8));
    for (int v = 0; v < 2; ++v) {
        CHECK(hipMalloc(&dX[v], R.size() * 8));
        CHECK(hipMalloc(&dY[v], G.size() * 8));
    }
    CHECK(hipMemcpy(dM, M.data(), M.size() * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dG, G.data(), G.size() * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dR, R.data(), R.size() * 8, hipMemcpyHostToDevice));
    const size_t lds = sizeof(double) * kSIZE * 2;
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<9>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<7>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<6>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipFuncSetAttribute((const void *)gj_kernel<5>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char *names[10] = {"right", "left", "right-synthetic-M", "left-synthetic-M", "stage-only", "inv-block",
                             "inv-block-synthetic-M", "chunk4", "chunk4-uni", "chunk8"};
    for (int round = 0; round < 2; ++round)
        for (int v = 0; v < 10; ++v) {
            Args a{dM, dG, dR, dX[v == 5 ? 2 : (v >= 7 ? v - 4 : (v & 1))], dY[v & 1], dst, dsel, B};
            auto launch = [&]() {
                switch (v) {
                case 0: hipLaunchKernelGGL(gj_kernel<0>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 1: hipLaunchKernelGGL(gj_kernel<1>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 2: hipLaunchKernelGGL(gj_kernel<2>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 3: hipLaunchKernelGGL(gj_kernel<3>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 5: hipLaunchKernelGGL(gj_kernel<5>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 6: hipLaunchKernelGGL(gj_kernel<6>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 7: hipLaunchKernelGGL(gj_kernel<7>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 8: hipLaunchKernelGGL(gj_kernel<8>, dim3(B / 2), dim3(64), lds, 0, a); break;
                case 9: hipLaunchKernelGGL(gj_kernel<9>, dim3(B / 2), dim3(64), lds, 0, a); break;
                default: hipLaunchKernelGGL(gj_kernel<4>, dim3(B / 2), dim3(64), lds, 0, a); break;
                }
            };
            for (int w = 0; w < 10; ++w) launch();
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0, 0));
            for (int r = 0; r < reps; ++r) launch();
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("%-6s %8.2f us/launch\n", names[v], 1000.0 * ms / reps);
            if (false) { // the last launch's stamps: mean cycles after the wave's start (s_memtime, 100 MHz?)
                std::vector<unsigned long long> h(16 * (B / 2));
                CHECK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
                unsigned long long t0 = ~0ull, t1 = 0;
                for (int w = 0; w < B / 2; ++w) {
                    t0 = std::min(t0, h[w * 16]);
                    t1 = std::max(t1, h[w * 16 + 10]);
                }
                std::printf("  launch span %llu ticks; per-wave mean ticks after its start:", t1 - t0);
                for (int k = 1; k <= 10; ++k) {
                    if (!v && k > 1 && k < 10) continue;
                    double m = 0;
                    for (int w = 0; w < B / 2; ++w) m += (double)(h[w * 16 + k] - h[w * 16]);
                    std::printf(" s%d=%.0f", k, m / (B / 2));
                }
                double m0 = 0;
                for (int w = 0; w < B / 2; ++w) m0 += (double)(h[w * 16] - t0);
                std::printf(" start=%.0f\n", m0 / (B / 2));
                CHECK(hipMemset(dst, 0, h.size() * 8));
            }
        }
    // (the comparison is of modes 0 / 1: rerun them last)
    for (int v = 0; v < 2; ++v) {
        Args a{dM, dG, dR, dX[v], dY[v], dst, dsel, B};
        if (v) hipLaunchKernelGGL(gj_kernel<1>, dim3(B / 2), dim3(64), lds, 0, a);
        else hipLaunchKernelGGL(gj_kernel<0>, dim3(B / 2), dim3(64), lds, 0, a);
    }
    CHECK(hipDeviceSynchronize());
    std::vector<double> X0(R.size()), X1(R.size()), Y0(G.size()), Y1(G.size());
    CHECK(hipMemcpy(X0.data(), dX[0], X0.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(X1.data(), dX[1], X1.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(Y0.data(), dY[0], Y0.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(Y1.data(), dY[1], Y1.size() * 8, hipMemcpyDeviceToHost));
    double dx = 0, dy = 0, res = 0;
    for (size_t k = 0; k < X0.size(); ++k) dx = std::fmax(dx, std::fabs(X0[k] - X1[k]));
    for (size_t k = 0; k < Y0.size(); ++k) dy = std::fmax(dy, std::fabs(Y0[k] - Y1[k]));
    for (int m = 0; m < NR; ++m) // residual of instance 0: M x - r
        for (int r = 0; r < N; ++r) {
            double s = -R[m * N + r];
            for (int c = 0; c < N; ++c) s += M[r * N + c] * X0[m * N + c];
            res = std::fmax(res, std::fabs(s));
        }
    double res1 = 0;
    for (int m = 0; m < NR; ++m)
        for (int r = 0; r < N; ++r) {
            double s = -R[m * N + r];
            for (int c = 0; c < N; ++c) s += M[r * N + c] * X1[m * N + c];
            res1 = std::fmax(res1, std::fabs(s));
        }
    std::printf("max |X_right - X_left| %.3e, max |Y_right - Y_left| %.3e, residual right %.3e left %.3e\n", dx, dy,
                res, res1);
    {
        std::vector<double> X2(R.size());
        CHECK(hipMemcpy(X2.data(), dX[2], X2.size() * 8, hipMemcpyDeviceToHost));
        double d2 = 0, r2 = 0, xm = 0;
        for (size_t k = 0; k < X0.size(); ++k) {
            d2 = std::fmax(d2, std::fabs(X0[k] - X2[k]));
            xm = std::fmax(xm, std::fabs(X0[k]));
        }
        for (int m = 0; m < NR; ++m)
            for (int r = 0; r < N; ++r) {
                double s = -R[m * N + r];
                for (int c = 0; c < N; ++c) s += M[r * N + c] * X2[m * N + c];
                r2 = std::fmax(r2, std::fabs(s));
            }
        std::printf("inv-block: max |X - X_right| %.3e (max |X| %.3e), residual %.3e\n", d2, xm, r2);
        for (int v = 3; v < 6; ++v) {
            CHECK(hipMemcpy(X2.data(), dX[v], X2.size() * 8, hipMemcpyDeviceToHost));
            double dv = 0;
            for (size_t k = 0; k < X0.size(); ++k) dv = std::fmax(dv, std::fabs(X0[k] - X2[k]));
            std::printf("%s: max |X - X_right| %.3e\n", names[v + 4], dv);
        }
    }
    return 0;
}
