// qppvm_repair.h -- pieces of the QPPVM path shared by the W1 = I kernels
// (qppvm_kernel.hip) and the W1 = M kernels (qppvm_w1m_kernel.hip): the active-set LDS
// layout, the level-0 repair (BVLS for y*, pins) and the follow-up work lists.
#pragma once
#include "wbq_kernels.h"
#include "wbq_device.h"

namespace wbq {

template <int NP>
struct ActiveLayout {
    static constexpr bool MREG = (NP == 32); // M rows and T rows in VGPRs (else in LDS)
    static constexpr int RS = NP + 1;
    int NR, QA, MA, TT, ZR, U, D1, D1B, NV, BC, SIZE;
    // n (NP = 64, round 6): the three row regions hold the rows an n-joint instance can use -- n rounded up to 8,
    // Q1^T's basis has at most n rows, M's and T's rows past n are padding -- instead of 64 (n = 39: 40 rows,
    // 101 -> 64 KB, two instances per CU instead of one); the lanes past NR read a zero row (ZR) and write nothing
    __host__ __device__ ActiveLayout(int, int, int n = NP)
    {
        NR = MREG ? NP : (n < NP ? ((n + 7) & ~7) : NP);
        QA = 0;                           // Q1^T rows [NR][RS]
        MA = QA + NR * RS;                // M rows (NP == 64)
        TT = MA + (MREG ? 0 : NR * RS);   // T = R_II^-1 rows (NP == 64)
        ZR = TT + (MREG ? 0 : NR * RS);   // a zero row (NP == 64)
        U = ZR + (MREG ? 0 : RS + 1);     // u
        D1 = U + NP;                      // d1 = Q1^T n_p, zero-padded to 2 NP
        D1B = D1 + 2 * NP;                // second Gram-Schmidt pass
        NV = D1B + NP;                    // n_p
        BC = NV + NP;                     // broadcast scratch
        SIZE = (BC + NP + 1) & ~1;
    }
};

// ============================================================== level-0 repair
// Packed lower triangle index (row-major).
__host__ __device__ constexpr int tri(int r, int c) { return r * (r + 1) / 2 + c; }

// Diagonal-pivoted Cholesky of a PSD K x K Gram held redundantly per lane (packed lower,
// original row order; rows >= m ignored): P Gram P^T = L L^T, rank k = number of pivots
// above tol * max diagonal. Pivoting keeps the left-over Schur diagonal at roundoff level,
// so the rank decision is reliable (without it, a small genuine pivot inflates the
// dependent rows' pivots far above roundoff). Static register indices throughout: the
// dynamic pivot is applied with select chains.
template <int K>
struct PivChol {
    static constexpr int T = K * (K + 1) / 2;
    int k;           // rank
    int piv[K];      // original row of pivot c (c < k)
    bool used[K];    // row pivoted (or >= m)
    double Lp[T];    // L restricted to the pivot rows, step order (packed lower)
    double Lo[K][K]; // L row of every original row (columns = pivot steps)

    __device__ static double gsym(const double (&g)[T], int i, int p)
    {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) v = (q == p) ? g[i >= q ? tri(i, q) : tri(q, i)] : v;
        return v;
    }

    // pivots at or below tol * (largest diagonal), and below `floor` (absolute: a matrix that is zero
    // up to roundoff has rank 0, which a relative cut alone would not see), end the factorisation
    __device__ void factor(const double (&g)[T], int m, double tol, double floor = 0.0)
    {
        double d[K], dmx = 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            d[i] = i < m ? g[tri(i, i)] : 0.0;
            dmx = fmax(dmx, d[i]);
            used[i] = i >= m;
            piv[i] = 0;
#pragma unroll
            for (int c = 0; c < K; ++c) Lo[i][c] = 0.0;
        }
#pragma unroll
        for (int t = 0; t < T; ++t) Lp[t] = 0.0;
        k = 0;
        bool stop = false;
#pragma unroll
        for (int c = 0; c < K; ++c) {
            int p = 0;
            double best = -1.0;
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (!used[i] && d[i] > best) {
                    best = d[i];
                    p = i;
                }
            stop = stop || !(best > tol * dmx) || !(best > floor);
            if (!stop) {
                piv[c] = p;
                k = c + 1;
                const double il = frsq(best), lpp = best * il; // (hardware estimate + Newton, ~0.5 ulp)
                double rp[K];
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    double v = 0.0;
#pragma unroll
                    for (int i = 0; i < K; ++i) v = (i == p) ? Lo[i][j] : v;
                    rp[j] = v;
                }
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    used[i] = used[i] || i == p;
                    if (!used[i]) {
                        double v = gsym(g, i, p);
#pragma unroll
                        for (int j = 0; j < c; ++j) v = fma(-Lo[i][j], rp[j], v);
                        v *= il;
                        Lo[i][c] = v;
                        d[i] = fma(-v, v, d[i]);
                    }
                    if (i == p) Lo[i][c] = lpp;
                }
#pragma unroll
                for (int j = 0; j < c; ++j) Lp[tri(c, j)] = rp[j];
                Lp[tri(c, c)] = lpp;
            }
        }
    }

    // Weights w (original row order) of the minimum-norm least-squares solution z = A^T w of
    // A z = r, where Gram = A A^T (rows m..K-1 absent). With C = L_D L_P^-1 relating the
    // dependent rows D to the pivot rows P:
    //   s = (I + C^T C)^-1 (r_P + C^T r_D),  w_P = Gram_PP^-1 s,  w_D = 0
    // (the oracle does this solve with an SVD: oracle/wbq_oracle.c:minnorm_ls).
    __device__ void solve(const double (&r)[K], int m, double (&w)[K]) const
    {
        double rh[K], H[T];
#pragma unroll
        for (int c = 0; c < K; ++c) {
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < K; ++i) v = (c < k && piv[c] == i) ? r[i] : v;
            rh[c] = v;
        }
#pragma unroll
        for (int p = 0; p < K; ++p)
#pragma unroll
            for (int q = 0; q <= p; ++q) H[tri(p, q)] = p == q ? 1.0 : 0.0;
        double ild[K];
#pragma unroll
        for (int c = 0; c < K; ++c) ild[c] = c < k ? frcp(Lp[tri(c, c)]) : 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            bool dep = i < m;
#pragma unroll
            for (int c = 0; c < K; ++c) dep = dep && !(c < k && piv[c] == i);
            if (dep) {
                double ci[K];
#pragma unroll
                for (int c = K - 1; c >= 0; --c) {
                    double v = Lo[i][c];
#pragma unroll
                    for (int c2 = c + 1; c2 < K; ++c2) v = fma(-Lp[tri(c2, c)], ci[c2], v);
                    ci[c] = v * ild[c];
                }
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    rh[p] = fma(ci[p], r[i], rh[p]);
#pragma unroll
                    for (int q = 0; q <= p; ++q) H[tri(p, q)] = fma(ci[p], ci[q], H[tri(p, q)]);
                }
            }
        }
        double ih[K]; // Cholesky of H (SPD, well conditioned: |C| is bounded under pivoting)
#pragma unroll
        for (int c = 0; c < K; ++c) {
            double dd = H[tri(c, c)];
#pragma unroll
            for (int j = 0; j < c; ++j) dd = fma(-H[tri(c, j)], H[tri(c, j)], dd);
            ih[c] = frsq(dd);
            H[tri(c, c)] = dd * ih[c];
#pragma unroll
            for (int r2 = c + 1; r2 < K; ++r2) {
                double t = H[tri(r2, c)];
#pragma unroll
                for (int j = 0; j < c; ++j) t = fma(-H[tri(r2, j)], H[tri(c, j)], t);
                H[tri(r2, c)] = t * ih[c];
            }
        }
        double sv[K];
#pragma unroll
        for (int c = 0; c < K; ++c) {
            double v = rh[c];
#pragma unroll
            for (int j = 0; j < c; ++j) v = fma(-H[tri(c, j)], sv[j], v);
            sv[c] = v * ih[c];
        }
#pragma unroll
        for (int c = K - 1; c >= 0; --c) {
            double v = sv[c];
#pragma unroll
            for (int j = c + 1; j < K; ++j) v = fma(-H[tri(j, c)], sv[j], v);
            sv[c] = v * ih[c];
        }
        // w_P = L_P^-T L_P^-1 s
#pragma unroll
        for (int c = 0; c < K; ++c) {
            double v = sv[c];
#pragma unroll
            for (int j = 0; j < c; ++j) v = fma(-Lp[tri(c, j)], sv[j], v);
            sv[c] = v * ild[c];
        }
#pragma unroll
        for (int c = K - 1; c >= 0; --c) {
            double v = sv[c];
#pragma unroll
            for (int j = c + 1; j < K; ++j) v = fma(-Lp[tri(j, c)], sv[j], v);
            sv[c] = v * ild[c];
        }
#pragma unroll
        for (int i = 0; i < K; ++i) {
            double v = 0.0;
#pragma unroll
            for (int c = 0; c < K; ++c) v = (c < k && piv[c] == i) ? sv[c] : v;
            w[i] = v;
        }
    }

    // Orthonormal basis of range(A^T) (lane-distributed rows): q_c = (L_P^-1 a_P)[c], c < k
    __device__ void basis(const double (&acol)[K], double (&q)[K]) const
    {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < K; ++i) v = (piv[c] == i) ? acol[i] : v;
#pragma unroll
            for (int j = 0; j < c; ++j) v = fma(-Lp[tri(c, j)], q[j], v);
            q[c] = c < k ? v * frcp(Lp[tri(c, c)]) : 0.0;
        }
    }
};

// w = Gram^-1 r by an unpivoted Cholesky of the leading m x m block of a packed PSD Gram (every lane
// alike, static indices: ~K^3 / 6 FMAs instead of PivChol's select chains). Returns false -- w
// untouched -- unless every pivot exceeds tol * (largest diagonal): then the Gram is far from
// singular, no rank decision is needed, and the caller's PivChol path (the same solution for a full
// rank Gram) is skipped. The BVLS steps of the level-0 repair are mostly such full-rank solves.
template <int K>
__device__ __forceinline__ bool chol_solve_full(const double (&g)[K * (K + 1) / 2], int m, const double (&r)[K],
                                                double (&w)[K], double tol)
{
    double L[K * (K + 1) / 2], il[K], dmx = 0.0;
    bool ok = true;
#pragma unroll
    for (int c = 0; c < K; ++c) dmx = fmax(dmx, c < m ? g[tri(c, c)] : 0.0);
#pragma unroll
    for (int c = 0; c < K; ++c) {
        double dd = c < m ? g[tri(c, c)] : 1.0;
#pragma unroll
        for (int k = 0; k < c; ++k) dd = fma(-L[tri(c, k)], L[tri(c, k)], dd);
        ok = ok && (c >= m || dd > tol * dmx);
        const double ic = c < m ? frsq(fmax(dd, 1e-300)) : 0.0;
        il[c] = ic;
        L[tri(c, c)] = dd * ic;
#pragma unroll
        for (int rr = c + 1; rr < K; ++rr) {
            double t = (rr < m && c < m) ? g[tri(rr, c)] : 0.0;
#pragma unroll
            for (int k = 0; k < c; ++k) t = fma(-L[tri(rr, k)], L[tri(c, k)], t);
            L[tri(rr, c)] = t * ic;
        }
    }
    if (!ok || !(dmx > 0.0)) return false;
    double y[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        double v = c < m ? r[c] : 0.0;
#pragma unroll
        for (int k = 0; k < c; ++k) v = fma(-L[tri(c, k)], y[k], v);
        y[c] = v * il[c];
    }
#pragma unroll
    for (int c = K - 1; c >= 0; --c) {
        double v = y[c];
#pragma unroll
        for (int k = c + 1; k < K; ++k) v = fma(-L[tri(k, c)], y[k], v);
        y[c] = v * il[c];
    }
#pragma unroll
    for (int c = 0; c < K; ++c) w[c] = c < m ? y[c] : 0.0;
    return true;
}

// Acceptance threshold of chol_solve_full's pivots (relative to the largest diagonal). It must be far
// above PivChol's rank cut (1e-12): an unpivoted pivot bounds the smallest eigenvalue only up to a factor
// that grows with K, so a Gram whose unpivoted pivots all pass 1e-10 can still be rank deficient to the
// pivoted factorisation, and the plain solve then takes a huge ill-conditioned step where PivChol takes
// the minimum-norm one. With 1e-10 a W1 = M config-2 instance's BVLS cycled to its cap and returned a
// wrong y* (tests/test_gpu_kkt.py; replayed in numpy: 1,600 steps vs 26, y* off by 2 %); at 1e-6 (1e-4 for
// 12 rows) the fast path only takes Grams PivChol also finds well inside full rank.
template <int K>
constexpr double kCholFastTol = K <= 6 ? 1e-6 : 1e-4;


// The BVLS free-set step in the column space, for a free set of at most m0 variables: with A_F (m0 x
// kfree) of full column rank the minimum-norm least-squares step is z_F = (A_F^T A_F)^-1 A_F^T r, a
// kfree x kfree SPD solve. The free columns are gathered into slots by ballot + v_readlane (per 32-lane
// half for NP = 32), every lane factors the small column Gram (unpivoted, static indices) and a free lane
// takes its slot's component. The row Gram A_F A_F^T of such a step is rank deficient, so the row-space
// path ran PivChol's select-chain factorisation: ~9.5k of a config-4 repair step's ~18k cycles
// (scripts/diag_mpc_repair.py). Accepted only when every pivot exceeds tol * (largest diagonal), the
// regime where PivChol on the row Gram (the same nonzero spectrum) finds full rank kfree and returns the
// same step; otherwise (dependent free columns) the caller's row path runs. Returns acceptance (the
// instance's lanes agree); z is this lane's component (free lanes only).
template <int NP, int M0>
__device__ __forceinline__ bool bvls_col_step(const double (&acol)[M0], const double (&rv)[M0], bool fr, double tol,
                                              double &z)
{
    const unsigned long long bal = __ballot(fr);
    const bool upper = NP == 32 && (threadIdx.x & 32);
    unsigned long long m0m = NP == 32 ? (bal & 0xffffffffull) : bal, m1m = NP == 32 ? (bal >> 32) : 0ull;
    const int lane = threadIdx.x & (NP - 1);
    const unsigned long long mine = upper ? m1m : m0m;
    const int kf = __popcll(mine);
    const int slot = __popcll(mine & ((1ull << lane) - 1ull));
    double col[M0][M0]; // [slot][row]
#pragma unroll
    for (int q = 0; q < M0; ++q) {
        const bool v0 = m0m != 0, v1 = m1m != 0;
        const int l0 = v0 ? (int)__builtin_ctzll(m0m) : 0, l1 = v1 ? (int)__builtin_ctzll(m1m) : 0;
        m0m &= m0m - 1ull;
        m1m &= m1m - 1ull;
#pragma unroll
        for (int r = 0; r < M0; ++r) {
            const double a0 = lane_f64(acol[r], l0);
            double v = v0 ? a0 : 0.0;
            if constexpr (NP == 32) {
                const double a1 = lane_f64(acol[r], 32 + l1);
                v = upper ? (v1 ? a1 : 0.0) : v;
            }
            col[q][r] = v;
        }
    }
    double L[M0 * (M0 + 1) / 2], d[M0], il[M0], cmx = 0.0;
#pragma unroll
    for (int q = 0; q < M0; ++q) {
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < M0; ++r) v = fma(col[q][r], rv[r], v);
        d[q] = v;
#pragma unroll
        for (int t = 0; t <= q; ++t) {
            double c = 0.0;
#pragma unroll
            for (int r = 0; r < M0; ++r) c = fma(col[q][r], col[t][r], c);
            L[tri(q, t)] = c;
        }
        cmx = fmax(cmx, L[tri(q, q)]);
    }
    bool ok = kf > 0;
#pragma unroll
    for (int c = 0; c < M0; ++c) {
        double dd = c < kf ? L[tri(c, c)] : 1.0;
#pragma unroll
        for (int k = 0; k < c; ++k) dd = fma(-L[tri(c, k)], L[tri(c, k)], dd);
        ok = ok && (c >= kf || dd > tol * cmx);
        const double ic = frsq(fmax(dd, 1e-300));
        il[c] = ic;
        L[tri(c, c)] = dd * ic;
#pragma unroll
        for (int r = c + 1; r < M0; ++r) {
            double t = (r < kf && c < kf) ? L[tri(r, c)] : 0.0;
#pragma unroll
            for (int k = 0; k < c; ++k) t = fma(-L[tri(r, k)], L[tri(c, k)], t);
            L[tri(r, c)] = t * ic;
        }
    }
    double y[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) {
        double v = c < kf ? d[c] : 0.0;
#pragma unroll
        for (int k = 0; k < c; ++k) v = fma(-L[tri(c, k)], y[k], v);
        y[c] = v * il[c];
    }
#pragma unroll
    for (int c = M0 - 1; c >= 0; --c) {
        double v = y[c];
#pragma unroll
        for (int k = c + 1; k < M0; ++k) v = fma(-L[tri(k, c)], y[k], v);
        y[c] = v * il[c];
    }
    double zz = 0.0;
#pragma unroll
    for (int q = 0; q < M0; ++q) zz = (q == slot) ? y[q] : zz;
    z = zz;
    return ok && cmx > 0.0;
}

// The same column-space step for the 12-row stacks (two 6-row tasks on level 0, the plugin's own
// configuration), through the instance's LDS scratch (>= M0 * M0 + NT + M0 doubles, dead during BVLS): a
// 12 x 12 slot matrix would not fit in registers. Free lanes write their columns into slots, lane e forms
// entry e of the column Gram (or of A_F^T r) from them, and every lane reads the packed Gram back and
// factors it as bvls_col_step does. Wave-uniform call (barriers).
template <int NP, int M0>
__device__ __forceinline__ bool bvls_col_step_lds(const double (&acol)[M0], const double (&rv)[M0], bool fr, double tol,
                                                  double &z, double *lds)
{
    constexpr int NT = M0 * (M0 + 1) / 2;
    const unsigned long long bal = __ballot(fr);
    const bool upper = NP == 32 && (threadIdx.x & 32);
    const unsigned long long mine = NP == 32 ? (upper ? (bal >> 32) : (bal & 0xffffffffull)) : bal;
    const int lane = threadIdx.x & (NP - 1);
    const int kf = __popcll(mine);
    const int slot = __popcll(mine & ((1ull << lane) - 1ull));
    double *colm = lds, *ent = lds + M0 * M0;
    __syncthreads(); // (the region's previous readers are done)
    if (fr && slot < M0) {
#pragma unroll
        for (int r = 0; r < M0; ++r) colm[slot * M0 + r] = acol[r];
    }
    __syncthreads();
    for (int e = lane; e < NT + M0; e += NP) {
        double v = 0.0;
        if (e < NT) {
            int q = 0;
            while ((q + 1) * (q + 2) / 2 <= e) ++q;
            const int t = e - q * (q + 1) / 2;
            if (q < kf && t < kf)
#pragma unroll
                for (int r = 0; r < M0; ++r) v = fma(colm[q * M0 + r], colm[t * M0 + r], v);
        } else {
            const int q = e - NT;
            if (q < kf)
#pragma unroll
                for (int r = 0; r < M0; ++r) v = fma(colm[q * M0 + r], rv[r], v);
        }
        ent[e] = v;
    }
    __syncthreads();
    double L[NT], d[M0], il[M0], cmx = 0.0;
#pragma unroll
    for (int e = 0; e < NT; ++e) L[e] = ent[e];
#pragma unroll
    for (int q = 0; q < M0; ++q) {
        d[q] = ent[NT + q];
        cmx = fmax(cmx, L[tri(q, q)]);
    }
    bool ok = kf > 0 && kf <= M0;
#pragma unroll
    for (int c = 0; c < M0; ++c) {
        double dd = c < kf ? L[tri(c, c)] : 1.0;
#pragma unroll
        for (int k = 0; k < c; ++k) dd = fma(-L[tri(c, k)], L[tri(c, k)], dd);
        ok = ok && (c >= kf || dd > tol * cmx);
        const double ic = frsq(fmax(dd, 1e-300));
        il[c] = ic;
        L[tri(c, c)] = dd * ic;
#pragma unroll
        for (int r = c + 1; r < M0; ++r) {
            double t = (r < kf && c < kf) ? L[tri(r, c)] : 0.0;
#pragma unroll
            for (int k = 0; k < c; ++k) t = fma(-L[tri(r, k)], L[tri(c, k)], t);
            L[tri(r, c)] = t * ic;
        }
    }
    double y[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) {
        double v = c < kf ? d[c] : 0.0;
#pragma unroll
        for (int k = 0; k < c; ++k) v = fma(-L[tri(c, k)], y[k], v);
        y[c] = v * il[c];
    }
#pragma unroll
    for (int c = M0 - 1; c >= 0; --c) {
        double v = y[c];
#pragma unroll
        for (int k = c + 1; k < M0; ++k) v = fma(-L[tri(k, c)], y[k], v);
        y[c] = v * il[c];
    }
    double zz = 0.0;
#pragma unroll
    for (int q = 0; q < M0; ++q) zz = (q == slot) ? y[q] : zz;
    z = zz;
    return ok && cmx > 0.0;
}

// BVLS (Stark-Parker; the algorithm of oracle/wbq_oracle.c:wbq_ref_level0) on
//   min 0.5 ||A z - b||^2  s.t.  lo <= z <= hi
// with lane i owning variable z_i and its column acol (rows c < m0 of the M0 slots) and every lane
// holding b; padding lanes have row = false (never free). active = this instance runs (lanes of an
// instance agree); st0 = the start state of the lane (0 free, -1 at lo, +1 at hi: a warm start,
// any state is valid). Returns the lane's z_i, its final state, the iterations and whether the
// iteration cap ended it.
struct BvlsOut {
    double xv;
    int st, it;
    bool capped;
#ifdef WBQ_STAMPS
    unsigned long long ph[8]; // diagnostic build: cycles in the step's parts, fast / pivoted solves
#endif
};
#ifdef WBQ_STAMPS
#define WBQ_T(v) do { __builtin_amdgcn_sched_barrier(0); v = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define WBQ_T(v) do {} while (0)
#endif
template <int NP, int M0>
__device__ __forceinline__ BvlsOut bvls(const double (&acol)[M0], const double (&b0v)[M0], int m0, double lo,
                                        double hi, bool row, bool active, int st0, int maxit, double *lds = nullptr)
{
    constexpr int NT = M0 * (M0 + 1) / 2;
    const int i = threadIdx.x & (NP - 1); // lane within the instance
    BvlsOut out{0.0, 0, 0, false};
#ifdef WBQ_STAMPS
    for (int k = 0; k < 8; ++k) out.ph[k] = 0;
#endif
    unsigned long long t0 = 0, t1 = 0;
    (void)t0;
    (void)t1;
    double xv = row ? fmin(fmax(0.0, lo), hi) : 0.0;
    int st = row ? 0 : 2; // 0 free, -1 at lo, +1 at hi, 2 padding lane (never free)
    if (row && st0 != 0) {
        st = st0 < 0 ? -1 : 1;
        xv = st < 0 ? lo : hi;
    }
    if (row && lo == hi) {
        st = -1;
        xv = lo;
    }
    bool ex = false; // excluded from the next KKT pick (Stark-Parker anti-cycling)
    double abm = 0.0;
#pragma unroll
    for (int c = 0; c < M0; ++c) abm = fma(acol[c], b0v[c], abm);
    const double wtb = fabs(abm);
    abm = fmax(1.0, imax<NP>(wtb));
    int freed = -1, it = 0;
    bool outer = active;
    while (__any(outer)) {
        bool inner = outer;
        while (__any(inner)) {
            if (inner) ++it;
            WBQ_T(t0);
            const bool fr = inner && st == 0;
            double rv[M0];
#pragma unroll
            for (int c = 0; c < M0; ++c) rv[c] = (st == -1 || st == 1) ? acol[c] * xv : 0.0;
            isum_vec<NP, M0>(rv);
            const double kfree = isum<NP>(fr ? 1.0 : 0.0);
#pragma unroll
            for (int c = 0; c < M0; ++c) rv[c] = b0v[c] - rv[c];
            WBQ_T(t1);
#ifdef WBQ_STAMPS
            out.ph[0] += t1 - t0;
            t0 = t1;
#endif
            // minimum-norm least squares on the free set: at most m0 free variables in the column space
            // (bvls_col_step); else z = A_F^T w, a full-rank row Gram by the plain Cholesky, a nearly
            // singular one by the rank-revealing PivChol
            double zc = 0.0;
            bool cok = false;
            {
                const bool colp = inner && kfree > 0.0 && kfree <= (double)m0;
                if constexpr (M0 <= 6) {
                    if (__any(colp)) cok = bvls_col_step<NP, M0>(acol, rv, fr, kCholFastTol<M0>, zc) && colp;
                } else { // (a 12 x 12 slot matrix: through LDS)
                    if (lds && __any(colp))
                        cok = bvls_col_step_lds<NP, M0>(acol, rv, fr, kCholFastTol<M0>, zc, lds) && colp;
                }
            }
            double wv[M0];
#pragma unroll
            for (int c = 0; c < M0; ++c) wv[c] = 0.0;
            if (__any(inner && !cok)) {
                // the row Gram (only where some instance of the wave needs the row-space step)
                double gp[NT];
#pragma unroll
                for (int p = 0; p < M0; ++p)
#pragma unroll
                    for (int c = 0; c <= p; ++c) gp[tri(p, c)] = fr ? acol[p] * acol[c] : 0.0;
                isum_vec<NP, NT>(gp);
                if (!chol_solve_full<M0>(gp, m0, rv, wv, kCholFastTol<M0>)) { // (per instance)
                    PivChol<M0> pc;
                    pc.factor(gp, m0, 1e-12);
                    pc.solve(rv, m0, wv);
#ifdef WBQ_STAMPS
                    out.ph[6] += cok ? 0 : 1;
#endif
                }
#ifdef WBQ_STAMPS
                else out.ph[5] += cok ? 0 : 1;
#endif
            }
#ifdef WBQ_STAMPS
            out.ph[7] += cok ? 1 : 0;
            WBQ_T(t1);
            out.ph[1] += t1 - t0;
            t0 = t1;
#endif
            double z = 0.0;
#pragma unroll
            for (int c = 0; c < M0; ++c) z = fma(acol[c], wv[c], z);
            if (cok) z = zc;
            // interpolate back into the box: blocking variable = smallest step fraction < 1
            double al = kInf;
            if (fr) {
                const double step = z - xv;
                if (z < lo && step < 0.0) al = (lo - xv) / step;
                else if (z > hi && step > 0.0) al = (hi - xv) / step;
                if (!(al < 1.0)) al = kInf;
            }
            int jb = i;
            iargmin<NP>(al, jb);
#ifdef WBQ_STAMPS
            WBQ_T(t1);
            out.ph[2] += t1 - t0;
            t0 = t1;
#endif
            if (inner) {
                if (!(kfree > 0.0)) {
                    inner = false;
                } else if (al >= kInf) { // z inside the box: take it
                    if (fr) xv = z;
                    freed = -1;
                    ex = false; // progress: exclusions expire
                    inner = false;
                } else {
                    const double alpha = fmax(al, 0.0);
                    if (jb == freed && alpha == 0.0) {
                        // the variable just freed wants back through its bound: re-bind, exclude
                        if (i == jb) {
                            ex = true;
                            st = (z < lo) ? -1 : 1;
                            xv = st < 0 ? lo : hi;
                        }
                        inner = false;
                    } else {
                        ex = false; // progress: exclusions expire
                        if (fr) {
                            xv = fma(alpha, z - xv, xv);
                            const double tl = 1e-14 * fmax(1.0, fabs(lo)), tu = 1e-14 * fmax(1.0, fabs(hi));
                            if (i == jb) st = (z < lo) ? -1 : 1;
                            else if (xv <= lo + tl && z < lo) st = -1;
                            else if (xv >= hi - tu && z > hi) st = 1;
                            if (st == -1) xv = lo;
                            if (st == 1) xv = hi;
                        }
                    }
                    freed = -1;
                    if (it >= maxit) inner = false;
                }
            }
#ifdef WBQ_STAMPS
            WBQ_T(t1);
            out.ph[3] += t1 - t0;
#endif
        }
        // KKT on the bound variables: w = A0^T (b0 - A0 x)
        WBQ_T(t0);
        double rf[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) rf[c] = acol[c] * xv;
        isum_vec<NP, M0>(rf);
        double w = 0.0, wx = 0.0;
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            w = fma(acol[c], b0v[c] - rf[c], w);
            wx = fma(acol[c], rf[c], wx);
        }
        // KKT tolerance relative to the terms of w = A0^T b0 - A0^T A0 x (with b0 ~ 0 the
        // second dominates, and its roundoff must not read as a descent direction)
        const double wtol = 1e-11 * fmax(abm, imax<NP>(fmax(wtb, fabs(wx))));
        double v = -kInf;
        if (outer && (st == -1 || st == 1) && !ex && lo != hi) v = st < 0 ? w : -w;
        int best = i;
        iargmax<NP>(v, best);
        if (outer) {
            if (!(v > wtol)) {
                outer = false;
            } else if (it >= maxit) {
                out.capped = true;
                outer = false;
            } else {
                if (i == best) st = 0; // exclusions persist until the inner loop makes progress
                freed = best;
            }
        }
#ifdef WBQ_STAMPS
        WBQ_T(t1);
        out.ph[4] += t1 - t0;
#endif
    }
    out.xv = xv;
    out.st = st;
    out.it = it;
    return out;
}

// BVLS with equality rows (the middle level of a three-level stack, wbq_desc.task_level: the elbow
// tasks of QPPVMPlugin.cpp:154-166,177-178; the oracle's wbq_ref_level_mid states the same steps with
// SVDs):
//   min 0.5 ||A1 z - b1||^2  s.t.  A0 z = A0 z_start (level 0 at its optimum),  lo <= z <= hi,
// from a feasible z_start (the level-0 point) with box state st0. Lane i owns variable z_i with its
// level-0 column ae (me rows) and level-1 column ao (mo rows). A free-set step keeps A0_F dz = 0: with
// Q0 = A0_F^T L^-T (PivChol<ME>::basis on each lane's own column; orthonormal basis of range(A0_F^T))
// and T = Q0^T A1_F^T, the projected level-1 Gram is S = K11 - T^T T, beta = S^+ r1 and
//   dz_j = a1_j . beta - q0_j . (T beta)  (= (P A1^T beta)_j, P = I - Q0 Q0^T),
// interpolated back into the box as BVLS; the multipliers of bound variables are
//   w_j = a1_j . r1 - (A0^T nu)_j,  A0_F^T nu = Q0 Q0^T g_F  =>  (A0^T nu)_j = qe_j . (Q0^T g_F),
// qe_j = L^-1 of lane j's own level-0 column (every lane, bound or free).
struct BvlsEqOut {
    double xv, w; // z_i and its final multiplier w_i (a bound variable held by it: |w_i| large)
    int st, it;
    bool capped;
};
template <int NP, int ME, int MO>
__device__ __forceinline__ BvlsEqOut bvls_eq(const double (&ae)[ME], int me, const double (&ao)[MO], const double (&bo)[MO],
                                             int mo, double lo, double hi, bool row, bool active, double x0, int st0,
                                             int maxit)
{
    constexpr int TE = ME * (ME + 1) / 2, TO = MO * (MO + 1) / 2;
    const int i = threadIdx.x & (NP - 1); // lane within the instance
    BvlsEqOut out{0.0, 0.0, 0, 0, false};
    double xv = row ? fmin(fmax(x0, lo), hi) : 0.0;
    int st = row ? st0 : 2;
    if (row && lo == hi) st = -1;
    if (st == -1) xv = lo;
    if (st == 1) xv = hi;
    bool ex = false;
    double abm = 0.0;
#pragma unroll
    for (int c = 0; c < MO; ++c) abm = fma(ao[c], bo[c], abm);
    const double wtb = fabs(abm);
    abm = fmax(1.0, imax<NP>(wtb));
    int freed = -1, it = 0;
    // the free set's projection: qe = L^-1 of this lane's level-0 column (PivChol of K00 = A0_F A0_F^T),
    // T = Q0^T A1_F^T, S = K11 - T^T T; k11d the diagonal of K11
    auto project = [&](bool fr, double (&qe)[ME], double (&S)[TO], double (&Tm)[ME][MO], double &k11max) {
        double k00[TE], k11[TO];
#pragma unroll
        for (int p = 0; p < ME; ++p)
#pragma unroll
            for (int c = 0; c <= p; ++c) k00[tri(p, c)] = fr ? ae[p] * ae[c] : 0.0;
#pragma unroll
        for (int p = 0; p < MO; ++p)
#pragma unroll
            for (int c = 0; c <= p; ++c) k11[tri(p, c)] = fr ? ao[p] * ao[c] : 0.0;
        isum_vec<NP, TE>(k00);
        isum_vec<NP, TO>(k11);
        PivChol<ME> pe;
        pe.factor(k00, me, 1e-12);
        pe.basis(ae, qe);
        double tv[ME * MO];
#pragma unroll
        for (int p = 0; p < ME; ++p)
#pragma unroll
            for (int c = 0; c < MO; ++c) tv[p * MO + c] = fr ? qe[p] * ao[c] : 0.0;
        isum_vec<NP, ME * MO>(tv);
        k11max = 0.0;
#pragma unroll
        for (int p = 0; p < ME; ++p)
#pragma unroll
            for (int c = 0; c < MO; ++c) Tm[p][c] = tv[p * MO + c];
#pragma unroll
        for (int p = 0; p < MO; ++p) {
            k11max = fmax(k11max, k11[tri(p, p)]);
#pragma unroll
            for (int c = 0; c <= p; ++c) {
                double v = k11[tri(p, c)];
#pragma unroll
                for (int e = 0; e < ME; ++e) v = fma(-Tm[e][p], Tm[e][c], v);
                S[tri(p, c)] = v;
            }
        }
    };
    bool outer = active;
    while (__any(outer)) {
        bool inner = outer;
        while (__any(inner)) {
            if (inner) ++it;
            const bool fr = inner && row && st == 0;
            const double kfree = isum<NP>(fr ? 1.0 : 0.0);
            double qe[ME], S[TO], Tm[ME][MO], k11max;
            project(fr, qe, S, Tm, k11max);
            double rv[MO];
#pragma unroll
            for (int c = 0; c < MO; ++c) rv[c] = row ? ao[c] * xv : 0.0;
            isum_vec<NP, MO>(rv);
#pragma unroll
            for (int c = 0; c < MO; ++c) rv[c] = bo[c] - rv[c];
            PivChol<MO> ps;
            ps.factor(S, mo, 1e-12, 1e-12 * k11max);
            double beta[MO], tb[ME];
            ps.solve(rv, mo, beta);
#pragma unroll
            for (int e = 0; e < ME; ++e) {
                double v = 0.0;
#pragma unroll
                for (int c = 0; c < MO; ++c) v = fma(Tm[e][c], beta[c], v);
                tb[e] = v;
            }
            double dz = 0.0;
            if (fr) {
#pragma unroll
                for (int c = 0; c < MO; ++c) dz = fma(ao[c], beta[c], dz);
#pragma unroll
                for (int e = 0; e < ME; ++e) dz = fma(-qe[e], tb[e], dz);
            }
            double al = kInf;
            if (fr) {
                const double zt = xv + dz;
                if (zt < lo && dz < 0.0) al = fmax(0.0, (lo - xv) / dz);
                else if (zt > hi && dz > 0.0) al = fmax(0.0, (hi - xv) / dz);
                if (!(al < 1.0)) al = kInf;
            }
            int jb = i;
            iargmin<NP>(al, jb);
            if (inner) {
                if (!(kfree > 0.0) || ps.k == 0) { // no direction left on the free set
                    inner = false;
                } else if (al >= kInf) { // the step stays in the box: take it
                    if (fr) xv += dz;
                    freed = -1;
                    ex = false;
                    inner = false;
                } else {
                    const double alpha = fmax(al, 0.0);
                    if (jb == freed && alpha == 0.0) { // Stark-Parker: re-bind the variable just freed
                        if (i == jb) {
                            ex = true;
                            st = dz < 0.0 ? -1 : 1;
                            xv = st < 0 ? lo : hi;
                        }
                        inner = false;
                    } else {
                        ex = false;
                        if (fr) {
                            xv = fma(alpha, dz, xv);
                            if (i == jb) st = dz < 0.0 ? -1 : 1;
                            if (st == -1) xv = lo;
                            if (st == 1) xv = hi;
                        }
                    }
                    freed = -1;
                    if (it >= maxit) inner = false;
                }
            }
        }
        // multipliers of the bound variables: w = a1 . r1 - (A0^T nu)
        const bool fr = row && st == 0;
        double qe[ME], S[TO], Tm[ME][MO], k11max;
        project(fr, qe, S, Tm, k11max);
        double rv[MO];
#pragma unroll
        for (int c = 0; c < MO; ++c) rv[c] = row ? ao[c] * xv : 0.0;
        isum_vec<NP, MO>(rv);
        double g = 0.0, wx = 0.0;
#pragma unroll
        for (int c = 0; c < MO; ++c) {
            g = fma(ao[c], bo[c] - rv[c], g);
            wx = fma(ao[c], rv[c], wx);
        }
        double qg[ME];
#pragma unroll
        for (int e = 0; e < ME; ++e) qg[e] = fr ? qe[e] * g : 0.0;
        isum_vec<NP, ME>(qg);
        double w = g;
#pragma unroll
        for (int e = 0; e < ME; ++e) w = fma(-qe[e], qg[e], w);
        out.w = row ? w : 0.0;
        const double wtol = 1e-11 * fmax(abm, imax<NP>(fmax(wtb, fabs(wx))));
        double v = -kInf;
        if (outer && row && (st == -1 || st == 1) && !ex && lo != hi) v = st < 0 ? w : -w;
        int best = i;
        iargmax<NP>(v, best);
        if (outer) {
            if (!(v > wtol)) {
                outer = false;
            } else if (it >= maxit) {
                out.capped = true;
                outer = false;
            } else {
                if (i == best) st = 0; // exclusions persist until the inner loop makes progress
                freed = best;
            }
        }
    }
    out.xv = xv;
    out.st = st;
    out.it = it;
    return out;
}

// rhs <- M^-1 rhs (lane i: row i of the NR right-hand sides) by block Gauss-Jordan on M's rows reloaded
// from HBM/L2 (the rare paths; Mb = this lane's column of its instance's M, 64-bit addressing: the
// instances of a wave come from a work list). NC = the columns held per lane: 40 when n <= 40 in 64
// lanes (the n = 39 CENTAURO size), as the fast kernel's MR -- 24 fewer columns to update and 48 fewer
// VGPRs than NP (the repair kernels' Gauss-Jordan spilled at NC = 64).
template <int NP, int NR, int NC>
__device__ __forceinline__ void minv_rows_nc(const double *Mb, int n, int i, bool row, double (&rhs)[NR], double *PN,
                                             double *RH)
{
    double A[NC];
#pragma unroll
    for (int r = 0; r < NC; ++r) A[r] = Mb[(r < n ? r : n - 1) * n];
#pragma unroll
    for (int r = 0; r < NC; ++r) A[r] = (row && r < n) ? A[r] : (r == i ? 1.0 : 0.0);
    (void)block_gj<NP, NR, NR, NC>(A, rhs, n, i, PN, RH);
}
template <int NP, int NR>
__device__ __forceinline__ void minv_rows(const double *Mb, int n, int i, bool row, double (&rhs)[NR], double *PN,
                                          double *RH)
{
    if constexpr (NP == 64) {
        if (n <= 40) {
            minv_rows_nc<NP, NR, 40>(Mb, n, i, row, rhs, PN, RH);
            return;
        }
    }
    minv_rows_nc<NP, NR, NP>(Mb, n, i, row, rhs, PN, RH);
}

struct RepairOut {
    double lo, hi, u; // (possibly pinned) limits and the new u of this lane
    double x;         // the BVLS point x* of this lane (level 0 in x-space)
    int status, it;   // status 1 if BVLS hit its cap; BVLS iterations
    int st;           // this lane's final BVLS state (-1 at lo, +1 at hi, 0 free or padding)
    bool l0inf;       // y* != b0: level 0 really is infeasible at b0 (warm-start hint)
    bool unique;      // the level-1 feasible set is the single point x*: level 1 has nothing left
};

// Level-0 repair for the instances with rep set (every lane of the wave calls this; the
// instance -> lane mapping is the kernel's). Level 0 in x-space is
//   min 0.5 ||A0 x - b0||^2  s.t. lo <= x <= hi,   A0 = G M^-1   (QPPVMPlugin.cpp:129-152,177)
// Solved by BVLS (Stark-Parker), the algorithm of oracle/wbq_oracle.c:wbq_ref_level0, with
// lane i owning column a_i = (M^-1 G^T)_i (block Gauss-Jordan on the M rows, reloaded from
// HBM/L2: this path is rare). Then y* = A0 x*, every variable the level-0 gradient
// w = A0^T (b0 - y*) holds at a bound is pinned there (lo = hi, as wbq_ref_qppvm_one does),
// and u is reset to the least-distance point of G u = y*, with the Q1 rows (orthonormal
// basis of range(G^T), zero rows past its rank) in LDS for a fresh dual active set.
// Not inlined: its registers do not weigh on the active-set loop.
template <int NP, int M0>
__device__ __forceinline__ RepairOut level0_repair(const QppvmArgs &a, int soff, long b, int i, bool rep, double lo,
                                                double hi, bool warm)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double *S = smem + soff;
    constexpr int RS = NP + 1;
    constexpr int NT = M0 * (M0 + 1) / 2;
    const ActiveLayout<NP> L(a.ntasks, a.m0);
    const int n = a.n, m0 = a.m0;
    const int ic = i < n ? i : n - 1;
    const bool row = rep && i < n;
    RepairOut out{lo, hi, 0.0, 0.0, 0, 0, 0, false, false};
    double gcol[M0], acol[M0], b0v[M0];
    const double uimp = rep ? a.ui_scr[b * NP + i] : 0.0;
#pragma unroll
    for (int c = 0; c < M0; ++c) {
        const bool on = rep && c < m0;
        const int rr = on ? a.row_sel[c] : 0;
        gcol[c] = (on && row) ? a.J[(b * a.ntasks * 6 + rr) * n + ic] : 0.0;
        b0v[c] = on ? a.b0_scr[b * kM0Max + c] : 0.0;
        acol[c] = gcol[c];
    }
    // a_i = row i of M^-1 G^T: Gauss-Jordan on the M rows (QA region as scratch; the Q1 rows
    // are rebuilt below)
    __syncthreads();
    minv_rows<NP, M0>(a.M + b * n * n + ic, n, i, row, acol, S + L.QA, S + L.QA + 2 * kGjBS * NP);
    WBQ_STAMP(9);
    // ---- BVLS (oracle/wbq_oracle.c:wbq_ref_level0); warm start (any state is valid): the bound
    // SET of the last repair, each variable on the side the level-0 gradient at that corner
    // points to now. Under saturation a 1 kHz loop's torques can swap sides between ticks
    // (a chattering plant): the last sides then cost one BVLS step per variable, this start
    // a few (scripts/diag_plugin_tick.py, the config-0 stress plant: 42 -> 7 steps).
    int st0 = 0;
    {
        const int w = (row && warm) ? a.ws_state[b * NP + i] : 0;
        const double xs = w < 0 ? lo : (w > 0 ? hi : (row ? fmin(fmax(0.0, lo), hi) : 0.0));
        double rs0[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) rs0[c] = acol[c] * xs;
        isum_vec<NP, M0>(rs0);
        double g = 0.0;
#pragma unroll
        for (int c = 0; c < M0; ++c) g = fma(acol[c], b0v[c] - rs0[c], g);
        // two candidate corners: the last sides kept, or every warm variable on the side the gradient at that
        // corner points to; the start is the one with the smaller level-0 residual. Flipping is what a chattering
        // plant needs (config 0 stress: the saturated torques swap sides every tick; kept sides there: p50 143 ->
        // 484 us), keeping what an MPC rollout needs (its bound set drifts; flipped there: up to 86 BVLS steps
        // against 34, config 4 18.6 vs 23.1 M QP/s; scripts/gpu_r04_p.sh)
        const int sf = w != 0 ? (g > 0.0 ? 1 : -1) : 0;
        const double xf = sf < 0 ? lo : (sf > 0 ? hi : xs);
        double rs1[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) rs1[c] = acol[c] * xf;
        isum_vec<NP, M0>(rs1);
        double rk = 0.0, rf = 0.0;
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            rk = fma(b0v[c] - rs0[c], b0v[c] - rs0[c], rk);
            rf = fma(b0v[c] - rs1[c], b0v[c] - rs1[c], rf);
        }
        if (w != 0) st0 = rf < rk ? sf : (w < 0 ? -1 : 1);
    }
    double abm = 0.0;
#pragma unroll
    for (int c = 0; c < M0; ++c) abm = fma(acol[c], b0v[c], abm);
    abm = fmax(1.0, imax<NP>(fabs(abm)));
    const double pintol = 1e-9 * abm;
    // level-0 rows: all m0 of them, or the first a.m_l0 when a middle level follows (task_level)
    const int ml = (M0 > 6 && a.m_l0 > 0 && a.m_l0 < m0) ? a.m_l0 : m0;
    double acol0[M0], b0v0[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) {
        acol0[c] = c < ml ? acol[c] : 0.0;
        b0v0[c] = c < ml ? b0v[c] : 0.0;
    }
    BvlsOut bv;
    if (M0 > 6 && ml <= 6) { // (a middle level: level 0 has at most 6 rows, the 6-row BVLS suffices)
        double a6[6], b6[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            a6[c] = acol0[c < M0 ? c : 0];
            b6[c] = b0v0[c < M0 ? c : 0];
        }
        bv = bvls<NP, 6>(a6, b6, ml, lo, hi, row, rep, st0, 50 * n + 100);
    } else {
        bv = bvls<NP, M0>(acol0, b0v0, ml, lo, hi, row, rep, st0, 50 * n + 100, S + L.QA);
    }
#ifdef WBQ_STAMPS
    if (threadIdx.x == 0 && a.stamps)
        for (int k = 0; k < 8; ++k) a.stamps[blockIdx.x * kStamps + 20 + k] = bv.ph[k];
#endif
    double xv = bv.xv;
    int st = bv.st, it = bv.it;
    if (bv.capped) out.status = 1;
    WBQ_STAMP(10);
    // ---- y* = A0 x*, pins, and the least-distance point of G u = y*
    if (row) a.ws_state[b * NP + i] = (signed char)(st == 2 ? 0 : st);
    double ys[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) ys[c] = acol[c] * xv;
    isum_vec<NP, M0>(ys);
    if constexpr (M0 > 6) {
        if (ml < m0) {
            // the middle level (the elbow tasks, QPPVMPlugin.cpp:154-166,177-178): level-0 pins first,
            // then min ||A1 x - b1|| keeping A0 x = y0* (bvls_eq), its own pins, and y1* = A1 x1*
            double l0w = 0.0;
#pragma unroll
            for (int c = 0; c < M0; ++c) l0w = fma(acol0[c], b0v0[c] - ys[c], l0w);
            double lo1 = lo, hi1 = hi;
            if (row && l0w > pintol) lo1 = hi;
            else if (row && l0w < -pintol) hi1 = lo;
            double ae[6], ao[6], bo[6];
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                ae[c] = c < ml ? acol[c] : 0.0;
                double v = 0.0, bb = 0.0;
#pragma unroll
                for (int r = 0; r < M0; ++r) {
                    v = (r == ml + c) ? acol[r] : v;
                    bb = (r == ml + c) ? b0v[r] : bb;
                }
                ao[c] = (ml + c < m0) ? v : 0.0;
                bo[c] = (ml + c < m0) ? bb : 0.0;
            }
            double abm1 = 0.0;
#pragma unroll
            for (int c = 0; c < 6; ++c) abm1 = fma(ao[c], bo[c], abm1);
            abm1 = fmax(1.0, imax<NP>(row ? fabs(abm1) : 0.0));
            const BvlsEqOut be = bvls_eq<NP, 6, 6>(ae, ml, ao, bo, m0 - ml, lo1, hi1, row, rep, xv, st, 50 * n + 100);
            xv = be.xv;
            st = be.st;
            it += be.it;
            if (be.capped) out.status = 1;
            // the variables the middle level's multipliers hold at a bound (level-0 pins stay)
            if (row && lo1 != hi1 && be.st == -1 && be.w < -1e-9 * abm1) hi1 = lo1;
            if (row && lo1 != hi1 && be.st == 1 && be.w > 1e-9 * abm1) lo1 = hi1;
            lo = lo1;
            hi = hi1;
            double y1[M0];
#pragma unroll
            for (int c = 0; c < M0; ++c) y1[c] = acol[c] * xv;
            isum_vec<NP, M0>(y1);
#pragma unroll
            for (int c = 0; c < M0; ++c) ys[c] = c < ml ? ys[c] : y1[c];
        }
    }
    {
        double gap = 0.0, bmx = 1.0;
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            gap = fmax(gap, fabs(ys[c] - b0v[c]));
            bmx = fmax(bmx, fabs(b0v[c]));
        }
        out.l0inf = rep && gap > 1e-9 * bmx;
    }
    if (row) {
        double w = 0.0;
#pragma unroll
        for (int c = 0; c < M0; ++c) w = fma(acol0[c], b0v0[c] - ys[c], w);
        out.lo = lo; // (with a middle level: its pins and level 0's already in lo / hi)
        out.hi = hi;
        if (w > pintol) out.lo = out.hi;       // pinned at the upper bound
        else if (w < -pintol) out.hi = out.lo; // pinned at the lower bound
    }
    out.x = row ? xv : 0.0;
    out.st = (row && (st == -1 || st == 1)) ? st : 0;
    // Level 1 keeps A0 x = y* and the (pinned) box. When the columns of A0 over the variables
    // left free are independent, x_F is fixed by A0_F x_F = y* - A0_P x_P: the feasible set is
    // the single point x* and the level-1 objective cannot move it (the generic saturated case:
    // the free columns span one facet of the zonotope A0 * box). The rank test is conservative
    // (pivots above 1e-8 of the largest): a nearly dependent free set goes to the active set.
    {
        const bool fl = row && out.lo != out.hi;
        double gf[NT];
#pragma unroll
        for (int p = 0; p < M0; ++p)
#pragma unroll
            for (int c = 0; c <= p; ++c) gf[tri(p, c)] = fl ? acol[p] * acol[c] : 0.0;
        isum_vec<NP, NT>(gf);
        const double kf = isum<NP>(fl ? 1.0 : 0.0);
        PivChol<M0> pf;
        pf.factor(gf, m0, 1e-8);
        out.unique = rep && !bv.capped && (double)pf.k == kf;
    }
    double gg[NT], rr[M0];
#pragma unroll
    for (int p = 0; p < M0; ++p) {
        rr[p] = gcol[p] * uimp;
#pragma unroll
        for (int c = 0; c <= p; ++c) gg[tri(p, c)] = gcol[p] * gcol[c];
    }
    isum_vec<NP, M0>(rr);
    isum_vec<NP, NT>(gg);
#pragma unroll
    for (int c = 0; c < M0; ++c) rr[c] = ys[c] - rr[c]; // y* - G u_imp (consistent)
    double q1[M0], cv[M0];
    {
        PivChol<M0> pc;
        pc.factor(gg, m0, 1e-12);
        pc.solve(rr, m0, cv);
        pc.basis(gcol, q1);
    }
    double un = uimp;
#pragma unroll
    for (int c = 0; c < M0; ++c) un = fma(gcol[c], cv[c], un);
    out.u = rep ? un : 0.0;
    __syncthreads(); // Gauss-Jordan scratch in QA is dead
    if (rep) {
#pragma unroll
        for (int c = 0; c < NP; ++c) S[L.QA + c * RS + i] = (c < M0 && c < m0) ? q1[c < M0 ? c : 0] : 0.0;
    }
    out.it = rep ? it : 0;
    return out;
}

// Work lists: the producing kernel appends every instance that needs a follow-up kernel
// (atomic counter work[epoch*2 + 0] / [+1], lists wl[0..B) / wl[B..2B)), and the follow-up
// kernels run a small grid-stride grid over the list. Without work a launch is one
// broadcast load per block of at most kFollowGrid blocks, instead of a batch-sized grid.
__device__ __forceinline__ void wl_push(const QppvmArgs &a, int list, long b)
{
    const int idx = atomicAdd(&a.work[list < 2 ? a.epoch * 2 + list : 4 + a.epoch], 1);
    a.wl[(long)list * a.B + idx] = (int)b;
    // (the host's completion check of an on-demand solve: some instance waits for the repair kernel)
    if (list == 1 && a.self_book && a.fg.seen)
        __hip_atomic_store(a.fg.seen + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Follow-up grid cap: 2 waves per SIMD over the whole chip (launch cost measured independent of
// the grid size, scripts/launch_probe.hip; a smaller cap starves a solve where many instances
// need the repair, e.g. diverging MPC rollouts)
constexpr unsigned kFollowGrid = 2048;

}  // namespace wbq
