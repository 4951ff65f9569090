// qppvm_kernel.hip -- fused batched QPPVM torque solve for gfx950 (MI355X), fp64.
//
// One QP instance per group of NP lanes (NP = 32: two instances per wave64; NP = 64: one),
// lane i <-> joint i. A launch covers assemble -> 2-level hierarchical QP -> tau for
// the whole batch; nothing goes back to the host in between.
//
// The math (reference src/QPPVMPlugin.cpp:201-259):
//   level 0  min 0.5 sum_t ||S_t J_t M^-1 x - S_t J_t M^-1 J_t^T F_t||^2      (:129-152, :177)
//   level 1  min 0.5 ||M^-1 x - M^-1 tau_imp||^2  s.t. level-0 optimality     (:114-118)
//   both     tau_min - h <= x <= tau_max - h                                  (:56-67, :203-205)
//   tau = x + h, and tau = h on failure                                        (:246-256)
// is solved in the transformed variable u = M^-1 x, where level 1 becomes the
// least-distance problem
//   min 0.5 ||u - u_imp||^2  s.t.  G u = b0,  lo <= M u <= hi
// with G = stacked selected rows of J (given data) and u_imp = M^-1 tau_imp. The Hessian
// is the identity, so the Goldfarb-Idnani dual active set needs no factorisation of H,
// the bound normals are rows of M (given data), and the conditioning is cond(M), not
// cond(M)^2 as in the reference's x-space H1 = M^-2. When level 0 is feasible
// (y* = b0, the generic case) the level-0 optimality constraint A0 x = y* is exactly
// G u = b0; an infeasible level 0 is reported as status 2 by this kernel.
//
// Per instance:
//   1. stage J rows / poses / q, qd in LDS, task-space force F_t = Kc e - Dc J qd;
//   2. Gauss-Jordan on [M | tau_imp, J_t^T F_t] in registers (M SPD: no pivoting; the
//      trailing block stays symmetric, so the pivot row is read back from the pivot
//      column every lane just published) -> u_imp, w_t = M^-1 J_t^T F_t;
//   3. b0 = G w, Cholesky-QR of G^T (rank-revealing) -> Q1, u_eq = u_imp + Q1 R^-T (b0 - G u_imp);
//   4. GI iterations on the bound rows of M: d1 = Q1^T n_p, z = (I - Q1 Q1^T) n_p (twice,
//      CGS2), r = R_II^-1 d1_I kept through T = R_II^-1, primal/dual steps, add/drop;
//   5. tau = M u + h.
#include "wbq_kernels.h"

#include <math.h>

namespace wbq {
namespace {

constexpr double kInf = 1.0e300;

// Per-instance LDS layout in doubles (T = ntasks is a launch constant).
// Rows of NP-wide matrices use stride NP+1 so that lane-per-row reads are bank-conflict free.
template <int NP>
struct Layout {
    static constexpr bool MREG = (NP == 32); // M rows in VGPRs (else in LDS)
    static constexpr int RS = NP + 1;        // row stride
    int MA, QA, TT, JR, BC, RH, U, D1, D1B, NV, WV, QD, F, B0, RES, RHO, GR, LC, PS, SIZE;
    __host__ __device__ Layout(int T)
    {
        MA = 0;                                     // staged M rows
        QA = MREG ? MA : MA + NP * RS;              // Q1^T rows (reuses MA once M is in VGPRs)
        TT = QA + NP * RS;                          // T = R_II^-1 rows (NP == 64 only)
        JR = TT + (NP == 64 ? NP * RS : 0);         // J rows [T*6][NP]
        BC = JR + T * 6 * NP;                       // GJ pivot column, double-buffered [2][NP]
        RH = BC + 2 * NP;                           // GJ pivot right-hand sides [2][8]
        U = RH + 16;                                // u
        D1 = U + NP;                                // d1 = Q1^T n_p, zero-padded to 2 NP
        D1B = D1 + 2 * NP;                          // second Gram-Schmidt pass
        NV = D1B + NP;                              // n_p
        WV = NV + NP;                               // w_t [T][NP]
        QD = WV + T * NP;                           // qdot
        F = QD + NP;                                // task forces [T*6]
        B0 = F + 6 * T;                             // b0 [kM0Max]
        RES = B0 + kM0Max;                          // b0 - G u_imp
        RHO = RES + kM0Max;                         // L^-1 (b0 - G u_imp)
        GR = RHO + kM0Max;                          // Gram, then its Cholesky factor L
        LC = GR + kM0Max * kM0Max;                  // broadcast column of L
        PS = LC + kM0Max;                           // poses [T][24]
        SIZE = (PS + 24 * T + 1) & ~1;              // keep 16-B alignment of the next instance
    }
};

// One row of an NP-column matrix per lane: in VGPRs (compile-time indices, runtime
// writes by select) or in LDS.
template <int NP, bool REG>
struct RowStore;

template <int NP>
struct RowStore<NP, true> {
    double v[NP];
    __device__ void bind(double *) {}
    __device__ void zero()
    {
#pragma unroll
        for (int j = 0; j < NP; ++j) v[j] = 0.0;
    }
    __device__ void set(int c, double x)
    {
#pragma unroll
        for (int j = 0; j < NP; ++j) v[j] = (j == c) ? x : v[j];
    }
    __device__ double get(int c) const
    {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j) r = (j == c) ? v[j] : r;
        return r;
    }
    __device__ double dot(const double *b, int cnt) const
    {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j)
            if (j < cnt) s = fma(v[j], b[j], s);
        return s;
    }
};

template <int NP>
struct RowStore<NP, false> {
    double *row;
    __device__ void bind(double *p) { row = p; }
    __device__ void zero()
    {
        for (int j = 0; j < NP; ++j) row[j] = 0.0;
    }
    __device__ void set(int c, double x) { row[c] = x; }
    __device__ double get(int c) const { return row[c]; }
    __device__ double dot(const double *b, int cnt) const
    {
        double s = 0.0;
        for (int j = 0; j < cnt; ++j) s = fma(row[j], b[j], s);
        return s;
    }
};

template <int NP>
__device__ __forceinline__ double isum(double v)
{
#pragma unroll
    for (int m = NP / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, NP);
    return v;
}

template <int NP>
__device__ __forceinline__ double imax(double v)
{
#pragma unroll
    for (int m = NP / 2; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, NP));
    return v;
}

// (value, index) reductions inside an instance; ties -> lowest index
template <int NP>
__device__ __forceinline__ void iargmax(double &v, int &idx)
{
#pragma unroll
    for (int m = NP / 2; m >= 1; m >>= 1) {
        const double ov = __shfl_xor(v, m, NP);
        const int oi = __shfl_xor(idx, m, NP);
        if (ov > v || (ov == v && oi < idx)) {
            v = ov;
            idx = oi;
        }
    }
}

template <int NP>
__device__ __forceinline__ void iargmin(double &v, int &idx)
{
#pragma unroll
    for (int m = NP / 2; m >= 1; m >>= 1) {
        const double ov = __shfl_xor(v, m, NP);
        const int oi = __shfl_xor(idx, m, NP);
        if (ov < v || (ov == v && oi < idx)) {
            v = ov;
            idx = oi;
        }
    }
}

// Cartesian error component r of e = [p_ref - p ; vec(quat(R_ref R^T)), w >= 0]
// (same specification as oracle/wbq_oracle.c:wbq_ref_cart_error).
__device__ double cart_error_component(const double *P, const double *Pr, int r)
{
    if (r < 3) return Pr[4 * r + 3] - P[4 * r + 3];
    double Re[9];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            Re[3 * a + c] = Pr[4 * a] * P[4 * c] + Pr[4 * a + 1] * P[4 * c + 1] + Pr[4 * a + 2] * P[4 * c + 2];
    const double tr = Re[0] + Re[4] + Re[8];
    double qw, qx, qy, qz;
    if (tr > 0.0) {
        const double s = sqrt(tr + 1.0) * 2.0;
        qw = 0.25 * s;
        qx = (Re[7] - Re[5]) / s;
        qy = (Re[2] - Re[6]) / s;
        qz = (Re[3] - Re[1]) / s;
    } else if (Re[0] > Re[4] && Re[0] > Re[8]) {
        const double s = sqrt(1.0 + Re[0] - Re[4] - Re[8]) * 2.0;
        qw = (Re[7] - Re[5]) / s;
        qx = 0.25 * s;
        qy = (Re[1] + Re[3]) / s;
        qz = (Re[2] + Re[6]) / s;
    } else if (Re[4] > Re[8]) {
        const double s = sqrt(1.0 + Re[4] - Re[0] - Re[8]) * 2.0;
        qw = (Re[2] - Re[6]) / s;
        qx = (Re[1] + Re[3]) / s;
        qy = 0.25 * s;
        qz = (Re[5] + Re[7]) / s;
    } else {
        const double s = sqrt(1.0 + Re[8] - Re[0] - Re[4]) * 2.0;
        qw = (Re[3] - Re[1]) / s;
        qx = (Re[2] + Re[6]) / s;
        qy = (Re[5] + Re[7]) / s;
        qz = 0.25 * s;
    }
    const double sg = (qw < 0.0) ? -1.0 : 1.0;
    return sg * (r == 3 ? qx : (r == 4 ? qy : qz));
}

template <int NP>
__device__ __forceinline__ void load_row(RowStore<NP, true> &R, const double *Mb, int n, int i, bool row)
{
#pragma unroll
    for (int j = 0; j < NP; ++j) R.v[j] = (row && j < n) ? Mb[i * n + j] : (j == i ? 1.0 : 0.0);
}

// Orthogonalise the normal held in NV against the rows of Q1T (two classical Gram-Schmidt
// passes). Rows >= q of Q1T are finite and D1[c >= q] = 0, so every loop runs to NP
// unguarded. Leaves d1 = Q1^T n in D1 and returns this lane's entry of z.
template <int NP>
__device__ __forceinline__ double project_out(double *S, const Layout<NP> &L, double npj, int q, int i)
{
    constexpr int RS = NP + 1;
    double d1 = 0.0;
    if (i < q) {
#pragma unroll
        for (int j = 0; j < NP; ++j) d1 = fma(S[L.QA + i * RS + j], S[L.NV + j], d1);
    }
    S[L.D1 + i] = d1;
    __syncthreads();
    double z = npj;
#pragma unroll
    for (int c = 0; c < NP; ++c) z = fma(-S[L.QA + c * RS + i], S[L.D1 + c], z);
    S[L.BC + i] = z;
    __syncthreads();
    double d1b = 0.0;
    if (i < q) {
#pragma unroll
        for (int j = 0; j < NP; ++j) d1b = fma(S[L.QA + i * RS + j], S[L.BC + j], d1b);
    }
    S[L.D1B + i] = d1b;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NP; ++c) z = fma(-S[L.QA + c * RS + i], S[L.D1B + c], z);
    S[L.D1 + i] = d1 + d1b;
    __syncthreads();
    return z;
}

template <int NP>
__global__ __launch_bounds__(64) void qppvm_solve_kernel(const QppvmArgs a)
{
    constexpr int IPW = kWave / NP;
    constexpr int RS = NP + 1;
    constexpr bool MREG = Layout<NP>::MREG;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int T = a.ntasks, n = a.n, m0 = a.m0;
    const Layout<NP> L(T);
    const int tid = threadIdx.x;
    const int sub = tid / NP;
    const int i = tid - sub * NP;
    const long b = (long)blockIdx.x * IPW + sub;
    const bool valid = b < a.B;
    double *S = smem + sub * L.SIZE;
    const bool row = valid && i < n;
    const long bn = valid ? b * n : 0;

    // ---------------------------------------------------------------- 1. stage
    const double q_i = row ? a.q[bn + i] : 0.0;
    const double qd_i = row ? a.qd[bn + i] : 0.0;
    const double qref_i = row ? a.qref[bn + i] : 0.0;
    const double h_i = row ? a.h[bn + i] : 0.0;
    S[L.QD + i] = qd_i;
    const double *Mb = a.M + (valid ? b * n * n : 0);
    {
        // M row by row: every load instruction reads whole contiguous rows (coalesced)
#pragma unroll
        for (int r = 0; r < NP; ++r)
            if (r < n) S[L.MA + r * RS + i] = row ? Mb[r * n + i] : 0.0;
        const double *Jb = a.J + (valid ? b * T * 6 * n : 0);
        for (int rr = 0; rr < T * 6; ++rr) S[L.JR + rr * NP + i] = row ? Jb[rr * n + i] : 0.0;
        for (int e = i; e < T * 24; e += NP) {
            const int t = e / 24, c = e - t * 24;
            double v = 0.0;
            if (valid)
                v = (c < 12) ? a.pose[(b * T + t) * 12 + c] : a.pose_ref[(b * T + t) * 12 + c - 12];
            S[L.PS + e] = v;
        }
        S[L.D1 + NP + i] = 0.0; // zero pad of d1
    }
    __syncthreads();
    // task-space force per task row (spring + damper, zero desired twist), QPPVMPlugin.cpp:136-137
    if (i < T * 6) {
        const int t = i / 6, r = i - t * 6;
        double xd = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j) xd = fma(S[L.JR + i * NP + j], S[L.QD + j], xd);
        const double er = cart_error_component(S + L.PS + t * 24, S + L.PS + t * 24 + 12, r);
        double F = a.Kc[i] * er - a.Dc[i] * xd;
        if (a.select_mode == 1 && !((a.row_mask[t] >> r) & 1)) F = 0.0;
        S[L.F + i] = F;
    }
    // rows of M into VGPRs (A for the elimination, Mr kept for the bound rows)
    double A[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) A[j] = (row && j < n) ? S[L.MA + i * RS + j] : (j == i ? 1.0 : 0.0);
    RowStore<NP, MREG> Mr;
    Mr.bind(S + L.MA + i * RS);
    if constexpr (MREG) {
#pragma unroll
        for (int j = 0; j < NP; ++j) Mr.v[j] = A[j];
    } else {
        // pad rows/columns of the LDS copy as identity
        for (int j = 0; j < NP; ++j)
            if (!(row && j < n)) S[L.MA + i * RS + j] = (j == i ? 1.0 : 0.0);
    }
    __syncthreads();

    // ------------------------------------------------- 2. Gauss-Jordan, M SPD
    double rhs[1 + kTMax];
    rhs[0] = row ? a.Kq[i] * (qref_i - q_i) - a.Dq[i] * qd_i : 0.0; // tau_imp (:105-106)
#pragma unroll
    for (int t = 0; t < kTMax; ++t) {
        double c = 0.0;
        if (t < T)
#pragma unroll
            for (int r = 0; r < 6; ++r) c = fma(S[L.JR + (t * 6 + r) * NP + i], S[L.F + t * 6 + r], c);
        rhs[1 + t] = c; // J_t^T F_t
    }
    double dval = 1.0;
    bool notspd = false;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        if (k < n) {
            double *bc = S + L.BC + (k & 1) * NP;
            double *rh = S + L.RH + (k & 1) * 8;
            bc[i] = A[k];
            if (i == k) {
#pragma unroll
                for (int m = 0; m < 1 + kTMax; ++m) rh[m] = rhs[m];
            }
            __syncthreads();
            const double piv = bc[k];
            notspd |= !(piv > 0.0);
            const double f = (i == k) ? 0.0 : A[k] / piv;
#pragma unroll
            for (int j = k + 1; j < NP; ++j) A[j] = fma(-f, bc[j], A[j]);
#pragma unroll
            for (int m = 0; m < 1 + kTMax; ++m) rhs[m] = fma(-f, rh[m], rhs[m]);
            dval = (i == k) ? piv : dval;
        }
    }
    const double u_imp = rhs[0] / dval;
    S[L.U + i] = u_imp;
#pragma unroll
    for (int t = 0; t < kTMax; ++t)
        if (t < T) S[L.WV + t * NP + i] = rhs[1 + t] / dval; // w_t = M^-1 J_t^T F_t
    __syncthreads();

    // ---------------------------------- 3. level-0 rows and the equality block
    if (i < m0) {
        const int rr = a.row_sel[i], t = rr / 6;
        double bb = 0.0, gu = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const double g = S[L.JR + rr * NP + j];
            bb = fma(g, S[L.WV + t * NP + j], bb);
            gu = fma(g, S[L.U + j], gu);
        }
        S[L.B0 + i] = bb;           // b0 = S J M^-1 J^T F
        S[L.RES + i] = bb - gu;
    }
    {
        const int npairs = m0 * (m0 + 1) / 2;
        for (int pp = i; pp < npairs; pp += NP) {
            int ra = 0;
            while ((ra + 1) * (ra + 2) / 2 <= pp) ++ra;
            const int ca = pp - ra * (ra + 1) / 2;
            const int r1 = a.row_sel[ra], r2 = a.row_sel[ca];
            double g = 0.0;
#pragma unroll
            for (int j = 0; j < NP; ++j) g = fma(S[L.JR + r1 * NP + j], S[L.JR + r2 * NP + j], g);
            S[L.GR + ra * kM0Max + ca] = g;
        }
    }
    __syncthreads();
    {
        // lane-parallel rank-revealing Cholesky G G^T = L L^T (lane r owns row r), fused with
        // the forward substitution rho = L^-1 (b0 - G u_imp); dependent rows get a zero column
        double g[kM0Max];
#pragma unroll
        for (int c = 0; c < kM0Max; ++c) {
            const int hi_ = i > c ? i : c, lo_ = i > c ? c : i;
            g[c] = (i < m0 && c < m0) ? S[L.GR + hi_ * kM0Max + lo_] : 0.0;
        }
        double res = i < m0 ? S[L.RES + i] : 0.0;
        double gdiag = 0.0;
#pragma unroll
        for (int c = 0; c < kM0Max; ++c) gdiag = (c == i) ? g[c] : gdiag;
        const double dmx = imax<NP>(gdiag);
        __syncthreads();
#pragma unroll
        for (int c = 0; c < kM0Max; ++c) {
            if (c < m0) {
                const double dc = __shfl(g[c], c, NP);
                const bool indep = dc > 1e-12 * dmx;
                const double Lcc = indep ? sqrt(dc) : 0.0;
                const double lrc = (i > c && indep) ? g[c] / Lcc : (i == c ? Lcc : 0.0);
                const double rc = __shfl(res, c, NP);
                const double rho_c = indep ? rc / Lcc : 0.0;
                if (i > c) res = fma(-lrc, rho_c, res);
                if (i == c) S[L.RHO + c] = rho_c;
                if (i < m0) {
                    S[L.LC + i] = lrc;
                    S[L.GR + i * kM0Max + c] = lrc;
                }
                __syncthreads();
#pragma unroll
                for (int j = c + 1; j < kM0Max; ++j) g[j] = fma(-lrc, S[L.LC + j], g[j]);
                __syncthreads();
            }
        }
    }
    // Q1 = G^T L^-T (row i of Q1 by forward substitution), u_eq = u_imp + Q1 rho
    double q1[kM0Max];
    double u_i = u_imp;
#pragma unroll
    for (int c = 0; c < kM0Max; ++c) {
        double v = 0.0;
        if (c < m0) {
            v = S[L.JR + a.row_sel[c] * NP + i];
#pragma unroll
            for (int k = 0; k < c; ++k) v = fma(-S[L.GR + c * kM0Max + k], q1[k], v);
            const double d = S[L.GR + c * kM0Max + c];
            v = d > 0.0 ? v / d : 0.0;
            u_i = fma(v, S[L.RHO + c], u_i);
        }
        q1[c] = v;
    }
    S[L.U + i] = u_i;
    __syncthreads();
    // residual of every level-0 row (catches rows dropped as dependent: level 0 infeasible)
    double eqres = 0.0;
    if (i < m0) {
        const int rr = a.row_sel[i];
        double gu = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j) gu = fma(S[L.JR + rr * NP + j], S[L.U + j], gu);
        const double bb = S[L.B0 + i];
        eqres = fabs(gu - bb) / fmax(1.0, fabs(bb));
    }
    eqres = imax<NP>(eqres);
    // Q1^T rows: the m0 equality directions, zero beyond
#pragma unroll
    for (int c = 0; c < NP; ++c) S[L.QA + c * RS + i] = (c < kM0Max && c < m0) ? q1[c < kM0Max ? c : 0] : 0.0;
    __syncthreads();

    // ------------------------------ 4. Goldfarb-Idnani on the torque bounds
    double nrm2 = 0.0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const double mij = Mr.get(j);
        nrm2 = fma(mij, mij, nrm2);
    }
    const double nrm = sqrt(nrm2);
    const double lo = row ? a.tau_min[i] - h_i : -kInf;
    const double hi = row ? a.tau_max[i] - h_i : kInf;
    RowStore<NP, NP == 32> Tr;
    Tr.bind(S + L.TT + i * RS);
    Tr.zero();

    int status = 0;
    if (imax<NP>((row && lo > hi) ? 1.0 : 0.0) > 0.0) status = 2; // crossed limits
    if (notspd) status = 3;
    if (status == 0 && eqres > 1e-9) status = 2; // level 0 infeasible (not handled here)
    bool go = valid && status == 0;
    int k = 0, q = m0, iters = 0;
    int act_p = -1, act_s = 0; // lane a < k: active inequality a (row index, sign)
    double lam = 0.0;          // lane a < k: its multiplier
    int p = 0, sg = 1;
    double lamp = 0.0;
    bool need_select = true;
    const int maxit = a.max_iter;

    while (__any(go)) {
        const double s_i = Mr.dot(S + L.U, NP); // s = M u = x
        if (need_select) {
            double v = -1.0;
            if (row) {
                const double tol = 1e-10 * fmax(1.0, fmax(fabs(s_i), fmax(fabs(lo), fabs(hi))));
                const double viol = fmax(lo - s_i, s_i - hi);
                if (viol > tol) v = viol / nrm;
            }
            int pi = i;
            iargmax<NP>(v, pi);
            if (!(v > 0.0)) go = false; // optimal
            p = pi;
            sg = (__shfl(lo - s_i, p, NP) > __shfl(s_i - hi, p, NP)) ? 1 : -1;
            lamp = 0.0;
        }
        const double s_p = __shfl(s_i, p, NP);
        const double sp = sg > 0 ? s_p - __shfl(lo, p, NP) : __shfl(hi, p, NP) - s_p; // slack < 0
        const double npn = __shfl(nrm, p, NP);
        const double npj = sg * Mr.get(p); // n_p = sg * M row p (M symmetric)
        S[L.NV + i] = npj;
        __syncthreads();
        const double z = project_out<NP>(S, L, npj, q, i);
        const double zz = isum<NP>(z * z);
        double ra = 0.0;
        if (i < k) ra = Tr.dot(S + L.D1 + m0, NP);
        const double rmax = imax<NP>(fabs(ra));
        double cand = (i < k && ra > 1e-13 * rmax) ? lam / ra : kInf;
        int ci = i;
        iargmin<NP>(cand, ci);
        const double t1 = cand;
        const double t2 = (zz > 1e-20 * npn * npn) ? -sp / zz : kInf;
        bool rebuild = false;
        int cdrop = 0;
        if (go && t1 >= kInf && t2 >= kInf) {
            status = 2; // infeasible
            go = false;
        }
        if (go) {
            const double t = fmin(t1, t2);
            if (i < k) lam = fma(-t, ra, lam);
            lamp += t;
            if (t2 < kInf) u_i = fma(t, z, u_i);
            ++iters;
            if (t2 <= t1) { // add p
                const double iz = 1.0 / sqrt(zz);
                S[L.QA + q * RS + i] = z * iz;
                if (i < k) Tr.set(k, -ra * iz);
                if (i == k) {
                    Tr.zero();
                    Tr.set(k, iz);
                    act_p = p;
                    act_s = sg;
                    lam = lamp;
                }
                ++k;
                ++q;
                need_select = true;
            } else { // drop ci (its multiplier hit zero), keep p
                const int nap = __shfl(act_p, i + 1, NP);
                const int nas = __shfl(act_s, i + 1, NP);
                const double nlam = __shfl(lam, i + 1, NP);
                if (i >= ci) {
                    act_p = nap;
                    act_s = nas;
                    lam = nlam;
                }
                --k;
                cdrop = ci;
                q = m0 + ci;
                rebuild = true;
                need_select = false;
            }
            if (iters >= maxit && go) {
                status = 1;
                go = false;
            }
        }
        S[L.U + i] = u_i;
        __syncthreads();
        if (__any(rebuild)) {
            // Re-factor the inequality directions from the dropped position on: Q1T rows
            // m0+cdrop.. and T columns cdrop.. (Gram-Schmidt is sequential, earlier ones stand).
            if (rebuild && i < NP) {
#pragma unroll
                for (int j = 0; j < NP; ++j)
                    if (j >= cdrop) Tr.set(j, 0.0);
            }
            const int kk = rebuild ? k : 0;
            int kmax = kk, amin = rebuild ? cdrop : NP;
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) {
                kmax = max(kmax, __shfl_xor(kmax, m, 64));
                amin = min(amin, __shfl_xor(amin, m, 64));
            }
            for (int a2 = amin; a2 < kmax; ++a2) {
                const bool on = rebuild && a2 >= cdrop && a2 < kk;
                const int pa = __shfl(act_p, a2, NP), sa = __shfl(act_s, a2, NP);
                const double nj = on ? sa * Mr.get(pa) : 0.0;
                S[L.NV + i] = nj;
                __syncthreads();
                const double zr = project_out<NP>(S, L, nj, on ? q : 0, i);
                const double zzr = isum<NP>(zr * zr);
                double rr2 = 0.0;
                if (on && i < a2) rr2 = Tr.dot(S + L.D1 + m0, NP);
                if (on) {
                    const double iz = 1.0 / sqrt(zzr);
                    S[L.QA + q * RS + i] = zr * iz;
                    if (i < a2) Tr.set(a2, -rr2 * iz);
                    if (i == a2) Tr.set(a2, iz);
                    ++q;
                }
                __syncthreads();
            }
        }
    }

    // ------------------------------------------------------------ 5. output
    const double x_i = Mr.dot(S + L.U, NP);
    double tau_i = x_i + h_i;
    if (imax<NP>((row && !isfinite(tau_i)) ? 1.0 : 0.0) > 0.0 && status == 0) status = 3;
    if (status != 0) tau_i = h_i; // "SOLVER ERROR!" fallback: tau_qp = 0 (QPPVMPlugin.cpp:246-249)
    if (row) a.tau[bn + i] = tau_i;
    if (valid && i == 0) {
        a.status[b] = status;
        a.iters[b] = iters;
    }
}

template <int NP>
hipError_t launch_np(const QppvmArgs &a, hipStream_t stream)
{
    constexpr int IPW = kWave / NP;
    const size_t lds = sizeof(double) * Layout<NP>(a.ntasks).SIZE * IPW;
    static size_t attr_set = 0;
    if (lds > attr_set) {
        hipError_t e = hipFuncSetAttribute((const void *)qppvm_solve_kernel<NP>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = lds;
    }
    const unsigned grid = (unsigned)((a.B + IPW - 1) / IPW);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(qppvm_solve_kernel<NP>, dim3(grid), dim3(kWave), lds, stream, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_qppvm(const QppvmArgs &a, hipStream_t stream)
{
    if (a.n <= 32) return launch_np<32>(a, stream);
    return launch_np<64>(a, stream);
}

}  // namespace wbq
