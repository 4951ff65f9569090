// qppvm_w1m_kernel.hip -- batched QPPVM torque solve with the inertia-weighted joint task
// W1 = M (the KAT-2 variant), gfx950 (MI355X), fp64.
//
// Level 1 with W1 = M in the reference's variable x = tau - h (src/QPPVMPlugin.cpp:114-118,
// A1 = M^-1, b1 = M^-1 tau_imp) is
//   min 0.5 (x - tau_imp)^T M^-1 (x - tau_imp)
//   s.t. G M^-1 x = y*  (level-0 optimality; y* = b0 when level 0 is attainable)
//        lo <= x <= hi  (torque limits shifted by -h, :56-67, :203-205)
// (H1 = A1^T W1 A1 = M^-1, g1 = -M^-1 tau_imp: oracle/wbq_oracle.c:wbq_ref_assemble). The
// inverse Hessian is M itself -- given data -- so the dual active set runs in constraint
// space (dual_gi.h) with nothing factorised but the m0 solves M^-1 G^T:
//   rows A = [G M^-1 ; I],  H^-1 A^T = [G^T, M],  Gamma = A M A^T = [G M^-1 G^T, G ; G^T, M],
//   x0 = tau_imp, s0 = [G u_imp ; tau_imp],  x = tau_imp + G^T lam_E + M lam_B.
// Equality rows enter the active set like any violated row and are never dropped, so
// dependent level-0 rows are simply never added; inconsistent ones leave no step (status 2
// inside the loop): level 0 is not attainable at b0, and the repair kernel computes y* and
// the pinned limits by BVLS (the level0_repair of the W1 = I path) and solves again.
//
// The stack without a joint task (a.minnorm, wbq_desc no_joint_task: the reference's commented
// elbow stack ((ee_r + ee_l) / (elbow_l + elbow_r)) << limits, QPPVMPlugin.cpp:177-178) runs the
// same loop with H = I -- the eps -> 0 limit of QPOases_sot's regularisation (:188) decides the
// last level's optima by min 0.5 ||x||^2:
//   rows A = [G M^-1 ; I],  H^-1 A^T = A^T = [M^-1 G^T, I],  Gamma = [G M^-2 G^T, G M^-1 ; M^-1 G^T, I],
//   x0 = 0,  x = (M^-1 G^T) lam_E + lam_B.
// Every Cartesian row (level 0 and a second level, task_level) enters as an equality at its
// target; the repair computes y0*, y1* and the pins of both levels (level0_repair) when some
// target is not attainable.
//
// One instance per wave64 block, lane i <-> joint i for the staging and the Gauss-Jordan,
// lane ci <-> constraint row ci for the active set (m0 + n <= 64).
#include "wbq_kernels.h"
#include "wbq_device.h"
#include "dual_gi.h"

#include "qppvm_repair.h"

#include <math.h>

namespace wbq {
namespace {

// Per-instance LDS layout in doubles. Constraint index ci (= GI lane):
//   ci < m0              level-0 row c = ci:  (G M^-1)_c x = b0_c (y*_c after the repair)
//   m0 <= ci < m0 + n    torque limit of joint j = ci - m0:  lo_j <= x_j <= hi_j
struct W1mLayout {
    int ME, QS, GS, TS, KT;
    int JR, XG, GM, TT, PN, RH, XV, X0, U0, WT, VV, LV, RV, WV, DUM, AC, PS, F, QD, SIZE;
    __host__ __device__ W1mLayout(int n, int T, int m0, int NQ, int NRC)
    {
        ME = m0 + n;
        QS = NQ + 1;
        GS = ME | 1;
        KT = n > m0 ? n : m0;      // T rows: the active set never exceeds the primal dimension n
                                   // (dual_gi's cap), the level-0 batch writes m0 rows
        TS = (KT + 8) | 1;
        int o = 0;
        XG = o; o += (m0 * QS + 1) & ~1; // row c = (M^-1 G^T)[:, c] over the joint lanes
        GM = o; o += (ME * GS + 1) & ~1; // Gamma; its columns >= m0 are the rows of A M = (H^-1 A^T)^T
        TT = o;                    // T = L^-1 of the active-set Gram (rows of TS)
        {
            // setup-only data overlays T (first written after the barrier that ends the Gamma
            // assembly): J rows, task data, J_t^T F_t and the Gauss-Jordan panel. With KT rows
            // this is 36.9 -> 26.6 KB per instance at n = 30: 6 instances per CU instead of 4
            int ov = 0;
            JR = TT + ov; ov += T * 6 * NQ;     // J rows
            WT = TT + ov; ov += T * NQ;         // J_t^T F_t
            PS = TT + ov; ov += 24 * T;         // poses [R|p], ref
            F = TT + ov; ov += (6 * T + 1) & ~1; // task forces
            QD = TT + ov; ov += 64;
            PN = TT + ov; ov += 2 * NQ * kGjBS;     // Gauss-Jordan pivot panel
            RH = TT + ov; ov += 2 * kGjBS * NRC;    // its right-hand sides
            const int tt = KT * TS;
            o += tt > ov ? tt : ov;
        }
        XV = o; o += 64;           // x
        X0 = o; o += 64;           // x0 = tau_imp (0 without a joint task)
        U0 = o; o += 64;           // u_imp = M^-1 tau_imp
        VV = o; o += 72;
        LV = o; o += 72;
        RV = o; o += 72;
        WV = o; o += 72;
        DUM = o; o += 72;          // row of the lanes that own no T row
        AC = o; o += 72;
        SIZE = (o + 1) & ~1;
    }
};

// repair hand-over after the level-0 BVLS: pinned limits per joint, y* per level-0 row
struct RepairIn {
    static constexpr int LO = 0, HI = 64, YS = 128, SIZE = 128 + kM0Max;
};

struct W1mGi {
    static constexpr bool kOwnRowActivity = false;
    // Gamma = [G M^-1 G^T, G; G^T, M] is well scaled, but degenerate active sets (level-0 rows
    // plus pinned limits) push cond(Gamma_AA) to ~1e7: complements below 1e-10 Gamma_pp are
    // roundoff (scripts/emulate_w1m.py)
    static constexpr double kDep = 1e-10;
    double *S;
    const W1mLayout *L;
    int m0, n, i;
    int dim; // n
    __device__ double gamma(int r, int c) const { return S[L->GM + r * L->GS + c]; }
    __device__ double activity(int r) const
    {
        if (r >= m0) return S[L->XV + r - m0];
        const double *xg = S + L->XG + r * L->QS; // (G M^-1)_r x, chunks of 8 loads
        double s = 0.0;
        for (int j0 = 0; j0 < n; j0 += 8) {
            double gv[8], xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                gv[u] = xg[j0 + u];
                xv[u] = S[L->XV + j0 + u];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) s = fma(j0 + u < n ? gv[u] : 0.0, xv[u], s);
        }
        return s;
    }
    __device__ void rebuild(int pass, int k) const
    {
        if (i >= n) return;
        double dx = 0.0; // x_i += sum_q w_q (H^-1 a_q)_i = sum_q w_q Gamma[ac_q][m0 + i]
        for (int q0 = 0; q0 < k; q0 += 8) {
            int cq[8];
            double wq[8], xq[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                cq[u] = q0 + u < k ? (int)S[L->AC + q0 + u] : 0;
                wq[u] = q0 + u < k ? S[L->RV + q0 + u] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) xq[u] = S[L->GM + cq[u] * L->GS + m0 + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) dx = fma(wq[u], xq[u], dx);
        }
        S[L->XV + i] = (pass == 0 ? S[L->X0 + i] : S[L->XV + i]) + dx;
    }
};

// The whole W1 = M solve of instance b by one wave. rep (the repair kernel): limits and
// level-0 targets from the RepairIn block at R instead of tau_min/max and b0.
template <int NQ, int M0, int TM>
__device__ __forceinline__ void w1m_solve(const QppvmArgs &a, double *S, long b, int i, const double *R, int it0,
                                          int st0, bool l0inf = false)
{
    constexpr int NRC = 1 + M0; // Gauss-Jordan right-hand sides: tau_imp, G^T
    const int T = a.ntasks, n = a.n, m0 = a.m0;
    const W1mLayout L(n, T, m0, NQ, NRC);
    const bool mn = a.minnorm; // H = I, x0 = 0: no joint task (wbq_desc no_joint_task)
    const bool row = i < n;
    const int ic = row ? i : n - 1;

    // ------------------------------------------------------------------ 1. stage
    // unconditional buffer loads (clamped offsets, values selected afterwards): one HBM trip
    // buffer resources start at the instance (one per wave): per-lane offsets stay small
    const long bu = uniform_long(b), B = a.B;
    const int voff = (int)(8 * ic);
    const double q_i = bload(rsrc_at(a.q, bu, B, n), voff, 0), qd_i = bload(rsrc_at(a.qd, bu, B, n), voff, 0);
    const double qref_i = bload(rsrc_at(a.qref, bu, B, n), voff, 0), h_i0 = bload(rsrc_at(a.h, bu, B, n), voff, 0);
    double jv[TM * 6];
    {
        const __amdgpu_buffer_rsrc_t Jrs = rsrc_at(a.J, bu, B, (long)T * 6 * n);
        const int joff = (int)(8 * ic);
#pragma unroll
        for (int rr = 0; rr < TM * 6; ++rr) jv[rr] = bload(Jrs, joff, 8 * (rr < T * 6 ? rr : T * 6 - 1) * n);
    }
    constexpr int kPoseIt = (TM * 24 + 63) / 64;
    double pv[kPoseIt];
    {
        const __amdgpu_buffer_rsrc_t Prs = rsrc_at(a.pose, bu, B, (long)T * 12);
        const __amdgpu_buffer_rsrc_t Rrs = rsrc_at(a.pose_ref, bu, B, (long)T * 12);
#pragma unroll
        for (int it = 0; it < kPoseIt; ++it) {
            int e = it * 64 + i;
            e = e < T * 24 ? e : T * 24 - 1;
            const int t = e / 24, c = e - t * 24;
            const int cc = c < 12 ? c : c - 12;
            const double p0 = bload(Prs, (int)(8 * (t * 12 + cc)), 0);
            const double p1 = bload(Rrs, (int)(8 * (t * 12 + cc)), 0);
            pv[it] = (c < 12) ? p0 : p1;
        }
    }
    double A[NQ]; // M is symmetric: lane i's row is its column, so the loads coalesce
    {
        const __amdgpu_buffer_rsrc_t Mrs = rsrc_at(a.M, bu, B, (long)n * n);
        const int moff = (int)(8 * ic);
#pragma unroll
        for (int r = 0; r < NQ; ++r) A[r] = bload(Mrs, moff, 8 * (r < n ? r : n - 1) * n);
    }
    const double h_i = row ? h_i0 : 0.0;
    S[L.QD + i] = row ? qd_i : 0.0;
    if (i < NQ) {
#pragma unroll
        for (int rr = 0; rr < TM * 6; ++rr)
            if (rr < T * 6) S[L.JR + rr * NQ + i] = row ? jv[rr] : 0.0;
    }
#pragma unroll
    for (int it = 0; it < kPoseIt; ++it)
        if (it * 64 + i < T * 24) S[L.PS + it * 64 + i] = pv[it];
#pragma unroll
    for (int r = 0; r < NQ; ++r) A[r] = (row && r < n) ? A[r] : (r == i ? 1.0 : 0.0);
    if (row) { // Gamma bound row m0 + i: [G^T row i | M row i]  (without a joint task: [X row i | e_i])
#pragma unroll
        for (int r = 0; r < NQ; ++r)
            if (r < n) S[L.GM + (m0 + i) * L.GS + m0 + r] = mn ? (r == i ? 1.0 : 0.0) : A[r];
    }
    wave_sync();
    // task-space force per task row (spring + damper, zero desired twist), QPPVMPlugin.cpp:136-137
    if (i < T * 6) {
        const int t = i / 6, r = i - t * 6;
        double xd = 0.0;
#pragma unroll
        for (int j = 0; j < NQ; ++j) xd = fma(S[L.JR + i * NQ + j], S[L.QD + j], xd);
        const double er = cart_error_component(S + L.PS + t * 24, S + L.PS + t * 24 + 12, r);
        double Fv = a.Kc[i] * er - a.Dc[i] * xd;
        if (a.select_mode == 1 && !((a.row_mask[t] >> r) & 1)) Fv = 0.0;
        S[L.F + i] = Fv;
    }
    // G = the selected J rows (level-0 rows, :129-152): into both off-diagonal Gamma blocks
    double gc[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) gc[c] = (c < m0 && i < NQ) ? S[L.JR + a.row_sel[c < m0 ? c : 0] * NQ + i] : 0.0;
    if (row && !mn) {
#pragma unroll
        for (int c = 0; c < M0; ++c)
            if (c < m0) {
                S[L.GM + (m0 + i) * L.GS + c] = gc[c];
                S[L.GM + c * L.GS + m0 + i] = gc[c];
            }
    }
    wave_sync();
    if (i < NQ) { // J_t^T F_t (joint i)
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            double c = 0.0;
            if (t < T)
#pragma unroll
                for (int r = 0; r < 6; ++r) c = fma(S[L.JR + (t * 6 + r) * NQ + i], S[L.F + t * 6 + r], c);
            if (t < T) S[L.WT + t * NQ + i] = c;
        }
    }

    // ---------------------------------- 2. [u_imp, M^-1 G^T] by block Gauss-Jordan, M SPD
    const double tau_imp_i = row ? a.Kq[ic] * (qref_i - q_i) - a.Dq[ic] * qd_i : 0.0; // (:105-106)
    double rhs[NRC];
    rhs[0] = tau_imp_i;
#pragma unroll
    for (int c = 0; c < M0; ++c) rhs[1 + c] = gc[c];
    const bool notspd = block_gj<NQ, NRC, NRC>(A, rhs, n, i, S + L.PN, S + L.RH);
    if (i < NQ) {
#pragma unroll
        for (int c = 0; c < M0; ++c)
            if (c < m0) S[L.XG + c * L.QS + i] = rhs[1 + c];
    }
    if (row && mn) { // both off-diagonal Gamma blocks: (G M^-1)_c j = X_j c
#pragma unroll
        for (int c = 0; c < M0; ++c)
            if (c < m0) {
                S[L.GM + (m0 + i) * L.GS + c] = rhs[1 + c];
                S[L.GM + c * L.GS + m0 + i] = rhs[1 + c];
            }
    }
    S[L.U0 + i] = (i < NQ && row) ? rhs[0] : 0.0;
    S[L.X0 + i] = mn ? 0.0 : tau_imp_i;
    S[L.XV + i] = mn ? 0.0 : tau_imp_i;
    wave_sync();

    // ---------------------- 3. level-0 rows: Gamma_EE, targets b0, activities at x0
    // b0_c = G_c M^-1 J_t^T F_t = X_c . (J_t^T F_t), s0_c = X_c . x0 (lane c < m0);
    // Gamma_EE row i = X_i . Gamma[c][m0 + :] = G M^-1 G^T (W1 = M) or X^T X (no joint task)
    double b0 = 0.0, s0 = 0.0;
    if (i < m0) {
        const double *xg = S + L.XG + i * L.QS;
        const double *wt = S + L.WT + (a.row_sel[i] / 6) * NQ;
        double ge[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) ge[c] = 0.0;
        for (int j = 0; j < n; ++j) {
            const double x = xg[j];
            b0 = fma(x, wt[j], b0);
            s0 = fma(x, S[L.X0 + j], s0);
#pragma unroll
            for (int c = 0; c < M0; ++c) ge[c] = fma(x, S[L.GM + (c < m0 ? c : 0) * L.GS + m0 + j], ge[c]);
        }
#pragma unroll
        for (int c = 0; c < M0; ++c)
            if (c < m0) S[L.GM + i * L.GS + c] = ge[c];
    }

    // ------------------------------------------ 4. rows: kind, limits, activities
    const int ci = i;
    int kind = 0; // 0 disabled, 2 limits [lo, hi] (lo == hi: an equality)
    double lo = -kInf, hi = kInf, s_i = 0.0;
    if (ci < m0) {
        kind = 2;
        lo = hi = R ? R[RepairIn::YS + ci] : b0;
        s_i = s0;
    } else if (ci < L.ME) {
        const int j = ci - m0;
        kind = 2;
        const double hj = a.h[b * n + j];
        torque_box(a, j, a.q[b * n + j], a.qd[b * n + j], hj, lo, hi);
        if (R) {
            lo = R[RepairIn::LO + j];
            hi = R[RepairIn::HI + j];
        }
        s_i = S[L.X0 + j];
    }
    wave_sync();
    const double nrm = kind != 0 ? sqrt(fmax(S[L.GM + ci * L.GS + ci], 1e-300)) : 1.0;

    // ------------------------------------ 5. dual active set in constraint space
    SlotVec<64, false> Trow;
    TColView Tcol;
    GAView GA;
    Trow.bind(S + (i < L.KT ? L.TT + i * L.TS : L.DUM), L.KT);
    Tcol.bind(S + L.TT + (i < L.KT ? i : 0), L.TS);
    GA.bind(S + L.GM + (ci < L.ME ? ci : 0) * L.GS, S + L.AC);
    Trow.zero_from(0);
    S[L.DUM + i] = 0.0;
    GiState gs;
    // the JointLimits box can empty per instance (a joint beyond its limit and moving outwards)
    const bool empty_box = a.joint_limits && __any(kind == 2 && ci >= m0 && lo > hi);
    gs.status = st0 != 0 ? st0 : (notspd ? 3 : ((a.limits_crossed || empty_box) ? 2 : 0));
    wave_sync();
    const W1mGi pb{S, &L, m0, n, i, n};
    const GiVecs gv{L.VV, L.LV, L.RV, L.WV, L.AC, L.TT, L.TS};
    if (gs.status == 0) {
        // The m0 level-0 rows in one batch when Gamma_EE is well conditioned (dependent rows
        // are left to the loop, which never adds them): lane r < m0 holds row r of Gamma_EE, a
        // right-looking Cholesky runs across the lanes (pivots and columns by readlane), lane c
        // forward-substitutes column c of T = L^-1, and lambda_E = T^T T (b0 - s_E).
        double g[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) g[c] = (i < m0 && c < m0) ? S[L.GM + i * L.GS + c] : 0.0;
        double gd = 0.0;
#pragma unroll
        for (int c = 0; c < M0; ++c) gd = (i == c) ? g[c] : gd;
        const double dmx = imax<64>(gd);
        bool sing = false;
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            if (c < m0) {
                const double dcc = bcast(g[c], c);
                sing |= !(dcc > 1e-10 * dmx);
                const double ilc = dcc > 0.0 ? frsq(dcc) : 0.0;
                g[c] = (i > c) ? g[c] * ilc : ((i == c) ? dcc * ilc : g[c]); // L[r][c], r >= c
#pragma unroll
                for (int j = c + 1; j < M0; ++j) {
                    if (j < m0) {
                        const double ljc = bcast(g[c], j);
                        if (i >= j) g[j] = fma(-g[c], ljc, g[j]);
                    }
                }
            }
        }
        if (!sing) {
            double t[M0]; // column i of T (lanes i < m0)
#pragma unroll
            for (int r = 0; r < M0; ++r) {
                double acc = (i == r) ? 1.0 : 0.0;
#pragma unroll
                for (int q = 0; q < r; ++q) acc = fma(-bcast(g[q], r < m0 ? r : 0), t[q], acc);
                const double lrr = r < m0 ? bcast(g[r], r) : 0.0;
                t[r] = (i < m0 && lrr > 0.0) ? acc / lrr : 0.0;
            }
#pragma unroll
            for (int r = 0; r < M0; ++r)
                if (r < m0 && i < m0) S[L.TT + r * L.TS + i] = t[r]; // T rows (lane c writes column c)
            if (i < m0) S[L.VV + i] = lo - s_i;                       // b0 - s_E
            S[L.AC + i] = (double)i;                                   // slot q = row q
            wave_sync();
            const double w = i < m0 ? Trow.dot(S + L.VV, m0) : 0.0;
            S[L.LV + i] = w;
            wave_sync();
            const double lm = i < m0 ? Tcol.dot(S + L.LV, m0) : 0.0; // lambda_E
            S[L.RV + i] = lm;
            wave_sync();
            if (kind != 0) s_i += GA.dot(S + L.RV, m0);
            if (i < m0) {
                gs.act = i;
                gs.aeq = true;
                gs.lam = lm;
                gs.onact = true;
            }
            gs.k = m0;
            gs.iters = 1;
            wave_sync();
        }
    }
    // the last solve's active bounds on top of the level-0 batch (dual_gi.h warm_extend)
    if (gs.status == 0 && gs.k == m0 && m0 > 0 && !R && a.ws_rows) {
        const int wsg = (ci >= m0 && kind == 2) ? (int)a.ws_rows[b * 64 + i] : 0;
        (void)warm_extend<64>(pb, S, gv, i, Trow, Tcol, GA, kind, lo, hi, s_i, gs, wsg);
    }
    dual_gi<64>(pb, S, gv, i, Trow, Tcol, GA, kind, lo, hi, nrm, s_i, gs, a.max_iter);
    wave_sync();
    int status = gs.status;
    if ((status == 2 || status == 3) && !R && !a.limits_crossed && !empty_box && !notspd) {
        // no step: level 0 is not attainable at b0 inside the limits; or the active set went
        // numerically dependent, which near-inconsistent level-0 rows also cause -> repair
        // kernel (y* and the pins make the level-1 rows consistent)
        if (i < 64) a.ui_scr[b * 64 + i] = S[L.U0 + i];
        if (i < m0) a.b0_scr[b * kM0Max + i] = b0;
        if (i == 0) {
            a.status[b] = -2;
            wl_push(a, 1, b);
        }
        return;
    }

    // ------------------------------------------------------------------ 6. outputs
    double tau_i = row ? S[L.XV + i] + h_i : h_i;
    if (imax<64>((row && !isfinite(tau_i)) ? 1.0 : 0.0) > 0.0 && status == 0) status = 3;
    if (status != 0) tau_i = h_i; // "SOLVER ERROR!" fallback: tau_qp = 0 (:246-249)
    if (row) a.tau[b * n + i] = tau_i;
    if (a.integrate && !mn) { // qdd = M^-1 x = u_imp + (M^-1 G^T) lam_E + lam_B (refused without a joint task)
        S[L.RV + i] = i < gs.k ? gs.sgn * gs.lam : 0.0;
        S[L.AC + i] = (double)gs.act;
        wave_sync();
        double u = S[L.U0 + i];
        for (int q = 0; q < gs.k; ++q) {
            const int c = (int)S[L.AC + q];
            const double w = S[L.RV + q];
            u = fma(w, c < m0 ? S[L.XG + c * L.QS + (i < NQ ? i : 0)] : (c - m0 == i ? 1.0 : 0.0), u);
        }
        rollout_step(a, b, i, row, u, status == 0);
    }
    if (a.ws_rows) { // the next solve's warm start (a repaired solve's pinned problem: cold then)
        const int wrec = warm_record(S, gv, i, gs);
        a.ws_rows[b * 64 + i] = (signed char)((status == 0 && !R && kind == 2 && ci >= m0) ? wrec : 0);
    }
    if (i == 0) {
        a.status[b] = status;
        a.iters[b] = it0 + gs.iters;
        a.ws_hint[b] = l0inf ? 1 : 0; // wbq_get_warmstart_hints: this solve needed the level-0 repair
    }
}

template <int NQ, int M0, int TM>
__global__ __launch_bounds__(64) void qppvm_w1m_kernel(const QppvmArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    w1m_solve<NQ, M0, TM>(a, smem, blockIdx.x, threadIdx.x, nullptr, 0, 0);
}

// LDS of the level-0 repair (level0_repair<64, M0>): only the QA region of the active-set layout -- the
// Gauss-Jordan panel for A0, the 12-row BVLS slot matrix and the Q1 rows (64 rows of stride 65) -- so the repair
// kernel reserves that, not the whole 64-lane active-set layout (101 KB: one block per CU; 34 KB: four)
constexpr int kL0RepairLds = 64 * 65;

// Level-0 repair for W1 = M: BVLS for y* and the pinned limits (level0_repair of the W1 = I
// path, one instance per wave), then the W1 = M solve again with those.
template <int NQ, int M0, int TM>
__global__ __launch_bounds__(64) void qppvm_w1m_repair_kernel(const QppvmArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int i = threadIdx.x;
    const int n = a.n, m0 = a.m0;
    const int ws = kL0RepairLds;
    const int wm = W1mLayout(n, a.ntasks, m0, NQ, 1 + M0).SIZE;
    double *R = smem + (ws > wm ? ws : wm);
    const int cnt = a.work[a.epoch * 2 + 1];
    if (blockIdx.x == 0 && i == 0) { // the next solve's counters
        a.work[(a.epoch ^ 1) * 2] = 0;
        a.work[(a.epoch ^ 1) * 2 + 1] = 0;
    }
    follow_publish(a.fg, 0, cnt);
    for (int e = blockIdx.x; e < cnt; e += gridDim.x) {
        const long b = a.wl[a.B + e];
        const bool row = i < n;
        const int ic = row ? i : n - 1;
        const double h_i = row ? a.h[b * n + i] : 0.0;
        wave_sync(); // the previous instance's LDS is dead
        double lo = -kInf, hi = kInf;
        if (row) torque_box(a, i, a.q[b * n + i], a.qd[b * n + i], h_i, lo, hi);
        const RepairOut ro = level0_repair<64, M0>(a, 0, b, i, true, lo, hi, false);
        if (ro.unique && !a.integrate) { // level 1 over a single feasible point: x = x* (wave-uniform)
            int status = ro.status;
            double tau_i = row ? ro.x + h_i : h_i;
            if (imax<64>((row && !isfinite(tau_i)) ? 1.0 : 0.0) > 0.0 && status == 0) status = 3;
            if (status != 0) tau_i = h_i; // "SOLVER ERROR!" fallback: tau_qp = 0 (:246-249)
            if (row) a.tau[b * n + i] = tau_i;
            if (i == 0) {
                a.status[b] = status;
                a.iters[b] = ro.it;
                a.ws_hint[b] = ro.l0inf ? 1 : 0;
            }
            continue;
        }
        // y* = G u at the least-distance point of G u = y* that the repair leaves in u
        double ys[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            const double g = (row && c < m0) ? a.J[(b * a.ntasks * 6 + a.row_sel[c < m0 ? c : 0]) * n + ic] : 0.0;
            ys[c] = g * ro.u;
        }
        isum_vec<64, M0>(ys);
        wave_sync(); // the repair's LDS is dead
        R[RepairIn::LO + i] = ro.lo;
        R[RepairIn::HI + i] = ro.hi;
        if (i < M0) {
            double y = 0.0;
#pragma unroll
            for (int c = 0; c < M0; ++c) y = (c == i) ? ys[c] : y;
            R[RepairIn::YS + i] = y;
        }
        wave_sync();
        w1m_solve<NQ, M0, TM>(a, smem, b, i, R, ro.it, ro.status, ro.l0inf);
    }
}

template <int NQ, int M0, int TM>
hipError_t launch_w1m_t(const QppvmArgs &a, hipStream_t stream, hipEvent_t mid)
{
    const W1mLayout L(a.n, a.ntasks, a.m0, NQ, 1 + M0);
    if (L.ME > 64) return hipErrorInvalidValue;
    const size_t lds = sizeof(double) * L.SIZE;
    const int ws = kL0RepairLds;
    const size_t lds2 = sizeof(double) * ((ws > L.SIZE ? ws : L.SIZE) + RepairIn::SIZE);
    if (a.prepare) {
        const hipError_t e = ensure_dynamic_lds((const void *)qppvm_w1m_kernel<NQ, M0, TM>, lds);
        return e != hipSuccess ? e : ensure_dynamic_lds((const void *)qppvm_w1m_repair_kernel<NQ, M0, TM>, lds2);
    }
    hipLaunchKernelGGL((qppvm_w1m_kernel<NQ, M0, TM>), dim3((unsigned)a.B), dim3(64), lds, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (mid) {
        e = hipEventRecord(mid, stream);
        if (e != hipSuccess) return e;
    }
    const unsigned grid = follow_blocks(a.fg.est[1], 1, kFollowGrid, a.B);
    hipLaunchKernelGGL((qppvm_w1m_repair_kernel<NQ, M0, TM>), dim3(grid), dim3(64), lds2, stream, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_qppvm_w1m(const QppvmArgs &a, hipStream_t stream, hipEvent_t mid)
{
    if (a.B <= 0) return hipSuccess;
    // TM = 2 when at most two tasks: 12 J-row loads per lane instead of 24 (the stage stays under
    // the 63 outstanding vector loads, as the W1 = I fast kernel)
    // (a second Cartesian level takes the 12-row instantiation: its repair carries the middle step)
    const bool six = a.m0 <= 6 && a.m_l0 >= a.m0;
    if (a.ntasks <= 2) {
        if (a.n <= 32)
            return six ? launch_w1m_t<32, 6, 2>(a, stream, mid) : launch_w1m_t<32, kM0Max, 2>(a, stream, mid);
        return six ? launch_w1m_t<64, 6, 2>(a, stream, mid) : launch_w1m_t<64, kM0Max, 2>(a, stream, mid);
    }
    if (a.n <= 32)
        return six ? launch_w1m_t<32, 6, kTMax>(a, stream, mid) : launch_w1m_t<32, kM0Max, kTMax>(a, stream, mid);
    return six ? launch_w1m_t<64, 6, kTMax>(a, stream, mid) : launch_w1m_t<64, kM0Max, kTMax>(a, stream, mid);
}

}  // namespace wbq
