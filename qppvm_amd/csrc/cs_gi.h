// cs_gi.h -- the n <= 32 dual active set carried in constraint space (round 6), two instances per
// wave64 (lanes [0, 32) and [32, 64)), lane i <-> joint i. It replaces qppvm_kernel.hip's gi_solve at
// the fast kernel's inline call (and in the fused rollout): same problem, same interface, same statuses.
//
// The problem (reference src/QPPVMPlugin.cpp:201-259, the limits :56-67):
//   min 0.5 ||u - u_hat||^2   s.t.  G u = b0,   lo <= M u <= hi
// from the equality-constrained optimum u0 (the fast path's u) and Q1 (an orthonormal basis of G's rows).
// With P = I - Q1^T Q1 the dual active set only ever needs Gamma = M P M -- the Gram of the bound normals
// projected onto null(G) -- and the activities s = M u:
//   adding bound p (side sg_p): v = sg_A sg_p Gamma[A][p], r = K^-1 v (K = Gamma_AA signed), d2 = Gamma_pp - v.r,
//   ds = sg_p Gamma[:][p] - Gamma[:][A] sg_A r (the change of every activity per unit step), the step
//   t = min(t1 (a multiplier reaches zero), t2 = -slack_p / (sg_p ds_p)); s += t ds, lambda_A -= t r.
// Gamma's columns are formed on demand, one per bound that enters the active set: w = P m_p (six DPP sums),
// c = M w (one LDS dot against M's row in registers), kept in LDS (GA, one row per lane over the slots). K is
// kept as T = L^-1 (K = L L^T, packed rows in LDS; an add appends one row in closed form, a drop re-appends the
// rows after it, as dual_gi.h). Per pass that is O(k) LDS reads per lane plus one 32-element dot, where the
// u-space loop it replaces (T rows and M rows in VGPRs, Gram-Schmidt against Q1 in LDS) read four 32-element
// dots per pass at the 256-VGPR cap, each LDS read waited for in turn (DESIGN.md 3.1, round 5 lap counters:
// ~20k cycles per select pass, ~46k per full pass, ~123k for the config-2 warm batch).
// The incremental activities drift from the exact ones by roundoff, so when no bound is violated u is rebuilt
// from the multipliers, u = u0 + P M rho (rho_j = sg lambda on the active joints), x = M u, with refinement
// passes on the active set (lambda += K^-1 (beta_A - sg_A x_A)), and every bound re-checked at the exact x.
// What the storage or the numerics cannot carry (more than KM active bounds, an active bound the rebuilt x
// misses, the rebuild-round cap) is handed to the level-0 repair as if level 0 were infeasible: its BVLS
// settles level 0 first and a feasible instance comes back unpinned to the u-space loop -- the same solution
// by another path (as the n > 32 hand-off).
// The numpy statement of this loop, step for step: scripts/emulate_cs_gi.py.
#pragma once
#include "wbq_kernels.h"
#include "wbq_device.h"

namespace wbq {

// Per-instance LDS (doubles), inside ActiveLayout<32>'s 1,248 (the caller's Q1 rows at the start of the
// region are read into registers first; GA then overlays them)
template <int NP_>
struct CsLayoutT {
    static constexpr int NP = NP_;
    static constexpr int KM = NP == 32 ? 24 : 40, GS = KM + 1; // slots; GA row stride (odd: lane rows conflict-free)
    static constexpr int GA = 0;                        // [NP][GS] Gamma[i][act_a]
    static constexpr int TP = GA + NP * GS;             // T = L^-1, packed lower rows, KM (KM + 1) / 2
    static constexpr int WV = TP + KM * (KM + 1) / 2;   // w = P m_p, then u (broadcast vectors)
    static constexpr int VV = WV + NP;                  // v, residuals, rho by joint
    static constexpr int LV = VV + NP;                  // l = T v
    static constexpr int RV = LV + NP;                  // sg r
    static constexpr int SIZE = RV + NP;
};
using CsLayout = CsLayoutT<32>;
static_assert(CsLayoutT<32>::SIZE <= 32 * 33 + 6 * 32, "CsLayout fits ActiveLayout<32>");
static_assert(CsLayoutT<64>::SIZE <= 64 * 65, "CsLayout<64> fits the QA region of ActiveLayout<64>");
static_assert(CsLayoutT<32>::WV % 2 == 0 && CsLayoutT<32>::TP % 2 == 0, "16-byte aligned vectors");
static_assert(CsLayoutT<64>::WV % 2 == 0 && CsLayoutT<64>::TP % 2 == 0, "16-byte aligned vectors");

// LDS ordering inside the loop. The fast kernel's workgroup is one wave, and the LDS unit executes one wave's
// DS instructions in issue order, so a write by one lane is seen by a later read of another lane of the same
// wave without a workgroup barrier: only the compiler must keep the order (a signal fence). lds_barrier() drains
// every outstanding LDS access first (s_waitcnt lgkmcnt(0)): one LDS round trip per use, ~6 per pass.
// WBQ_CS_WAVE_LDS = 0: lds_barrier() (A/B).
#ifndef WBQ_CS_WAVE_LDS
#define WBQ_CS_WAVE_LDS 1
#endif
__device__ __forceinline__ void cs_order()
{
#if WBQ_CS_WAVE_LDS
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
#else
    lds_barrier();
#endif
}

// ---------------------------------------------------------------- NP = 32 lane helpers
// value of v at lane idx of this lane's instance (idx instance-uniform): v_readlane, no LDS (NP = 32: one per half)
template <int NP>
__device__ __forceinline__ double cs_bcast(double v, int idx)
{
    if constexpr (NP == 64) {
        return lane_f64(v, __builtin_amdgcn_readfirstlane(idx) & 63);
    } else {
        const int i0 = __builtin_amdgcn_readlane(idx, 0) & 31, i1 = __builtin_amdgcn_readlane(idx, 32) & 31;
        const double a0 = lane_f64(v, i0), a1 = lane_f64(v, 32 + i1);
        return (threadIdx.x & 32) ? a1 : a0;
    }
}
template <int NP>
__device__ __forceinline__ int cs_bcast_i(int v, int idx)
{
    if constexpr (NP == 64) {
        return __builtin_amdgcn_readlane(v, __builtin_amdgcn_readfirstlane(idx) & 63);
    } else {
        const int i0 = __builtin_amdgcn_readlane(idx, 0) & 31, i1 = __builtin_amdgcn_readlane(idx, 32) & 31;
        const int a0 = __builtin_amdgcn_readlane(v, i0), a1 = __builtin_amdgcn_readlane(v, 32 + i1);
        return (threadIdx.x & 32) ? a1 : a0;
    }
}
// value at lane s of each instance (s wave-uniform)
template <int NP>
__device__ __forceinline__ double cs_at(double v, int s)
{
    if constexpr (NP == 64) {
        return lane_f64(v, s);
    } else {
        const double a0 = lane_f64(v, s), a1 = lane_f64(v, 32 + s);
        return (threadIdx.x & 32) ? a1 : a0;
    }
}
// wave-uniform max / min of an instance-uniform count (SGPR: loops over it are scalar loops)
template <int NP>
__device__ __forceinline__ int cs_wmax(int v)
{
    if constexpr (NP == 64) return __builtin_amdgcn_readfirstlane(v);
    const int a0 = __builtin_amdgcn_readlane(v, 0), a1 = __builtin_amdgcn_readlane(v, 32);
    return a0 > a1 ? a0 : a1;
}
template <int NP>
__device__ __forceinline__ int cs_wmin(int v)
{
    if constexpr (NP == 64) return __builtin_amdgcn_readfirstlane(v);
    const int a0 = __builtin_amdgcn_readlane(v, 0), a1 = __builtin_amdgcn_readlane(v, 32);
    return a0 < a1 ? a0 : a1;
}

// M's row (in registers) times an NP-vector in LDS, the reads in chunks issued before their FMAs (NP = 32: all 32,
// one LDS round trip; NP = 64: chunks of 16, the row itself already takes 128 VGPRs)
template <int NP>
__device__ __forceinline__ double cs_rdot(const double (&m)[NP], const double *b)
{
    constexpr int CH = NP == 64 ? 16 : 32;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int j0 = 0; j0 < NP; j0 += CH) {
        double bv[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) bv[j] = b[j0 + j];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < CH; ++j) s[j & 3] = fma(m[j0 + j], bv[j], s[j & 3]);
    }
    return (s[0] + s[1]) + (s[2] + s[3]);
}

// sum_j row[j] vec[j] over the slots j < kmax (row: this lane's GA row, finite everywhere -- zeroed at the
// start; vec: a broadcast LDS vector, zero past the live slots, so no masks), chunks of eight reads issued
// together; kmax (wave-uniform, <= KM) bounds the scalar loop
__device__ __forceinline__ double cs_gdot(const double *row, const double *vec, int kmax)
{
    double s0 = 0.0, s1 = 0.0;
    for (int j0 = 0; j0 < kmax; j0 += 8) {
        double rv[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            rv[u] = row[j0 + u];
            bv[u] = vec[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            s0 = fma(rv[u], bv[u], s0);
            s1 = fma(rv[u + 1], bv[u + 1], s1);
        }
    }
    return s0 + s1;
}
// sum_{j <= a} T[a][j] vec[j]: row a of the packed T (entries past the diagonal belong to later rows: masked;
// vec is zero past the live slots)
template <int KM>
__device__ __forceinline__ double cs_trowdot(const double *tp, int a, const double *vec, int kmax)
{
    const int ac = a < KM ? a : KM - 1;
    const double *row = tp + ac * (ac + 1) / 2;
    double s0 = 0.0, s1 = 0.0;
    for (int j0 = 0; j0 < kmax; j0 += 8) {
        double rv[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            rv[u] = row[j0 + u];
            bv[u] = vec[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            s0 = fma(j0 + u <= a ? rv[u] : 0.0, bv[u], s0);
            s1 = fma(j0 + u + 1 <= a ? rv[u + 1] : 0.0, bv[u + 1], s1);
        }
    }
    return s0 + s1;
}
// sum_{j >= a} T[j][a] vec[j]: column a of the packed T (T finite everywhere -- zeroed at the start; vec zero
// past the live slots)
template <int KM>
__device__ __forceinline__ double cs_tcol(const double *tp, int a, const double *vec, int kmax)
{
    const int ac = a < KM ? a : KM - 1;
    double s0 = 0.0, s1 = 0.0;
    for (int j0 = 0; j0 < kmax; j0 += 8) {
        double tv[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + u < KM ? j0 + u : KM - 1;
            tv[u] = tp[j * (j + 1) / 2 + ac];
            bv[u] = vec[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            s0 = fma(j0 + u >= a ? tv[u] : 0.0, bv[u], s0);
            s1 = fma(j0 + u + 1 >= a ? tv[u + 1] : 0.0, bv[u + 1], s1);
        }
    }
    return s0 + s1;
}

// Lane state of the loop. Slot a (lane a < k): act (its joint), sg (normal = sg * M row act), lam, beta (the
// bound in the signed form sg s_act >= beta), aeq (lo == hi: never dropped). Lane j (joint j): onact.
struct CsSlots {
    int k = 0, act = 0;
    double sg = 1.0, lam = 0.0, beta = 0.0;
    bool aeq = false;
};

// Gamma[:][p] for the instance-uniform joint p: w = P m_p, c_i = M_i . w; cpp = |w|^2 = Gamma_pp. vcol: this
// lane's column of V = Q1 M, so Q1 m_p is lane p's (no reduction)
template <int NP, int M0>
__device__ __forceinline__ double cs_column(double *S, const double (&mrow)[NP], const double (&q1)[M0],
                                           const double (&vcol)[M0], int i, int p, double &cpp)
{
    // M[i][p] = M[p][i] (a select chain: a select tree on p's bits became a dynamically indexed copy of the row
    // in scratch, 0 -> 496 B)
    double mp = 0.0;
#pragma unroll
    for (int r = 0; r < NP; ++r) mp = (r == p) ? mrow[r] : mp;
    double w = mp;
#pragma unroll
    for (int c = 0; c < M0; ++c) w = fma(-q1[c], cs_bcast<NP>(vcol[c], p), w);
    cpp = isum<NP>(w * w);
    cs_order(); // (the previous readers of WV)
    S[CsLayoutT<NP>::WV + i] = w;
    cs_order();
    return cs_rdot<NP>(mrow, S + CsLayoutT<NP>::WV);
}

// l = T v, r = T^T l on the slot lanes (a < cnt; v on those lanes), through VV / LV
template <int NP>
__device__ __forceinline__ void cs_tsolve(double *S, int i, double v, int cnt, int kmax, double &l, double &r)
{
    S[CsLayoutT<NP>::VV + i] = i < cnt ? v : 0.0;
    cs_order();
    l = i < cnt ? cs_trowdot<CsLayoutT<NP>::KM>(S + CsLayoutT<NP>::TP, i, S + CsLayoutT<NP>::VV, kmax) : 0.0;
    S[CsLayoutT<NP>::LV + i] = l;
    cs_order();
    r = i < cnt ? cs_tcol<CsLayoutT<NP>::KM>(S + CsLayoutT<NP>::TP, i, S + CsLayoutT<NP>::LV, kmax) : 0.0;
}

// u = u0 + P M rho, x = M u on the lanes with on set (instance-uniform); collective
template <int NP, int M0>
__device__ __forceinline__ void cs_rebuild(double *S, const double (&mrow)[NP], const double (&q1)[M0], int i,
                                           bool on, const CsSlots &g, double u0, double &u, double &x)
{
    cs_order();
    S[CsLayoutT<NP>::VV + i] = 0.0;
    cs_order();
    if (on && i < g.k) S[CsLayoutT<NP>::VV + g.act] = g.sg * g.lam;
    cs_order();
    const double y = cs_rdot<NP>(mrow, S + CsLayoutT<NP>::VV);
    double vq[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) vq[c] = q1[c] * y;
    isum_vec<NP, M0>(vq);
    double py = y;
#pragma unroll
    for (int c = 0; c < M0; ++c) py = fma(-q1[c], vq[c], py);
    const double un = u0 + py;
    S[CsLayoutT<NP>::WV + i] = un;
    cs_order();
    const double xn = cs_rdot<NP>(mrow, S + CsLayoutT<NP>::WV);
    if (on) {
        u = un;
        x = xn;
    }
}

constexpr int kCsRounds = 8;       // rebuilds per solve before the hand-off
constexpr double kCsDep = 1e-14;   // a row whose Schur complement is below kCsDep Gamma_pp is dependent

// The loop (see the head of this file). Q1's rows are in S's first rows (stride 33, the active-set layout's
// QA) on entry; vcol = this lane's column of V = Q1 M (the fast path has it from Y = M G^T: V^T = Y L^-T). Returns this lane's x = M u (exact, rebuilt); u_out = u. status 1: step cap; infeasible: no
// step exists (level 0 not attainable at b0 inside the bounds) or the hand-off described above. wsg: the
// warm side of this lane's bound (+1 lower, -1 upper, 0 none); record: the final active set to ws_rows.
// bail: the hand-off described at the head of this file (more than KM active bounds, an active bound the rebuilt
// x misses, the rebuild-round cap); with VIN false the instance's Q1 rows are back in LDS then, so the u-space
// loop can take it.
// (LAPB / LAPC: stamp slots of the diagnostic build's lap counters, as gi_solve: 8 phases from LAPB -- setup,
// warm appends, warm multipliers, select, column, step, drop, rebuild -- and 2 counts from LAPC: passes, rebuilds)
// VIN: vcol and x0 = M u0 are given (the fast path); else they are formed here (vcol from Q1's rows in LDS: the
// repair)
template <int NP, int M0, int LAPB = 0, int LAPC = 0, bool VIN = true>
__device__ __forceinline__ double cs_solve(const QppvmArgs &a, double *S, long b, int i, bool row, bool go,
                                           double lo, double hi, double u0, int &status, int &iters,
                                           bool &infeasible, int wsg, bool record, double &u_out,
                                           const double (&vin)[M0], bool &bail, double x0 = 0.0, int handoff = 0)
{
    using L = CsLayoutT<NP>;
    constexpr int KM = L::KM, GS = L::GS;
    const int n = a.n, m0 = a.m0;
    const int ic = i < n ? i : n - 1;
    WBQ_LAP_INIT;
    double q1[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) q1[c] = c < m0 ? S[c * (NP + 1) + i] : 0.0;
    const double *Mb = a.M + b * n * n + ic;
    double mrow[NP];
#pragma unroll
    for (int r = 0; r < NP; ++r) mrow[r] = Mb[(r < n ? r : n - 1) * n];
#pragma unroll
    for (int r = 0; r < NP; ++r) mrow[r] = (row && r < n) ? mrow[r] : (r == i ? 1.0 : 0.0);
    double nrm2 = 0.0;
#pragma unroll
    for (int r = 0; r < NP; ++r) nrm2 = fma(mrow[r], mrow[r], nrm2);
    const double inrm = frsq(nrm2); // (the selection's scale: 1 / |M row i|)
    double vcol[M0];
    if constexpr (VIN) {
#pragma unroll
        for (int c = 0; c < M0; ++c) vcol[c] = vin[c];
    } else { // V[c][i] = Q1 row c . M column i
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            double v = 0.0;
            if (c < m0)
#pragma unroll
                for (int r = 0; r < NP; ++r) v = fma(S[c * (NP + 1) + r], mrow[r], v);
            vcol[c] = v;
        }
    }
    bail = false;
    int dim;
    {
        double qq[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) qq[c] = q1[c] * q1[c];
        isum_vec<NP, M0>(qq);
        int rk = 0;
#pragma unroll
        for (int c = 0; c < M0; ++c) rk += (c < m0 && qq[c] > 0.5) ? 1 : 0;
        dim = n - rk; // independent bound normals the loop can hold (rank cap)
    }
    const bool eqb = lo == hi;
    cs_order(); // every lane has its Q1 column: the region is the loop's now
    // GA and T are read (masked or against zero vector entries) past the live slots: finite from the start
#pragma unroll
    for (int j = 0; j < KM; ++j) S[L::GA + i * GS + j] = 0.0;
#pragma unroll
    for (int j = 0; j < (KM * (KM + 1) / 2 + NP - 1) / NP; ++j)
        if (j * NP + i < KM * (KM + 1) / 2) S[L::TP + j * NP + i] = 0.0;
    double s;
    if constexpr (VIN) {
        s = x0; // the fast path's x = M u0 (the activities its bound check saw)
    } else {
        S[L::WV + i] = u0;
        cs_order();
        s = cs_rdot<NP>(mrow, S + L::WV); // s = M u0
    }
    double u = u0, x = s;
    CsSlots g;
    bool onact = false;
    WBQ_LAP(0);
    infeasible = false;
    bool dirty = false;
    // ------------------------------------------------ warm start: the last active set in one batch
    if (__any(go && row && wsg != 0)) {
        const bool wme = go && row && wsg != 0;
        const unsigned long long bal = __ballot(wme);
        unsigned long long rem = NP == 64 ? bal : ((bal >> (threadIdx.x & 32)) & 0xffffffffull);
        const int kw = __popcll(rem);
        const int kwmax = cs_wmax<NP>(kw);
        bool dep = kw > KM || kw > dim;
        for (int a2 = 0; a2 < kwmax; ++a2) {
            const bool on = a2 < kw && !dep;
            const int j = rem ? __builtin_ctzll(rem) : 0;
            rem &= rem ? rem - 1ull : 0ull;
            const double sj = (double)cs_bcast_i<NP>(wsg, j);
            double cpp;
            const double c = cs_column<NP, M0>(S, mrow, q1, vcol, i, j, cpp);
            const double cg = __shfl(c, g.act, NP);
            const double v = (on && i < a2) ? g.sg * sj * cg : 0.0;
            double l, r;
            cs_tsolve<NP>(S, i, v, on ? a2 : 0, a2 < KM ? a2 + 1 : KM, l, r);
            const double d2 = cpp - isum<NP>(l * l);
            if (on && !(d2 > kCsDep * cpp)) dep = true; // a dependent batch: start cold
            const bool on2 = on && !dep;
            const double id = d2 > 0.0 ? frsq(d2) : 0.0;
            if (on2 && i < a2) S[L::TP + a2 * (a2 + 1) / 2 + i] = -r * id;
            if (on2 && i == a2) S[L::TP + a2 * (a2 + 1) / 2 + a2] = id;
            if (on2) S[L::GA + i * GS + a2] = c;
            const double loj = cs_bcast<NP>(lo, j), hij = cs_bcast<NP>(hi, j);
            const bool eqj = cs_bcast_i<NP>(eqb ? 1 : 0, j) != 0;
            if (on2 && i == a2) {
                g.act = j;
                g.sg = sj;
                g.lam = 0.0;
                g.aeq = eqj;
                g.beta = sj > 0.0 ? loj : -hij;
            }
        }
        WBQ_LAP(1);
        // multipliers of the batch optimum from u0: K lambda = beta_W - sg_W s_W
        const int kk = dep ? 0 : kw;
        const double xa = __shfl(s, g.act, NP);
        double l, lw;
        cs_tsolve<NP>(S, i, g.beta - g.sg * xa, kk, kwmax < KM ? kwmax : KM, l, lw);
        const double lmx = imax<NP>(i < kk ? fabs(lw) : 0.0);
        const bool bad = imax<NP>((i < kk && !g.aeq && lw < -1e-12 * (1.0 + lmx)) ? 1.0 : 0.0) > 0.0;
        const bool keep = kk > 0 && !bad;
        S[L::RV + i] = (keep && i < kk) ? g.sg * lw : 0.0;
        cs_order();
        const double dsw = cs_gdot(S + L::GA + i * GS, S + L::RV, kwmax < KM ? kwmax : KM);
        if (keep) {
            s += dsw;
            if (i < kk) g.lam = g.aeq ? lw : fmax(lw, 0.0);
            g.k = kk;
            onact = wme;
            iters += 1;
            dirty = true;
        }
        WBQ_LAP(2);
    }
    // ------------------------------------------------ the loop
    const int maxit = a.max_iter;
    bool need_select = true, recheck = false, have_col = false;
    int rounds = 0, p = 0, cdrop = -1;
    double sgp = 1.0, bnd = 0.0, lamp = 0.0, c = 0.0, cpp = 0.0;
    bool peq = false;
    while (true) {
        if (__any(cdrop >= 0)) {
            // drop slot cdrop: the slots after it move down; T rows before it stand, the later ones are
            // re-appended from their Gamma columns (GA)
            const bool dr = cdrop >= 0;
            const int cd = dr ? cdrop : 0;
            const int cb = cs_bcast_i<NP>(g.act, cd);
            if (dr && i == cb) onact = false;
            const int na = __shfl(g.act, i + 1, NP);
            const double ns = __shfl(g.sg, i + 1, NP), nl = __shfl(g.lam, i + 1, NP), nb = __shfl(g.beta, i + 1, NP);
            const bool ne = __shfl(g.aeq ? 1 : 0, i + 1, NP) != 0;
            if (dr && i >= cd) {
                g.act = na;
                g.sg = ns;
                g.lam = nl;
                g.beta = nb;
                g.aeq = ne;
            }
            if (dr) {
                for (int a3 = cd; a3 + 1 < g.k; ++a3) S[L::GA + i * GS + a3] = S[L::GA + i * GS + a3 + 1];
                --g.k;
            }
            cs_order();
            const int amin = cs_wmin<NP>(dr ? cd : KM), amax = cs_wmax<NP>(dr ? g.k : 0);
            for (int a2 = amin; a2 < amax; ++a2) {
                const bool on = dr && a2 >= cd && a2 < g.k;
                const double sa = cs_at<NP>(g.sg, a2);
                const double gv = S[L::GA + g.act * GS + a2]; // Gamma[act_b][act_a2]
                const double diag = cs_at<NP>(gv, a2);
                double l, r;
                cs_tsolve<NP>(S, i, sa * g.sg * gv, on ? a2 : 0, a2 + 1, l, r);
                const double e2 = diag - isum<NP>(l * l);
                const double id = e2 > 0.0 ? frsq(e2) : 0.0;
                if (on && i < a2) S[L::TP + a2 * (a2 + 1) / 2 + i] = -r * id;
                if (on && i == a2) S[L::TP + a2 * (a2 + 1) / 2 + a2] = id;
            }
            cdrop = -1;
            cs_order();
            WBQ_LAP(6);
        }
        bool rb = false;
        if (need_select) {
            double v = -1.0;
            if (go && row && !onact) {
                const double tol = 1e-10 * fmax(1.0, fmax(fabs(s), fmax(fabs(lo), fabs(hi))));
                const double viol = fmax(lo - s, s - hi);
                if (viol > tol) v = viol * inrm;
            }
            int pi = i;
            iargmax<NP>(v, pi);
            if (!(v > 0.0) || recheck) {
                recheck = false;
                // no violated bound at these activities: optimal if they are exact, else rebuild first
                rb = go && dirty;
                if (go && !dirty) go = false;
            } else {
                p = pi;
                sgp = (cs_bcast<NP>(lo - s, p) > cs_bcast<NP>(s - hi, p)) ? 1.0 : -1.0;
                bnd = sgp > 0.0 ? cs_bcast<NP>(lo, p) : cs_bcast<NP>(hi, p);
                peq = cs_bcast_i<NP>(eqb ? 1 : 0, p) != 0;
                lamp = 0.0;
                have_col = false;
            }
        }
        WBQ_LAP(3);
        if (__any(rb)) {
            // u and x from the multipliers, refinement on the active set, then every bound re-checked
            cs_rebuild<NP, M0>(S, mrow, q1, i, rb, g, u0, u, x);
            const int kmx = cs_wmax<NP>(rb ? g.k : 0);
            if (kmx > 0) {
                for (int pass = 0; pass < 3; ++pass) {
                    const double xa = __shfl(x, g.act, NP);
                    const double res = (rb && i < g.k) ? g.beta - g.sg * xa : 0.0;
                    const double rmx = imax<NP>(rb ? fabs(res) / (1.0 + fabs(xa)) : 0.0);
                    if (!__any(rb && rmx > 1e-13)) break;
                    double l, dl;
                    cs_tsolve<NP>(S, i, res, rb ? g.k : 0, kmx, l, dl);
                    if (rb && i < g.k) g.lam += dl;
                    cs_rebuild<NP, M0>(S, mrow, q1, i, rb, g, u0, u, x);
                }
                // every active bound must hold at the rebuilt x, else the factor is too poor: hand off
                const double xa = __shfl(x, g.act, NP);
                const double miss = (rb && i < g.k) ? fabs(g.beta - g.sg * xa) / (1.0 + fabs(xa)) : 0.0;
                if (rb && imax<NP>(miss) > 1e-8) {
                    bail = true;
                    go = false;
                }
            }
            if (rb) {
                s = x;
                dirty = false;
                if (++rounds > kCsRounds && go) {
                    bail = true;
                    go = false;
                }
            }
            WBQ_LAP(7);
            WBQ_LAP_ADD(1, 1);
            continue;
        }
        if (!__any(go)) break;
        if (__any(go && !have_col)) { // (a drop keeps stepping on p: its column is kept)
            double cppn;
            const double cn = cs_column<NP, M0>(S, mrow, q1, vcol, i, p, cppn);
            if (!have_col) {
                c = cn;
                cpp = cppn;
                have_col = true;
            }
        }
        WBQ_LAP(4);
        WBQ_LAP_ADD(0, 1);
        // ---- the step for bound p
        const int k = g.k, kmx = cs_wmax<NP>(go ? k : 0);
        const double cg = __shfl(c, g.act, NP); // Gamma[act_a][p] on slot lane a
        const double v = (i < k) ? g.sg * sgp * cg : 0.0;
        double l, r;
        cs_tsolve<NP>(S, i, v, go ? k : 0, kmx, l, r);
        const double d2 = cpp - isum<NP>(l * l);
        S[L::RV + i] = (go && i < k) ? g.sg * r : 0.0;
        cs_order();
        const double ds = sgp * c - cs_gdot(S + L::GA + i * GS, S + L::RV, kmx);
        const double zz = sgp * cs_bcast<NP>(ds, p);
        const double slack = sgp * (cs_bcast<NP>(s, p) - bnd); // < 0: violated
        const double rmax = imax<NP>(i < k ? fabs(r) : 0.0);
        double cand = (i < k && !g.aeq && r > 1e-13 * rmax) ? g.lam * frcp(r) : kInf;
        int ci = i;
        iargmin<NP>(cand, ci);
        const double t1 = cand;
        const double t2 = (k < dim && d2 > kCsDep * cpp && zz > 0.0) ? -slack * frcp(zz) : kInf;
        if (go) {
            if (t1 >= kInf && t2 >= kInf) {
                // no step: the bounds cannot all be met -- unless the incremental activities drifted; then
                // rebuild, re-check, select again, and report it only if the exact activities agree
                if (dirty) {
                    recheck = true;
                    need_select = true;
                } else {
                    infeasible = true;
                    go = false;
                }
            } else if (t2 <= t1 && k >= KM) {
                bail = true; // slot storage: hand off
                go = false;
            } else {
                dirty = true;
                const double t = fmin(t1, t2);
                s = fma(t, ds, s);
                if (i < k) g.lam = fma(-t, r, g.lam);
                lamp += t;
                ++iters;
                if (t2 <= t1) { // add p: T row k = [-r^T / d, 1 / d], Gamma column k = c
                    const double id = frsq(d2);
                    if (i < k) S[L::TP + k * (k + 1) / 2 + i] = -r * id;
                    if (i == k) {
                        S[L::TP + k * (k + 1) / 2 + k] = id;
                        g.act = p;
                        g.sg = sgp;
                        g.lam = lamp;
                        g.aeq = peq;
                        g.beta = sgp > 0.0 ? bnd : -bnd;
                    }
                    S[L::GA + i * GS + k] = c;
                    if (i == p) onact = true;
                    ++g.k;
                    need_select = true;
                } else { // drop slot ci (its multiplier reached zero), keep stepping on p
                    cdrop = ci;
                    need_select = false;
                }
                if (iters >= maxit && go) {
                    status = 1;
                    go = false;
                }
                // handoff > 0: a loop still running after that many steps goes to the level-0 repair as if
                // infeasible (its BVLS settles level 0 first; a feasible instance comes back unpinned: the same
                // result), as gi_solve's
                if (handoff > 0 && iters >= handoff && go) {
                    infeasible = true;
                    go = false;
                }
            }
        }
        WBQ_LAP(5);
    }
    if (record) { // the final active set, by joint, for the next solve of this instance
        cs_order();
        S[L::VV + i] = 0.0;
        cs_order();
        if (i < g.k && !g.aeq) S[L::VV + g.act] = g.sg;
        cs_order();
        const double sgn = S[L::VV + i];
        const bool ok = status == 0 && !infeasible;
        if (row && a.ws_rows) a.ws_rows[b * 64 + i] = (signed char)(ok ? (sgn > 0.0 ? 1 : (sgn < 0.0 ? -1 : 0)) : 0);
        cs_order();
    }
    WBQ_LAP(3);
    if constexpr (LAPB > 0) WBQ_LAP_FLUSH(LAPB, LAPC);
    if (!VIN && __any(bail)) { // (the repair) Q1's rows back where the u-space loop reads them
        cs_order();
#pragma unroll
        for (int c = 0; c < M0; ++c)
            if (bail && c < m0) S[c * (NP + 1) + i] = q1[c];
        cs_order();
    }
    u_out = u;
    return x;
}

}  // namespace wbq
