// dual_gi.h -- Goldfarb-Idnani dual active set carried in constraint space, one lane per
// constraint row (gfx950, wave64, fp64). Shared by the contact-form kernel and the QPPVM
// W1 = M kernel: both solve
//   min 0.5 (x - x0)^T H (x - x0)   s.t.  lo_j <= a_j x <= hi_j  (lo_j == hi_j: equality)
// knowing only Gamma = A H^-1 A^T (m x m), the activities s = A x and H^-1 A^T. The
// active-set Gram Gamma_AA = L L^T is kept as T = L^-1 (an add appends one row of T in
// closed form, a drop re-appends the rows after it) and x is rebuilt from the multipliers,
// x = x0 + H^-1 A_A^T lambda, only when the active set settles; two steps of iterative
// refinement on the final active set (residuals exact in x-space; up to four while an active row
// still misses, for nearly dependent sets) and a re-check of every row follow (the algorithm the oracle restates in
// oracle/wbq_oracle_contact.c and oracle/wbq_oracle.c).
//
// The problem supplies a policy P with
//   double gamma(int r, int c) const      Gamma[r][c]
//   double activity(int r) const          a_r . x at x = the current rebuilt x (LDS)
//   static bool kOwnRowActivity           activity(r) only for the lane's own row (r == lane, or 0
//                                         on no-row lanes): its row lives in registers
//   void rebuild(int pass, int k) const   x = (pass 0: x0, else x) + H^-1 A^T w with the
//                                          weights w in RV[0..k) on the rows AC[0..k)
//   static constexpr double kDep          dependent-row threshold on Schur complement / Gamma_pp
//   int dim                               primal dimension (at most dim independent rows)
// and the LDS offsets of five 72-double scratch vectors (VV, LV, RV, WV, AC).
#pragma once
#include "wbq_device.h"

namespace wbq {

// LDS ordering inside the loop (round 6). Every kernel that runs this loop is one wave per workgroup, and the LDS
// unit executes one wave's DS instructions in issue order: a write by one lane is seen by a later read of another
// lane of the same wave without a workgroup barrier, so only the compiler must keep the order. __syncthreads()
// is a workgroup fence on every address space: it waits for all of the wave's outstanding memory accesses
// (s_waitcnt vmcnt(0) lgkmcnt(0)) at each of the loop's ~30 uses. WBQ_GI_WAVE_LDS = 0: __syncthreads() (A/B).
#ifndef WBQ_GI_WAVE_LDS
#define WBQ_GI_WAVE_LDS 1
#endif
__device__ __forceinline__ void gi_sync()
{
#if WBQ_GI_WAVE_LDS
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
#else
    __syncthreads();
#endif
}

// Per-lane vector of active-slot values (T rows, T columns, Gamma columns of the active
// set): in registers (KM static; dynamic writes by select) or one LDS row per lane, whose
// dots load in chunks of 8 independent reads. Either way the loads of a dot issue back to
// back instead of one dependent LDS round trip per term.
template <int KM, bool REG>
struct SlotVec;

template <int KM>
struct SlotVec<KM, true> {
    double v[KM];
    __device__ void bind(double *, int) {}
    __device__ void zero_from(int c)
    {
#pragma unroll
        for (int j = 0; j < KM; ++j) v[j] = (j >= c) ? 0.0 : v[j];
    }
    __device__ void zero_if(bool cond)
    {
#pragma unroll
        for (int j = 0; j < KM; ++j) v[j] = cond ? 0.0 : v[j];
    }
    __device__ void put(int c, bool cond, double x) { v[c] = cond ? x : v[c]; } // c static after unrolling
    __device__ double get(int c) const
    {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < KM; ++j) r = (j == c) ? v[j] : r;
        return r;
    }
    __device__ void put_dyn(int c, bool cond, double x)
    {
#pragma unroll
        for (int j = 0; j < KM; ++j) v[j] = (cond && j == c) ? x : v[j];
    }
    __device__ void load_if(bool cond, const double *src, int cnt)
    {
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const double w = src[j];
            v[j] = (cond && j < cnt) ? w : v[j];
        }
    }
    // after refactor_T: row `row` (this lane's slot row) of T from the LDS factor, or column
    // `row` (col = true); zero past cnt
    __device__ void load_factor(const double *tb, int ts, int row, int cnt, bool col)
    {
        const bool own = row < cnt;
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const double w = tb[col ? j * ts + (own ? row : 0) : (own ? row : 0) * ts + j];
            v[j] = (own && j < cnt && (col ? j >= row : j <= row)) ? w : 0.0;
        }
    }
    __device__ void shift_down(int c, int cnt) // v[j] = v[j + 1] for c <= j < cnt - 1
    {
#pragma unroll
        for (int j = 0; j + 1 < KM; ++j) v[j] = (j >= c && j + 1 < cnt) ? v[j + 1] : v[j];
    }
    __device__ double dot(const double *b, int cnt) const
    {
        double s0 = 0.0, s1 = 0.0; // two accumulators: half the dependent FMA chain
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const double bj = b[j];
            if (j & 1) s1 = fma(j < cnt ? v[j] : 0.0, j < cnt ? bj : 0.0, s1);
            else s0 = fma(j < cnt ? v[j] : 0.0, j < cnt ? bj : 0.0, s0);
        }
        return s0 + s1;
    }
};

template <int KM>
struct SlotVec<KM, false> {
    double *p;
    int cap;
    __device__ void bind(double *row, int capacity)
    {
        p = row;
        cap = capacity;
    }
    __device__ void zero_from(int c)
    {
        for (int j = c; j < cap; ++j) p[j] = 0.0;
    }
    __device__ void zero_if(bool cond)
    {
        if (cond)
            for (int j = 0; j < cap; ++j) p[j] = 0.0;
    }
    __device__ void put(int c, bool cond, double x)
    {
        if (cond) p[c] = x;
    }
    __device__ double get(int c) const { return p[c]; }
    __device__ void put_dyn(int c, bool cond, double x)
    {
        if (cond) p[c] = x;
    }
    __device__ void load_if(bool cond, const double *src, int cnt)
    {
        if (cond)
            for (int j = 0; j < cnt; ++j) p[j] = src[j];
    }
    __device__ void load_factor(const double *, int, int, int, bool) {} // the factor is these rows
    __device__ void shift_down(int c, int cnt)
    {
        for (int j = c; j + 1 < cnt; ++j) p[j] = p[j + 1];
    }
    __device__ double dot(const double *b, int cnt) const
    {
        double s = 0.0, s1 = 0.0;
        for (int c0 = 0; c0 < cnt; c0 += 8) {
            double pv[8], bv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                pv[u] = p[c0 + u];
                bv[u] = b[c0 + u];
            }
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                s = fma(c0 + u < cnt ? pv[u] : 0.0, c0 + u < cnt ? bv[u] : 0.0, s);
                s1 = fma(c0 + u + 1 < cnt ? pv[u + 1] : 0.0, c0 + u + 1 < cnt ? bv[u + 1] : 0.0, s1);
            }
        }
        return s + s1;
    }
};

// value of v in lane `lane` (uniform), as a scalar broadcast (v_readlane, no LDS)
__device__ __forceinline__ double bcast(double v, int lane)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// LDS views with no storage of their own: column a of T read from the T rows (lane a:
// T[c][a] = TT[c TS + a]), and Gamma[j][act_q] gathered from lane j's Gamma row through the
// slot list AC; chunks of 8 independent loads. Their writes are no-ops (the data is in the
// T rows and in Gamma).
struct TColView {
    const double *tt;
    int ts;
    __device__ void bind(const double *col, int stride)
    {
        tt = col;
        ts = stride;
    }
    __device__ void zero_from(int) {}
    __device__ void put(int, bool, double) {}
    __device__ void put_dyn(int, bool, double) {}
    __device__ void load_factor(const double *, int, int, int, bool) {}
    __device__ double dot(const double *b, int cnt) const
    {
        double s = 0.0, s1 = 0.0;
        for (int c0 = 0; c0 < cnt; c0 += 8) {
            double pv[8], bv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                pv[u] = tt[(c0 + u) * ts];
                bv[u] = b[c0 + u];
            }
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                s = fma(c0 + u < cnt ? pv[u] : 0.0, c0 + u < cnt ? bv[u] : 0.0, s);
                s1 = fma(c0 + u + 1 < cnt ? pv[u + 1] : 0.0, c0 + u + 1 < cnt ? bv[u + 1] : 0.0, s1);
            }
        }
        return s + s1;
    }
};

struct GAView {
    const double *grow, *ac;
    __device__ void bind(const double *row, const double *slots)
    {
        grow = row;
        ac = slots;
    }
    __device__ void zero_from(int) {}
    __device__ void put(int, bool, double) {}
    __device__ void put_dyn(int, bool, double) {}
    __device__ void shift_down(int, int) {}
    __device__ double dot(const double *b, int cnt) const
    {
        double s = 0.0, s1 = 0.0;
        for (int q0 = 0; q0 < cnt; q0 += 8) {
            int cq[8];
            double bv[8], gv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                cq[u] = q0 + u < cnt ? (int)ac[q0 + u] : 0;
                bv[u] = b[q0 + u];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) gv[u] = grow[cq[u]];
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                s = fma(q0 + u < cnt ? gv[u] : 0.0, q0 + u < cnt ? bv[u] : 0.0, s);
                s1 = fma(q0 + u + 1 < cnt ? gv[u + 1] : 0.0, q0 + u + 1 < cnt ? bv[u + 1] : 0.0, s1);
            }
        }
        return s + s1;
    }
};

constexpr int kGiRounds = 8; // x rebuilds (each followed by a re-check of every row)
constexpr int kGiPasses = 5; // per rebuild: x from the multipliers, then up to 4 refinement passes
constexpr double kDropPivot = 1e-9; // relative pivot below which a slot is dropped when a rebuild misses

// LDS scratch vectors of the loop (72 doubles each: slot dots read 8 past the active count), and
// where the rebuild re-factors T: rows TB + r * TST (the T rows themselves when they live in LDS,
// else scratch of at least KM rows of KM + 1)
struct GiVecs {
    int VV, LV, RV, WV, AC, TB, TST;
};

// Lane state. Slot a (lane a < k) = the a-th active row: act (its index), sgn (normal =
// sgn * a_act), lam (its multiplier), aeq (an equality: never dropped). Lane j (row j)
// keeps onact = row j is active.
struct GiState {
    int k = 0, act = 0, iters = 0, status = 0, rounds = 0;
    double sgn = 1.0, lam = 0.0;
    bool aeq = false, onact = false;
};

// T = L^-1 of the active-set Gram Gamma_AA (signed normals, slot order) from scratch, into LDS rows
// S[tb + r ts]: a left-looking Cholesky (lane r computes row r of L; one barrier per column), then
// the triangle inverted in place column by column from the last (T[r][c] = -sum_{q>c} T[r][q]
// L[q][c] / L[c][c]). The incremental factor the loop carries (closed-form appends, re-appends after
// a drop) picks up the roundoff of every cancellation d^2 = Gamma_pp - |l|^2; on a nearly dependent
// active set (relative pivots ~1e-11, scripts/emulate_dual_gi.py) it is too poor for the refinement
// of (x, lambda) to converge, the rebuilt x misses an active row, and the slot-drop / re-add cycle
// ends at the rounds cap. A backward-stable factor of the final set is what the refinement needs;
// the loop re-factors only after a rebuild on the incremental factor missed an active row (the
// common path keeps its cost: configs 1 and 2 of the contact form rebuild once, cleanly).
template <class P>
__device__ void refactor_T(const P &pb, double *S, int tb, int ts, int i, int k, const GiState &g)
{
    const bool own = i < k;
#pragma unroll 1
    for (int c = 0; c < k; ++c) {
        const int ac = __shfl(g.act, c);
        const double sc = __shfl(g.sgn, c);
        if (own) S[tb + i * ts + c] = c <= i ? g.sgn * sc * pb.gamma(g.act, ac) : 0.0;
    }
    gi_sync();
    const double *ri = S + tb + (own ? i : 0) * ts;
#pragma unroll 1
    for (int c = 0; c < k; ++c) {
        const double *rc = S + tb + c * ts;
        double s = 0.0;
        if (own && i >= c) {
            double s0 = ri[c], s1 = 0.0;
            int j = 0;
            for (; j + 1 < c; j += 2) {
                s0 = fma(-ri[j], rc[j], s0);
                s1 = fma(-ri[j + 1], rc[j + 1], s1);
            }
            if (j < c) s0 = fma(-ri[j], rc[j], s0);
            s = s0 + s1;
        }
        const double gcc = pb.gamma(__shfl(g.act, c), __shfl(g.act, c));
        const double d = fmax(bcast(s, c), 1e-30 * gcc); // a non-positive pivot: the miss check drops it
        const double il = frsq(d);
        if (own && i >= c) S[tb + i * ts + c] = i == c ? d * il : s * il;
        gi_sync();
    }
#pragma unroll 1
    for (int c = k - 1; c >= 0; --c) {
        const double lcc = S[tb + c * ts + c];
        double acc = 0.0;
        if (own && i > c)
            for (int q = c + 1; q <= i; ++q) acc = fma(ri[q], S[tb + q * ts + c], acc);
        gi_sync();
        if (own && i >= c) S[tb + i * ts + c] = i == c ? 1.0 / lcc : -acc / lcc;
        gi_sync();
    }
}

// Warm start on top of an existing active set (the equalities, already in the slots with their
// multipliers and activities): the inequality rows the previous solve ended with active (wsg = their
// side) are appended one by one with the loop's own closed-form T update (no re-factorisation), then
// one correction of all multipliers, dlambda = T^T T (b_A - s_A) (zero residual on the rows already
// in), makes x the optimum on the enlarged set. Kept only when every appended row is independent and
// every inequality multiplier stays >= 0; otherwise the slots are truncated back and nothing changes.
// It replaced a batch that re-factored the whole set from scratch (refactor_T): 52k of a 200k-cycle
// contact-form block (profiles/r03_diag_contact.log), more than the cold path it saved. A warm start
// changes the path, never the solution (the qpOASES hot-start analogue, SURVEY.md 8b ownership row).
template <int KM, class P, class TrowT, class TcolT, class GAT>
__device__ bool warm_extend(const P &pb, double *S, const GiVecs &V, int i, TrowT &Trow, TcolT &Tcol, GAT &GA,
                            int kind, double lo, double hi, double &s_i, GiState &g, int wsg)
{
    const bool isw = kind == 2 && wsg != 0 && !g.onact;
    unsigned long long m = __ballot(isw);
    const int k0 = g.k, kw = __popcll(m);
    if (kw == 0 || k0 + kw > KM || k0 + kw > pb.dim) return false;
    int k = k0;
    bool ok = true;
    for (int j = 0; j < kw; ++j) {
        const int cp = __ffsll((long long)m) - 1;
        m &= m - 1;
        const double sgp = (double)__shfl(wsg, cp);
        const double gpp = pb.gamma(cp, cp);
        S[V.VV + i] = i < k ? g.sgn * sgp * pb.gamma(g.act, cp) : 0.0;
        S[V.AC + i] = (double)g.act;
        gi_sync();
        const double l = i < k ? Trow.dot(S + V.VV, k) : 0.0;
        S[V.LV + i] = l;
        gi_sync();
        const double r = i < k ? Tcol.dot(S + V.LV, k) : 0.0;
        const double d2 = gpp - isum<64>(l * l);
        if (!(d2 > P::kDep * gpp)) { // dependent on the set: no warm start
            ok = false;
            break;
        }
        const double id = frsq(d2);
        const double tk = i < k ? -r * id : (i == k ? id : 0.0);
        Tcol.put_dyn(k, i <= k, tk);
        GA.put_dyn(k, kind != 0, kind != 0 ? pb.gamma(i, cp) : 0.0);
        S[V.WV + i] = tk;
        gi_sync();
        Trow.load_if(i == k, S + V.WV, k + 1);
        if (i == k) {
            g.act = cp;
            g.sgn = sgp;
            g.aeq = false;
            g.lam = 0.0;
        }
        ++k;
        gi_sync();
    }
    if (ok) { // dlambda = T^T T (b_A - s_A); rows already in have zero residual
        const double lo_a = __shfl(lo, g.act), hi_a = __shfl(hi, g.act), s_a = __shfl(s_i, g.act);
        const double res = (i >= k0 && i < k) ? g.sgn * ((g.sgn > 0.0 ? lo_a : hi_a) - s_a) : 0.0;
        S[V.VV + i] = res;
        S[V.AC + i] = (double)g.act;
        gi_sync();
        const double y = i < k ? Trow.dot(S + V.VV, k) : 0.0;
        S[V.LV + i] = y;
        gi_sync();
        const double dl = i < k ? Tcol.dot(S + V.LV, k) : 0.0;
        const double lam = g.lam + dl;
        const double lmx = imax<64>(i < k ? fabs(lam) : 0.0);
        ok = !(imax<64>((i < k && !g.aeq && lam < -1e-12 * (1.0 + lmx)) ? 1.0 : 0.0) > 0.0);
        if (ok) {
            if (i < k) g.lam = g.aeq ? lam : fmax(lam, 0.0);
            S[V.RV + i] = i < k ? g.sgn * dl : 0.0;
            gi_sync();
            if (kind != 0) s_i += GA.dot(S + V.RV, k);
            if (isw) g.onact = true;
            g.k = k;
            gi_sync();
            return true;
        }
    }
    // truncate back to the k0 slots: the slot state of lanes k0.. returns to its defaults too (every
    // reader masks by g.k, but no rejected row may linger in act / sgn / lam / aeq)
    Trow.zero_if(i >= k0);
    Tcol.zero_from(k0);
    GA.zero_from(k0);
    if (i >= k0) {
        const GiState d0;
        g.act = d0.act;
        g.sgn = d0.sgn;
        g.lam = d0.lam;
        g.aeq = d0.aeq;
    }
    S[V.AC + i] = (double)g.act;
    gi_sync();
    return false;
}

// The side (+1 lower, -1 upper; 0 inactive or an equality slot) with which this lane's row ended
// in the active set: what the next solve of the instance warm-starts from. Every lane calls it.
__device__ __forceinline__ int warm_record(double *S, const GiVecs &V, int i, const GiState &g)
{
    S[V.WV + i] = 0.0;
    gi_sync();
    if (i < g.k && !g.aeq) S[V.WV + g.act] = g.sgn;
    gi_sync();
    const double v = S[V.WV + i];
    gi_sync();
    return v > 0.0 ? 1 : (v < 0.0 ? -1 : 0);
}

// The loop itself (lane i = constraint row i; kind 0 disabled, 1 equality already in the
// active set, 2 a row with limits [lo, hi], lo == hi an equality added when violated).
// Statuses: 1 step cap, 2 no step exists (the rows are inconsistent: infeasible), 3 the slot
// storage overflowed or the rebuilt x misses an active row (a numerically dependent set). On exit with status 0, x in LDS and s_i are exact.
template <int KM, class P, class TrowT, class TcolT, class GAT>
__device__ __forceinline__ void dual_gi(const P &pb, double *S, const GiVecs &V, int i, TrowT &Trow, TcolT &Tcol,
                                        GAT &GA, int kind, double lo, double hi, double nrm, double &s_i, GiState &g,
                                        int maxit)
{
    bool need_select = true, dirty = true, recheck = false;
    bool refac = false; // the next rebuild re-factors T first (after one that missed an active row)
    int cp = 0;
    double sgp = 1.0, bnd = 0.0, lamp = 0.0;
    bool peq = false;
    bool go = g.status == 0;
    int drop = -1; // slot to remove at the top of the next pass (uniform)
    while (go) {
        if (drop >= 0) {
            // remove slot drop from the active set: the slots after it move down, the rows and
            // columns of T before it stand and the ones after it are re-appended
            const int cb = __shfl(g.act, drop);
            if (i == cb) g.onact = false;
            const int na = __shfl(g.act, i + 1);
            const double ns = __shfl(g.sgn, i + 1), nl = __shfl(g.lam, i + 1);
            const bool ne = __shfl(g.aeq ? 1 : 0, i + 1) != 0;
            if (i >= drop) {
                g.act = na;
                g.sgn = ns;
                g.lam = nl;
                g.aeq = ne;
            }
            GA.shift_down(drop, g.k);
            --g.k;
            Trow.zero_if(i >= drop);
            Tcol.zero_from(drop);
            gi_sync();
            for (int a2 = drop; a2 < g.k; ++a2) {
                const int cq = __shfl(g.act, a2);
                const double sq = __shfl(g.sgn, a2);
                S[V.VV + i] = i < a2 ? g.sgn * sq * pb.gamma(g.act, cq) : 0.0;
                gi_sync();
                const double l2 = i < a2 ? Trow.dot(S + V.VV, a2) : 0.0;
                S[V.LV + i] = l2;
                gi_sync();
                const double r2 = i < a2 ? Tcol.dot(S + V.LV, a2) : 0.0;
                const double e2 = pb.gamma(cq, cq) - isum<64>(l2 * l2);
                const double id2 = e2 > 0.0 ? frsq(e2) : 0.0;
                const double tk2 = i < a2 ? -r2 * id2 : (i == a2 ? id2 : 0.0);
                Tcol.put_dyn(a2, i <= a2, tk2);
                S[V.WV + i] = tk2;
                gi_sync();
                Trow.load_if(i == a2, S + V.WV, a2 + 1);
                gi_sync();
            }
            drop = -1;
        }
        if (need_select) {
            double v = -1.0;
            if (kind == 2 && !g.onact) {
                // (an unbounded side, +-kInf -- the one-sided friction faces -- does not scale it)
                const double tol = 1e-10 * fmax(1.0, fmax(fabs(s_i), fmax(fin_abs(lo), fin_abs(hi))));
                const double viol = fmax(lo - s_i, s_i - hi);
                if (viol > tol) v = viol / nrm;
            }
            int pi = i;
            iargmax<64>(v, pi);
            if (!(v > 0.0) || recheck) {
                recheck = false;
                // no violated row: x is current unless steps were taken since the last
                // rebuild; otherwise rebuild x from the multipliers, refine (x, lambda) on the
                // active set, and re-check every row with the exact activities. A re-check
                // that keeps finding rows the incremental activities missed is capped; x is
                // stale then, so that is a failure (status 1), never a silent success.
                if (!dirty) break;
                if (g.rounds >= kGiRounds) {
                    g.status = 1;
                    break;
                }
                ++g.rounds;
                dirty = false;
                if (refac && g.k > 0) { // a backward-stable factor of the final set for the refinement
                    refactor_T(pb, S, V.TB, V.TST, i, g.k, g);
                    Trow.load_factor(S + V.TB, V.TST, i, g.k, false);
                    Tcol.load_factor(S + V.TB, V.TST, i, g.k, true);
                }
                const bool fresh = refac;
                refac = false;
                const double lo_a = __shfl(lo, g.act), hi_a = __shfl(hi, g.act); // all lanes active
                S[V.RV + i] = i < g.k ? g.sgn * g.lam : 0.0;
                S[V.AC + i] = (double)g.act;
                gi_sync();
#pragma unroll 1
                for (int pass = 0; pass < kGiPasses; ++pass) {
                    if (pass > 0) {
                        // residual of the active rows, exact in x-space; correction through T
                        double a_act;
                        if constexpr (P::kOwnRowActivity) { // every lane its own row, slots gather
                            const double a_own = pb.activity(kind != 0 ? i : 0);
                            a_act = __shfl(a_own, g.act);
                        } else {
                            a_act = i < g.k ? pb.activity(g.act) : 0.0;
                        }
                        const double res = i < g.k ? g.sgn * ((g.sgn > 0.0 ? lo_a : hi_a) - a_act) : 0.0;
                        // two refinement passes always; more only while an active row still misses:
                        // a nearly dependent active set gains ~eps cond(Gamma_AA) per pass
                        if (pass > 2 && imax<64>(i < g.k ? fabs(res) / (1.0 + fabs(a_act)) : 0.0) <= 1e-13) break;
                        S[V.VV + i] = res;
                        gi_sync();
                        const double y = Trow.dot(S + V.VV, g.k);
                        S[V.LV + i] = i < g.k ? y : 0.0;
                        gi_sync();
                        const double dl = i < g.k ? Tcol.dot(S + V.LV, g.k) : 0.0;
                        g.lam += dl;
                        S[V.RV + i] = i < g.k ? g.sgn * dl : 0.0;
                        gi_sync();
                    }
                    pb.rebuild(pass, g.k);
                    gi_sync();
                }
                if (kind != 0) s_i = pb.activity(i);
                // the active rows must hold at the rebuilt x; if one does not, T (the factor
                // of a nearly dependent active set) is garbage and so is x: fail loudly
                const double miss = (kind != 0 && g.onact) ? fmin(fabs(s_i - lo), fabs(s_i - hi)) / (1.0 + fabs(s_i)) : 0.0;
                if (imax<64>(miss) > 1e-8) {
                    if (!fresh) { // the incremental factor first: rebuild once more on a fresh one
                        refac = dirty = recheck = true;
                        continue;
                    }
                    // a nearly dependent row added by the loop: drop the slot with the smallest
                    // relative pivot d^2 / Gamma_pp = 1 / (T_aa^2 Gamma_pp) -- an implied row, which
                    // the exact activities of the next rebuild still meet -- and rebuild; the
                    // rounds cap bounds this. No such slot: fail (status 3)
                    const double tdi = Trow.get(i);
                    const int ka = __shfl(kind, g.act);
                    double pv = (i < g.k && ka == 2) ? 1.0 / (tdi * tdi * pb.gamma(g.act, g.act)) : kInf;
                    int blk = i;
                    iargmin<64>(pv, blk);
                    if (pv < kDropPivot) {
                        drop = blk;
                        dirty = true;
                        recheck = true;
                        continue;
                    }
                    g.status = 3;
                    break;
                }
                continue;
            }
            cp = pi;
            const double vl = __shfl(lo - s_i, cp), vh = __shfl(s_i - hi, cp);
            sgp = vl > vh ? 1.0 : -1.0;
            bnd = sgp > 0.0 ? __shfl(lo, cp) : __shfl(hi, cp);
            peq = __shfl(lo == hi ? 1 : 0, cp) != 0;
            lamp = 0.0;
        }
        if (++g.iters > maxit) {
            g.status = 1;
            break;
        }
        // ---- step for row cp: r = Gamma_AA^-1 v, ds = A z (change of every activity)
        const double gpp = pb.gamma(cp, cp);
        S[V.VV + i] = i < g.k ? g.sgn * sgp * pb.gamma(g.act, cp) : 0.0;
        S[V.AC + i] = (double)g.act;
        gi_sync();
        const double l = i < g.k ? Trow.dot(S + V.VV, g.k) : 0.0;
        S[V.LV + i] = l;
        gi_sync();
        const double r = i < g.k ? Tcol.dot(S + V.LV, g.k) : 0.0;
        const double d2 = gpp - isum<64>(l * l);
        S[V.RV + i] = i < g.k ? g.sgn * r : 0.0;
        gi_sync();
        const double gjp = (kind != 0) ? pb.gamma(i, cp) : 0.0;
        const double ds = (kind != 0) ? sgp * gjp - GA.dot(S + V.RV, g.k) : 0.0;
        const double zz = sgp * __shfl(ds, cp);
        const double slack = sgp * (__shfl(s_i, cp) - bnd); // < 0: violated
        const double rmax = imax<64>(i < g.k ? fabs(r) : 0.0);
        double cand = (i < g.k && !g.aeq && r > 1e-13 * rmax) ? g.lam / r : kInf;
        int blk = i;
        iargmin<64>(cand, blk);
        const double t1 = cand;
        // zz is the Schur complement of row cp against the active set, formed by cancellation:
        // its roundoff is ~eps cond(Gamma_AA) gpp, so a row whose complement is below
        // P::kDep gpp is dependent (no primal step), whatever its sign
        // and with k = dim active rows the set spans the primal space: cp is dependent
        const double t2 = (g.k < pb.dim && zz > P::kDep * gpp) ? -slack / zz : kInf;
        if (t1 >= kInf && t2 >= kInf) {
            // no step: the rows cannot all be met -- unless the incremental activities drifted
            // since the last exact rebuild; then rebuild x, re-check every row exactly and select
            // again (the row's partial multiplier is dropped with the rebuild), and report 2 only
            // when the exact activities still leave no step
            if (dirty) {
                recheck = true;
                need_select = true;
                continue;
            }
            g.status = 2;
            break;
        }
        if (t2 <= t1 && g.k >= KM) { // cannot happen for independent rows; guard the storage
            g.status = 3;
            break;
        }
        dirty = true; // a step is taken: the incremental activities drift from the exact ones
        const double t = fmin(t1, t2);
        s_i = fma(t, ds, s_i);
        if (i < g.k) g.lam = fma(-t, r, g.lam);
        lamp += t;
        if (t2 <= t1) { // add cp: T row k = [-(T^T l)^T / d, 1/d]
            const double id = frsq(d2 > 0.0 ? d2 : zz);
            const double tk = i < g.k ? -r * id : (i == g.k ? id : 0.0);
            Tcol.put_dyn(g.k, i <= g.k, tk);
            GA.put_dyn(g.k, kind != 0, gjp);
            S[V.WV + i] = tk;
            gi_sync();
            Trow.load_if(i == g.k, S + V.WV, g.k + 1);
            if (i == g.k) {
                g.act = cp;
                g.sgn = sgp;
                g.lam = lamp;
                g.aeq = peq;
            }
            if (i == cp) g.onact = true;
            ++g.k;
            need_select = true;
            gi_sync();
        } else { // drop slot blk (its multiplier reached zero), keep stepping on cp
            drop = blk;
            need_select = false;
        }
    }
}

}  // namespace wbq
