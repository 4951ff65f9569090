// qppvm_kernel.hip -- batched QPPVM torque solve for gfx950 (MI355X), fp64.
//
// One QP instance per group of NP lanes (NP = 32: two instances per wave64; NP = 64: one),
// lane i <-> joint i. A solve is two (NP = 32) or three launches on one stream, nothing goes back
// to the host:
//
//   qppvm_fast_kernel    every instance: stage -> task forces -> Gauss-Jordan on M ->
//                        equality-constrained optimum -> bound check -> tau. An instance whose
//                        optimum violates a torque bound parks (u, Q1) in scratch (status -1);
//                        one whose level-0 rows are inconsistent (level 0 infeasible at b0)
//                        is marked status -2.
//   qppvm_active_kernel  status -1: Goldfarb-Idnani dual active set on the torque bounds -> tau;
//                        an instance it finds level-0 infeasible is re-marked -2. For NP = 32
//                        this runs inline at the end of the fast kernel instead (its LDS
//                        layout fits in the same budget), saving a launch.
//   qppvm_repair_kernel  status -2: level 0 by BVLS (y*), pins, fresh dual active set -> tau.
// All three use the same instance -> block mapping; blocks without work exit at once.
// Each kernel has its own register budget: the common path stays spill-free, the rare
// ones do not weigh on it.
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
// is the identity, so the dual active set needs no factorisation of H, the bound normals
// are rows of M (given data), and the conditioning is cond(M), not cond(M)^2 as in the
// reference's x-space H1 = M^-2. When level 0 is feasible (y* = b0, the generic case) the
// level-0 optimality constraint A0 x = y* is exactly G u = b0; otherwise the repair kernel
// computes y* and the pinned bounds first (as oracle/wbq_oracle.c:wbq_ref_qppvm_one does).
//
// M must be symmetric (it is read column-wise as rows).
#include "wbq_kernels.h"
#include "wbq_device.h"
#include "qppvm_repair.h"
#include "cs_gi.h"

#include <math.h>
#include <type_traits>

// Fast-kernel schedule switches (round 5; the A/B builds set them, scripts/ab_bench.py):
//   WBQ_FAST_GJ_CH / _UNI  block_gj's trailing-read chunk and one-form update (wbq_device.h)
//   WBQ_FAST_Y_CH          Y = M G^T with the G rows read a chunk of columns ahead (0: as compiled)
//   WBQ_FAST_EQ_EARLY      1: the Gram G G^T (J only) as per-lane outer products summed by DPP and its
//                          factor before M is waited for; after the elimination only res = G (w - u_imp)
//                          (six DPP sums) and the small solves remain. 2: the same sums (Gram and res in
//                          one 27-wide DPP reduction) after the elimination, the factor in registers.
//                          0: LDS dots after the elimination
// (same box, config 1: chunk 4 + one-form update 127.5 -> 131.8 M QP/s, chunk 2 within noise of it; the
// DPP equality block, mode 2, 124.5 alone and 129.3 with them, mode 1 106.9: not kept)
#ifndef WBQ_FAST_GJ_CH
#define WBQ_FAST_GJ_CH 4
#endif
#ifndef WBQ_FAST_GJ_UNI
#define WBQ_FAST_GJ_UNI 1
#endif
#ifndef WBQ_FAST_Y_CH
#define WBQ_FAST_Y_CH 0
#endif
#ifndef WBQ_FAST_EQ_EARLY
#define WBQ_FAST_EQ_EARLY 0
#endif
// Round 6: the n <= 32 fast path (at most two tasks, six level-0 rows) factors M by a streamed left-looking
// block LDL^T that follows M's arrival, instead of the block Gauss-Jordan after all of M (fast_body). 0: the
// Gauss-Jordan path (rounds 1-5), for A/B builds
#ifndef WBQ_FAST_LDL
#define WBQ_FAST_LDL 1
#endif
// Round 6: the n <= 32 inline dual active set carried in constraint space (cs_gi.h: Gamma = M P M columns on
// demand, T = L^-1 of the active Gram in LDS); 0: the u-space loop of rounds 1-5 (gi_solve), for A/B builds
#ifndef WBQ_GI_CS
#define WBQ_GI_CS 1
#endif
// dual active set, n > 32 (T rows in LDS): a dropped bound leaves the basis by Givens rotations (1) or by
// re-projecting the later active normals (0, rounds 1-4; always for n <= 32)
#ifndef WBQ_GI_GIVENS
#define WBQ_GI_GIVENS 1
#endif

namespace wbq {
namespace {

// LDS ordering inside the u-space loop (gi_solve, project_out; round 6): every kernel that runs it is one wave per
// workgroup and the LDS unit executes one wave's DS instructions in issue order, so a compiler fence orders a
// lane's write before another lane's later read; __syncthreads() also waited for every outstanding memory access
// (s_waitcnt vmcnt(0) lgkmcnt(0)) at each of the loop's barriers. WBQ_GS_WAVE_LDS = 0: __syncthreads() (A/B).
#ifndef WBQ_GS_WAVE_LDS
#define WBQ_GS_WAVE_LDS 1
#endif
__device__ __forceinline__ void gs_sync()
{
#if WBQ_GS_WAVE_LDS
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
#else
    __syncthreads();
#endif
}

// Per-instance LDS layouts in doubles (T = ntasks and m0 are launch constants). Rows of
// NP-wide matrices use stride NP+1 so that lane-per-row reads are bank-conflict free.
template <int NP>
struct FastLayout {
    static constexpr int BS = kGjBS; // Gauss-Jordan pivot block
    int JR, PN, RH, U, WV, QD, F, RES, GR, PS, LF, SIZE;
    __host__ __device__ FastLayout(int T, int m0)
    {
        JR = 0;                  // J rows [T*6][NP]
        PN = JR + T * 6 * NP;    // pivot panel, double-buffered [2][NP][BS]
        RH = PN + 2 * NP * BS;   // right-hand sides of the pivot rows [2][BS][8]
        U = RH + 2 * BS * 8;     // u
        WV = U + NP;             // w_t - u_imp [T][NP]
        QD = WV + T * NP;        // qdot
        F = QD + NP;             // task forces [T*6]
        RES = F + 6 * T;         // b0 - G u_imp [m0]
        GR = RES + m0;           // Gram G G^T, lower triangle [m0][kM0Max]
        PS = GR + m0 * kM0Max;   // poses [T][24]
        LF = PS + 24 * T;        // factor of the Gram (WBQ_FAST_EQ_EARLY): packed L, then 1 / diag
        SIZE = (LF + kM0Max * (kM0Max + 1) / 2 + kM0Max + 1) & ~1;
    }
};

// Streamed block LDL^T of the fast path (round 6, NP = 32, at most two tasks and six level-0 rows; see
// fast_body): the left-looking elimination keeps every pivot block's Schur-updated column block ("panel",
// t_j(p), rows 4p.. only) for the later blocks, instead of the Gauss-Jordan's double-buffered panel.
// The stage-only regions (qdot, forces, poses) lie under the panels: they are dead before the first
// panel is written (one wave per workgroup, so LDS program order is the order).
struct LdlLayout {
    static constexpr int NP = 32, BS = kGjBS, NBLK = NP / BS;
    static constexpr int NB = 9;   // forward-substituted columns: 6 rows of G, J_t^T F_t - tau_imp (2), tau_imp
    static constexpr int RHS = 12; // (row stride of the pivot rows' columns)
    static constexpr int PANELS = BS * (NBLK * NP - BS * NBLK * (NBLK - 1) / 2); // sum_p 4 (32 - 4p) = 576
    int JR, QD, F, PS, PL, RH, GR, LF, RES, U, SIZE;
    // panel p starts at PL + pofs(p); row j >= 4p of it at + 4 (j - 4p)
    __host__ __device__ static constexpr int pofs(int p) { return BS * (NP * p - BS * p * (p - 1) / 2); }
    __host__ __device__ LdlLayout(int T, int)
    {
        JR = 0;                  // J rows [T*6][NP]
        QD = JR + T * 6 * NP;    // qdot (stage)
        F = QD + NP;             // task forces [T*6] (stage)
        PS = F + 6 * T;          // poses [T][24] (stage)
        PL = QD;                 // panels (over the stage regions)
        RH = PL + PANELS;        // the pivot rows' forward-substituted columns, double-buffered [2][BS][RHS]
        GR = RH + 2 * BS * RHS;  // Gram G G^T, lower triangle [6][kM0Max]
        LF = GR + 6 * kM0Max;    // its factor: packed L (21), then 1 / diag (6)
        RES = LF + 28;           // b0 - G u_imp [6] (the repair reads it)
        U = RES + 8;             // u
        SIZE = (U + NP + 1) & ~1;
    }
};

// Per-instance LDS of the fast kernel: with MERGED the active-set layout reuses it afterwards
template <int NP, bool MERGED>
struct FastLdsLayout {
    int SIZE;
    __host__ __device__ FastLdsLayout(int T, int m0)
    {
        // (the streamed LDL^T variant's layout, NP = 32, is smaller than the merged active-set layout: checked
        // by launch_np. Not folded in here: a further select in this expression cost the compiler the proof
        // that every instance's LDS is 16-byte aligned, and every 16-byte LDS read fell back to ds_read2_b64 --
        // config 1 32.4 -> 39.6 us on one box)
        const int f = FastLayout<NP>(T, m0).SIZE, g = ActiveLayout<NP>(T, m0).SIZE;
        SIZE = (MERGED && g > f) ? g : f;
    }
};



// lanes that own a joint row of a valid instance store its warm side (ws_rows exists for W1 = I)
__device__ __forceinline__ bool go_rec(bool row, long, const QppvmArgs &a) { return row && a.ws_rows; }

// Orthogonalise the normal held in NV against the rows of Q1T by classical Gram-Schmidt, a second
// pass only where the first lost more than half the norm (|z|^2 <= |n|^2 / 2, "twice is enough":
// after a pass that keeps |z| >= |n| / sqrt(2) the residual is orthogonal to roundoff; the loop's
// normals, rows of M, rarely lean that far into the active span). Rows >= q of Q1T are finite and
// D1[c >= q] = 0, so every loop runs to NP unguarded. Leaves d1 = Q1^T n in D1, |z|^2 in zz (every
// lane of the instance) and returns this lane's entry of z. nn2 = |n|^2; act: the instance takes part
// (the second pass runs for the whole wave when any taking part needs it: barriers stay uniform).
// (Each pass is two LDS dot products per lane: with eight waves per CU in this loop the LDS port is
// the bound, and the second pass was half of it.)
// sum_{j < cnt} a[j stride] b[j] with a wave-uniform bound (rounded up to chunks of eight reads issued together;
// the entries past cnt are zero in the callers' data, so no masks): NP = 64 only, where one instance is the wave
__device__ __forceinline__ double dotw(const double *a, int stride, const double *b, int cnt)
{
    double s0 = 0.0, s1 = 0.0;
    for (int j0 = 0; j0 < cnt; j0 += 8) {
        double av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            av[u] = a[(j0 + u) * stride];
            bv[u] = b[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            s0 = fma(av[u], bv[u], s0);
            s1 = fma(av[u + 1], bv[u + 1], s1);
        }
    }
    return s0 + s1;
}

template <int NP>
__device__ __forceinline__ double project_out(double *S, const ActiveLayout<NP> &L, double npj, int q, int i,
                                              double nn2, bool act, double &zz, int n = NP)
{
    constexpr int RS = NP + 1;
    // (measured, round 6: the LDS reads of these dots issued a chunk ahead -- dot4p / dot4sp, wbq_device.h --
    // spilled the n <= 32 fast kernel that inlines this loop, 0 -> ~300 B of scratch even at 4-element chunks)
    // NP = 64 (one instance per wave, q and n wave-uniform): a basis row past n and D1 past q are zero, so the dots
    // stop there (n = 39: 40 of 64 entries; q = m0 + k rows of Q1^T) instead of running to NP
    const int nq = NP == 64 ? (q + 7) & ~7 : NP, nn = NP == 64 ? (n + 7) & ~7 : NP;
    double d1 = 0.0;
    if constexpr (NP == 64) d1 = i < q ? dotw(S + L.QA + i * RS, 1, S + L.NV, nn) : 0.0;
    else d1 = i < q ? dot4<NP>(S + L.QA + i * RS, S + L.NV) : 0.0;
    S[L.D1 + i] = d1;
    gs_sync();
    double z;
    if constexpr (NP == 64) z = npj - dotw(S + L.QA + i, RS, S + L.D1, nq);
    else z = npj - dot4s<NP>(S + L.QA + i, RS, S + L.D1);
    zz = isum<NP>(z * z);
    if (__any(act && !(zz > 0.5 * nn2))) {
        S[L.BC + i] = z;
        gs_sync();
        double d1b;
        if constexpr (NP == 64) d1b = i < q ? dotw(S + L.QA + i * RS, 1, S + L.BC, nn) : 0.0;
        else d1b = i < q ? dot4<NP>(S + L.QA + i * RS, S + L.BC) : 0.0;
        S[L.D1B + i] = d1b;
        gs_sync();
        if constexpr (NP == 64) z -= dotw(S + L.QA + i, RS, S + L.D1B, nq);
        else z -= dot4s<NP>(S + L.QA + i, RS, S + L.D1B);
        S[L.D1 + i] = d1 + d1b;
        zz = isum<NP>(z * z);
        gs_sync();
    }
    return z;
}


// ============================================================== active-set path
// Goldfarb-Idnani dual active set on the torque bounds (QPPVMPlugin.cpp:203-205 limits) in
// u-space, for the instances with go set, starting from u_i (the equality-constrained
// optimum) with the Q1 rows in LDS (QA rows < m0, the others zero). Pinned or equal limits
// (lo == hi) act as equalities and are never dropped. Returns this lane's x = M u; sets
// infeasible when no step exists (then level 0 is not attainable at b0: y* != b0).
// Warm start (the qpOASES hot-start analogue): wsg = the side (+1 lower, -1 upper) on
// which this lane's bound ended active in the instance's last solve. Those bounds enter the active
// set in one batch (slot order = joint order): Gram-Schmidt of their normals against Q1, T = R^-1,
// the step to the batch's equality-constrained optimum u += Q_W w with w = T^T r (r = the bounds'
// residuals) and the multipliers lambda = T w. The batch is kept only if it is independent and dual
// feasible (lambda >= 0 but on equality bounds); the loop then continues from it as from any of its
// own states, else it starts cold. It changes the path, never the solution. With record set, the
// final active set goes to ws_rows (status 0).
// (LAPB / LAPC: stamp slots of the diagnostic build's lap counters of this call site, 8 phases from LAPB
// and 2 counts from LAPC; 0: none)
template <int NP, int M0, int LAPB = 0, int LAPC = 0>
__device__ __forceinline__ double gi_solve(const QppvmArgs &a, double *S, long b, int i, bool row, bool go,
                                           double lo, double hi, double u_i, int &status, int &iters,
                                           bool &infeasible, int wsg = 0, bool record = false, int handoff = 0,
                                           bool skipdep = false)
{
    constexpr int RS = NP + 1;
    constexpr bool MREG = ActiveLayout<NP>::MREG;
    // (the Givens drop with T rows in LDS only: in the NP = 32 merged kernel, T in registers, its
    // temporaries spilled the fast path, 0 -> 428 B)
    constexpr bool kGivens = WBQ_GI_GIVENS != 0 && !MREG;
    const int n = a.n, m0 = a.m0;
    const ActiveLayout<NP> L(a.ntasks, m0, n);
    const int ic = i < n ? i : n - 1;
    const bool lrow = i < L.NR; // (NP = 64: a lane past the layout's rows reads the zero row, writes nothing)
    WBQ_LAP_INIT; // (diagnostic build: cycles per phase of the loop, stamp slots 20-27, counts 13-14)
    // M rows (columns, coalesced); 64-bit addressing: the instances of a wave come from a work
    // list here, so no wave-uniform base exists for a buffer resource
    const double *Mb = a.M + b * n * n + ic;
    RowStore<NP, MREG> Mr;
    Mr.bind(lrow ? S + L.MA + i * RS : S + L.ZR, lrow);
    if constexpr (!MREG) {
        S[L.ZR + i] = 0.0;
        if (i == 0) S[L.ZR + NP] = 0.0;
    }
    double mrow[NP];
#pragma unroll
    for (int r = 0; r < NP; ++r) mrow[r] = Mb[(r < n ? r : n - 1) * n];
#pragma unroll
    for (int r = 0; r < NP; ++r) mrow[r] = (row && r < n) ? mrow[r] : (r == i ? 1.0 : 0.0);
    if constexpr (MREG) {
#pragma unroll
        for (int r = 0; r < NP; ++r) Mr.v[r] = mrow[r];
    } else {
        if (lrow)
#pragma unroll
            for (int r = 0; r < NP; ++r) S[L.MA + i * RS + r] = mrow[r];
    }
    double nrm2 = 0.0;
#pragma unroll
    for (int j = 0; j < NP; ++j) nrm2 = fma(mrow[j], mrow[j], nrm2);
    const double nrm = sqrt(nrm2);
    S[L.D1 + NP + i] = 0.0;
    S[L.U + i] = u_i;
    RowStore<NP, MREG> Tr;
    Tr.bind(lrow ? S + L.TT + i * RS : S + L.ZR, lrow);
    Tr.zero();
    int k = 0, q = m0;
    int act_p = -1, act_s = 0; // lane a < k: active inequality a (row index, sign)
    bool act_e = false;        // lane a < k: that constraint is an equality (lo == hi)
    double lam = 0.0;          // lane a < k: its multiplier
    int p = 0, sg = 1;
    double lamp = 0.0;
    bool need_select = true;
    const int maxit = a.max_iter;
    const bool eqb = lo == hi;
    infeasible = false;
    gs_sync();
    WBQ_LAP(0);
    if (__any(go && row && wsg != 0)) {
        // ------------------------------------------------ warm start: the last active set in one batch
        const bool wme = go && row && wsg != 0;
        const unsigned long long bal = __ballot(wme);
        const int base = (int)(threadIdx.x & (64 - NP)); // first lane of this instance in the wave
        const unsigned long long mi = NP == 64 ? bal : ((bal >> base) & 0xffffffffull);
        const int kw = __popcll(mi);
        if (wme) S[L.BC + __popcll(mi & ((1ull << i) - 1ull))] = (double)i; // slot -> joint
        int kwmax = kw;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) kwmax = max(kwmax, __shfl_xor(kwmax, m, 64));
        gs_sync();
        const int myp0 = i < kw ? (int)S[L.BC + i] : 0; // the a-th warm bound's joint on lane a
        bool dep = false;
        // skipdep (warm sets from a level-0 repair: its BVLS bound set holds the pins, dependent on G u = y* by
        // construction): a dependent member is left out of the batch instead of rejecting it -- it is implied by
        // the others, so it holds at the batch optimum. Else a dependent member sends the batch cold.
        int kk = 0, myp = 0; // members kept (instance-uniform), this slot lane's joint
        for (int a2 = 0; a2 < kwmax; ++a2) {
            const bool on = a2 < kw;
            const int pa = on ? __shfl(myp0, a2, NP) : 0; // (project_out overwrites BC)
            const int sa = __shfl(wsg, pa, NP);
            const double nj = on ? sa * Mr.get(pa) : 0.0;
            S[L.NV + i] = nj;
            gs_sync();
            const double npn = __shfl(nrm, pa, NP);
            double zzr;
            const double zr = project_out<NP>(S, L, nj, on ? q : 0, i, npn * npn, on, zzr, n);
            const bool indep = zzr > 1e-16 * npn * npn;
            if (on && !indep && !skipdep) dep = true; // a dependent batch: start cold
            if (on && (indep || !skipdep) && q >= L.NR) dep = true; // (the basis rows the layout holds: cold)
            const bool add = on && (indep || !skipdep) && q < L.NR;
            double rr2 = 0.0;
            if (add && i < kk) rr2 = Tr.dot(S + L.D1 + m0, NP == 64 ? kk : NP);
            if (add) {
                const double iz = zzr > 0.0 ? frsq(zzr) : 0.0;
                S[L.QA + q * (NP + 1) + i] = zr * iz;
                if (i < kk) Tr.set(kk, -rr2 * iz);
                if (i == kk) {
                    Tr.set(kk, iz);
                    myp = pa;
                }
                ++q;
                ++kk;
            }
            gs_sync();
        }
        int kkmax = kk;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) kkmax = max(kkmax, __shfl_xor(kkmax, m, 64));
        WBQ_LAP(1);
        // residuals r_a = beta_a - n_a . u on the slot lanes, w = T^T r (lane j: w_j), lambda = T w
        const double s0 = Mr.dot(S + L.U, NP == 64 ? n : NP);
        const double xp = __shfl(s0, myp, NP), lop = __shfl(lo, myp, NP), hip = __shfl(hi, myp, NP);
        const int sp = __shfl(wsg, myp, NP);
        const double r = i < kk ? (sp > 0 ? lop - xp : xp - hip) : 0.0; // sgn (bound - x)
        double w_own = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            if (j < kkmax) {
                const double t = isum<NP>(i < kk ? Tr.at(j) * r : 0.0);
                w_own = i == j ? t : w_own;
            }
        }
        S[L.BC + i] = i < kk ? w_own : 0.0;
        gs_sync();
        const double lw = i < kk ? Tr.dot(S + L.BC, NP == 64 ? kk : NP) : 0.0;
        const bool peqw = __shfl(eqb ? 1 : 0, myp, NP) != 0;
        const double lmx = imax<NP>(fabs(lw));
        dep |= imax<NP>((i < kk && !peqw && lw < -1e-12 * (1.0 + lmx)) ? 1.0 : 0.0) > 0.0;
        dep = imax<NP>(dep ? 1.0 : 0.0) > 0.0; // instance-uniform
        if (kk > 0 && !dep) { // keep: step to the batch optimum, slots take the batch
            double du = 0.0;
            for (int c = 0; c < kkmax; ++c)
                if (c < kk) du = fma(S[L.QA + (m0 + c) * (NP + 1) + i], S[L.BC + c], du);
            u_i += du;
            if (i < kk) {
                act_p = myp;
                act_s = sp;
                act_e = peqw;
                lam = peqw ? lw : fmax(lw, 0.0);
            }
            k = kk;
            iters += 1;
        } else { // cold: drop the batch (rows of Q1 past m0 and T are rewritten before they are read)
            Tr.zero();
            q = m0;
        }
        gs_sync();
        S[L.U + i] = u_i;
        gs_sync();
        WBQ_LAP(2);
    }
    while (true) {
        const double s_i = Mr.dot(S + L.U, NP == 64 ? n : NP); // s = M u = x
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
            // (p is instance-uniform: v_readlane broadcasts, no ds_bpermute round trips)
            sg = (cs_bcast<NP>(lo - s_i, p) > cs_bcast<NP>(s_i - hi, p)) ? 1 : -1;
            lamp = 0.0;
        }
        if (!__any(go)) break;
        WBQ_LAP_ADD(0, 1);
        const double s_p = cs_bcast<NP>(s_i, p);
        const double sp = sg > 0 ? s_p - cs_bcast<NP>(lo, p) : cs_bcast<NP>(hi, p) - s_p; // slack < 0
        const double npn = cs_bcast<NP>(nrm, p);
        const bool peq = cs_bcast_i<NP>(eqb ? 1 : 0, p) != 0;
        const double npj = sg * Mr.get(p); // n_p = sg * M row p (M symmetric)
        S[L.NV + i] = npj;
        gs_sync();
        WBQ_LAP(3);
        double zz;
        const double z = project_out<NP>(S, L, npj, q, i, npn * npn, go, zz, n);
        WBQ_LAP(4);
        double ra = 0.0;
        if (i < k) ra = Tr.dot(S + L.D1 + m0, NP == 64 ? k : NP);
        const double rmax = imax<NP>(fabs(ra));
        // equality rows (pinned or lo == hi) are never dropped
        double cand = (i < k && !act_e && ra > 1e-13 * rmax) ? lam / ra : kInf;
        int ci = i;
        iargmin<NP>(cand, ci);
        const double t1 = cand;
        // (q < NR: the basis has at most n rows; a candidate past the layout's rows is treated as dependent)
        const double t2 = (zz > 1e-20 * npn * npn && q < L.NR) ? -sp / zz : kInf;
        bool rebuild = false;
        int cdrop = 0;
        if (go && t1 >= kInf && t2 >= kInf) {
            // infeasible: level 0 is not attainable at b0 inside the bounds (y* != b0)
            infeasible = true;
            go = false;
        }
        if (go) {
            const double t = fmin(t1, t2);
            if (i < k) lam = fma(-t, ra, lam);
            lamp += t;
            if (t2 < kInf) u_i = fma(t, z, u_i);
            ++iters;
            if (t2 <= t1) { // add p
                const double iz = frsq(zz);
                S[L.QA + q * RS + i] = z * iz;
                if (i < k) Tr.set(k, -ra * iz);
                if (i == k) {
                    Tr.zero();
                    Tr.set(k, iz);
                    act_p = p;
                    act_s = sg;
                    act_e = peq;
                    lam = lamp;
                }
                ++k;
                ++q;
                need_select = true;
            } else { // drop ci (its multiplier hit zero), keep p
                const int nap = __shfl(act_p, i + 1, NP);
                const int nas = __shfl(act_s, i + 1, NP);
                const bool nae = __shfl(act_e ? 1 : 0, i + 1, NP) != 0;
                const double nlam = __shfl(lam, i + 1, NP);
                if (i >= ci) {
                    act_p = nap;
                    act_s = nas;
                    act_e = nae;
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
            // handoff > 0: a loop still running after that many steps goes to the level-0 repair as if
            // infeasible (its BVLS settles level 0 first; a feasible instance comes back unpinned, so the
            // result is the same)
            if (handoff > 0 && iters >= handoff && go) {
                infeasible = true;
                go = false;
            }
        }
        S[L.U + i] = u_i;
        gs_sync();
        WBQ_LAP(5);
        if (__any(rebuild)) {
          if constexpr (kGivens) {
            // Drop slot c by a QR downdate. With the active normals N = Q^T R (Q: the basis rows m0.. of
            // Q1T, R = T^-1), deleting column c of R leaves it upper Hessenberg from c; the plane rotations
            // G_c .. G_{k-1} that restore the triangle are the ones that carry row c of T onto e_k
            // (G^T e_k spans the left null space of R without column c, which is row c of T), so they are
            // found from T alone by a chase down that row. Then Q <- G Q (its last row leaves the basis),
            // T <- (T without row c) G^T (its last column drops out): two LDS rows and two entries per lane
            // per rotation, where re-projecting every later normal cost two to four LDS dot products each
            // (the stress plant's n = 39 dual loops spent ~60 % of their cycles there, scripts/diag_plugin_tick.py).
            const int kold = k + 1; // (the drop above decremented k)
            // (one instance per wave here: kold and cdrop are wave-uniform, and T's entries past kold are zero, so
            // the row copies below stop at kold -- they ran over all 64 columns, ~24k cycles per drop in the
            // stress plant's hand-back loop, profiles/r06_v14_diag_tick_stress.log)
            if (rebuild && i == cdrop) {
#pragma unroll
                for (int j = 0; j < NP; ++j)
                    if (j < kold) S[L.BC + j] = Tr.at(j); // row c of T, every lane reads it
            }
            gs_sync();
            double xr = rebuild ? S[L.BC + cdrop] : 0.0; // the chase's running entry
#pragma unroll
            for (int j = 0; j + 1 < NP; ++j) {
                const bool on = rebuild && j >= cdrop && j + 1 < kold;
                if (__any(on)) {
                    const double xn = S[L.BC + j + 1];
                    const double h = sqrt(fma(xr, xr, xn * xn));
                    const double ih = h > 0.0 ? 1.0 / h : 0.0;
                    const double cs = h > 0.0 ? xn * ih : 1.0, sn = h > 0.0 ? -xr * ih : 0.0;
                    if (on) {
                        const double t0 = Tr.at(j), t1 = Tr.at(j + 1);
                        Tr.set(j, fma(cs, t0, sn * t1));
                        Tr.set(j + 1, fma(-sn, t0, cs * t1));
                        double *q0 = S + L.QA + (m0 + j) * RS + i;
                        const double a0 = q0[0], a1 = q0[RS];
                        q0[0] = fma(cs, a0, sn * a1);
                        q0[RS] = fma(-sn, a0, cs * a1);
                        xr = h;
                    }
                }
            }
            // rows c.. of T move up one slot (the multipliers and slot rows did above)
            const int nxt = i + 1 < NP ? i + 1 : i;
            {
                double nrow[NP];
                const int kw = cs_wmax<NP>(rebuild ? kold : 0);
#pragma unroll
                for (int j = 0; j < NP; ++j) nrow[j] = j < kw ? __shfl(Tr.at(j), nxt, NP) : 0.0;
                gs_sync(); // (T rows in LDS: every read of row i + 1 before its owner writes it)
#pragma unroll
                for (int j = 0; j < NP; ++j) {
                    if (j < kw) {
                        double v = (rebuild && i >= cdrop) ? nrow[j] : Tr.at(j);
                        if (rebuild && (j >= k || i >= k)) v = 0.0; // the last column and the dead rows
                        if (rebuild) Tr.set(j, v);
                    }
                }
            }
            if (rebuild) q = m0 + k;
            gs_sync();
            WBQ_LAP_ADD(1, 1);
          } else {
            // Re-factor the inequality directions from the dropped position on: Q1T rows
            // m0+cdrop.. and T columns cdrop.. (Gram-Schmidt is sequential, earlier ones stand).
            if (rebuild) {
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
                gs_sync();
                const double npa = __shfl(nrm, pa, NP);
                double zzr;
                const double zr = project_out<NP>(S, L, nj, on ? q : 0, i, npa * npa, on, zzr, n);
                double rr2 = 0.0;
                if (on && i < a2) rr2 = Tr.dot(S + L.D1 + m0, NP == 64 ? a2 : NP);
                if (on) {
                    const double iz = frsq(zzr);
                    S[L.QA + q * RS + i] = zr * iz;
                    if (i < a2) Tr.set(a2, -rr2 * iz);
                    if (i == a2) Tr.set(a2, iz);
                    ++q;
                }
                gs_sync();
                WBQ_LAP_ADD(1, 1);
            }
          }
            WBQ_LAP(6);
        }
    }
    WBQ_LAP(3); // (the last pass: select only)
    if (record) { // the final active set, by joint, for the next solve of this instance
        S[L.NV + i] = 0.0;
        gs_sync();
        if (i < k && !act_e) S[L.NV + act_p] = (double)act_s;
        gs_sync();
        const double sgn = S[L.NV + i];
        const bool ok = status == 0 && !infeasible;
        if (go_rec(row, b, a)) a.ws_rows[b * 64 + i] = (signed char)(ok ? (sgn > 0.0 ? 1 : (sgn < 0.0 ? -1 : 0)) : 0);
        gs_sync();
    }
    const double xf = Mr.dot(S + L.U, NP == 64 ? n : NP);
    WBQ_LAP(7);
    if constexpr (LAPB > 0) WBQ_LAP_FLUSH(LAPB, LAPC);
    return xf;
}

// Active-set kernel (NP = 64; NP = 32 runs it inline in the fast kernel): instances parked
// with status -1. An instance whose active set finds level 0 infeasible is handed on to the
// repair kernel with status -2.
// PIN (NP = 64): the hand-back pass after the repair kernel -- work list 2, the instances' pinned limits
// from lo_scr / hi_scr, warm from the BVLS bound set; "no step" there is status 2, as in the repair kernel.
template <int NP, int M0, bool PIN = false>
__global__ __launch_bounds__(64, NP == 32 ? 2 : 1) void qppvm_active_kernel(const QppvmArgs a)
{
    constexpr int IPW = kWave / NP;
    constexpr int RS = NP + 1;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const ActiveLayout<NP> L(a.ntasks, a.m0, a.n); // (rows sized by n: launch_one's kNSized)
    const int sub = threadIdx.x / NP;
    const int i = threadIdx.x - sub * NP;
    double *S = smem + sub * L.SIZE;
    const int cnt = PIN ? a.work[4 + a.epoch] : a.work[a.epoch * 2]; // instances parked in this solve
    for (long e0 = (long)blockIdx.x * IPW; e0 < cnt; e0 += (long)gridDim.x * IPW) {
        const long e = e0 + sub;
        const bool valid = e < cnt;
        WBQ_STAMP(4);
        WBQ_RTSTAMP(PIN ? 42 : 30); // (diagnostic: the hand-back pass keeps its own realtime slots, 42-43)
        const long b = valid ? a.wl[(PIN ? 2 * a.B : 0) + e] : 0;
        const int n = a.n;
        const bool row = valid && i < n;
        const double h_i = row ? a.h[b * n + i] : 0.0;
        double lo = -kInf, hi = kInf;
        if constexpr (PIN) {
            if (row) {
                lo = a.lo_scr[b * NP + i];
                hi = a.hi_scr[b * NP + i];
            }
        } else {
            if (row) torque_box(a, i, a.q[b * n + i], a.qd[b * n + i], h_i, lo, hi);
        }
        const double *qs = a.q1_scr + b * kM0Max * NP;
        __syncthreads(); // the previous instance's LDS is dead
#pragma unroll
        for (int c = 0; c < NP; ++c)
            if (c < L.NR) S[L.QA + c * RS + i] = (valid && c < M0 && c < a.m0) ? qs[(c < M0 ? c : 0) * NP + i] : 0.0;
        int status = 0, iters = 0;
        bool infeasible = false;
        WBQ_STAMP(6);
        const bool warm_gi = valid && (PIN || (a.ws_hint[b] & 2));
        const int wsg = (warm_gi && row) ? (int)a.ws_rows[b * 64 + i] : 0;
        // (round 6: the constraint-space loop of cs_gi.h at 64 lanes here -- Gamma columns over n <= 64 rows, T = L^-1
        // over the QA region, a hand-off to this u-space loop -- ended 3 of 96 heavily saturated n = 39 instances of
        // tests/test_gpu_handback.py at the step cap (4 n + 32) where this loop converges: not used for n > 32)
        const double x_i = gi_solve<NP, M0, PIN ? 48 : 32, PIN ? 56 : 40>(a, S, b, i, row, valid, lo, hi,
                                                                        valid ? a.u_scr[b * NP + i] : 0.0, status,
                                                                        iters, infeasible, wsg, true,
                                                                        PIN ? 0 : a.gi_handoff, PIN);
        if constexpr (PIN) { // (the repair kernel's epilogue)
            if (infeasible && status == 0) status = 2;
            double tau_i = x_i + h_i;
            if (imax<NP>((row && !isfinite(tau_i)) ? 1.0 : 0.0) > 0.0 && status == 0) status = 3;
            if (status != 0) tau_i = h_i;
            if (row) a.tau[b * n + i] = tau_i;
            rollout_step(a, b, i, row, S[L.U + i], status == 0);
            if (valid && i == 0) {
                a.status[b] = status;
                a.iters[b] += iters;
                a.ws_hint[b] = (a.ws_hint[b] & 1) | (status == 0 ? 2 : 0);
            }
        } else if (infeasible) {
            if (valid && i == 0) {
                a.status[b] = -2; // level-0 repair kernel
                wl_push(a, 1, b);
            }
        } else {
            double tau_i = x_i + h_i;
            if (imax<NP>((row && !isfinite(tau_i)) ? 1.0 : 0.0) > 0.0 && status == 0) status = 3;
            if (status != 0) tau_i = h_i; // "SOLVER ERROR!" fallback: tau_qp = 0 (:246-249)
            if (row) a.tau[b * n + i] = tau_i;
            rollout_step(a, b, i, row, S[L.U + i], status == 0); // qdd = M^-1 x = u
            if (valid && i == 0) {
                a.status[b] = status;
                a.iters[b] = iters;
                a.ws_hint[b] = status == 0 ? 2 : 0; // ws_rows now holds this solve's active set
            }
        }
        WBQ_STAMP(7);
        WBQ_RTSTAMP(PIN ? 43 : 31);
    }
}

// u = M^-1 x (lane i: x_i in, u_i out; lanes with row unset carry identity rows): block
// Gauss-Jordan on M's rows reloaded from HBM/L2, the QA region as its panel scratch (rare path)
template <int NP>
__device__ double minv_apply(const QppvmArgs &a, double *S, const ActiveLayout<NP> &L, long b, int i, bool row, double x)
{
    const int n = a.n;
    const int ic = i < n ? i : n - 1;
    double rhs[1] = {row ? x : 0.0};
    __syncthreads();
    minv_rows<NP, 1>(a.M + b * n * n + ic, n, i, row, rhs, S + L.QA, S + L.QA + 2 * kGjBS * NP);
    return rhs[0];
}

// Level-0 repair of one instance (the lanes with rep set; every lane of the wave calls it):
// y* by BVLS, the pins, and a fresh dual active set (or, when the pinned level-0 point is the
// only feasible one, that point) -> tau, status, iters, warm-start hint. S is the instance's
// active-set LDS.
template <int NP, int M0>
__device__ __forceinline__ void repair_instance(const QppvmArgs &a, double *S, long b, int i, bool rep)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int n = a.n;
    const bool row = rep && i < n;
    const double h_i = row ? a.h[b * n + i] : 0.0;
    const bool warm = rep && (a.ws_hint[b] & 1); // bit 0: the last solve went through this repair
    double lo = -kInf, hi = kInf;
    if (row) torque_box(a, i, a.q[b * n + i], a.qd[b * n + i], h_i, lo, hi);
    const RepairOut ro = level0_repair<NP, M0>(a, (int)(S - smem), b, i, rep, lo, hi, warm);
    WBQ_STAMP(11);
    int status = ro.status, iters = 0;
    bool infeasible = false;
    // level 1 over a single feasible point needs no active set: x = x*. (The active set on that
    // point is degenerate by construction -- the pins and G u = y* are dependent -- and could end
    // with "no step", status 2: the config-4 rollouts once did, scripts/diag_mpc.py.)
    const bool uniq = ro.unique;
    const ActiveLayout<NP> L(a.ntasks, a.m0, n); // (gi_solve's layout: u at L.U)
    double x_i = ro.x;
    // the dual active set starts from the BVLS point's bound set in one batch (gi_solve's warm start:
    // kept only if independent and dual feasible, else cold; the path changes, never the solution). The
    // level-1 optimum keeps level 0 at y*, so its active bounds are mostly those BVLS ended on: a config-4
    // rollout's repaired instance-steps took up to ~90 cold steps (scripts/diag_mpc_steps.py)
    const int wsr = (row && !uniq) ? -ro.st : 0; // gi_solve's sides: +1 lower, -1 upper
    if constexpr (NP == 64) {
        // hand the pinned level 1 to the active-set pass over work list 2 (qppvm_active_kernel<..., true>):
        // the dual loop there runs ~2x faster per step than here, where it shares the BVLS's frame
        // (scripts/diag_plugin_tick.py, stress plant: ~39k vs ~19k cycles per step)
        if (a.handback && rep && ro.status == 0 && !uniq) { // (one instance per wave: wave-uniform)
            if (row) {
                a.lo_scr[b * NP + i] = ro.lo;
                a.hi_scr[b * NP + i] = ro.hi;
            }
            a.u_scr[b * NP + i] = ro.u;
#pragma unroll
            for (int c = 0; c < M0; ++c)
                if (c < a.m0) a.q1_scr[(b * kM0Max + c) * NP + i] = S[L.QA + c * (NP + 1) + i];
            a.ws_rows[b * 64 + i] = (signed char)(row ? wsr : 0);
            if (i == 0) {
                a.status[b] = -1;
                a.iters[b] = ro.it;
                a.ws_hint[b] = ro.l0inf ? 1 : 0;
                wl_push(a, 2, b);
            }
            return;
        }
    }
    if (__any(rep && !uniq)) {
        const bool g1 = rep && status == 0 && !uniq;
        if constexpr (NP == 32 && WBQ_GI_CS != 0) {
            // the pinned level 1 by the constraint-space loop (cs_gi.h); a hand-off there takes the u-space loop
            bool bail;
            double uo;
            const double vnone[M0] = {};
            x_i = cs_solve<NP, M0, 48, 56, false>(a, S, b, i, row, g1, ro.lo, ro.hi, ro.u, status, iters, infeasible, wsr,
                                              true, uo, vnone, bail);
            if (__any(bail)) {
                int st3 = 0, it3 = 0;
                bool inf3 = false;
                const double x3 = gi_solve<NP, M0>(a, S, b, i, row && bail, bail, ro.lo, ro.hi, ro.u, st3, it3, inf3, wsr,
                                                   true, 0, true);
                if (bail) {
                    x_i = x3;
                    status = st3;
                    iters += it3;
                    infeasible = inf3;
                }
            }
            __syncthreads();
            if (!bail) S[L.U + i] = uo; // (rollout_step below reads u there; gi_solve wrote every lane's)
            __syncthreads();
        } else {
            x_i = gi_solve<NP, M0, 48, 56>(a, S, b, i, row, g1, ro.lo, ro.hi, ro.u, status, iters, infeasible, wsr, true, 0,
                                           true);
        }
    }
    if (uniq) x_i = ro.x;
    if (a.integrate && __any(rep && uniq)) { // rollouts integrate qdd = u = M^-1 x*
        const bool r2 = row && uniq;
        const double u2 = minv_apply<NP>(a, S, L, b, i, r2, ro.x);
        if (rep && uniq) S[L.U + i] = u2;
        __syncthreads();
    }
    WBQ_STAMP(12);
#ifdef WBQ_STAMPS
    if (threadIdx.x == 0 && a.stamps) { // step counts of the diagnostic build
        a.stamps[blockIdx.x * kStamps + 13] = (unsigned long long)ro.it;
        a.stamps[blockIdx.x * kStamps + 14] = (unsigned long long)iters;
    }
#endif
    if (infeasible && status == 0) status = 2;
    double tau_i = x_i + h_i;
    if (imax<NP>((row && !isfinite(tau_i)) ? 1.0 : 0.0) > 0.0 && status == 0) status = 3;
    if (status != 0) tau_i = h_i; // "SOLVER ERROR!" fallback: tau_qp = 0 (:246-249)
    if (row) a.tau[b * n + i] = tau_i;
    rollout_step(a, b, i, row, S[L.U + i], status == 0);
    if (rep && (i & (NP - 1)) == 0) {
        a.status[b] = status;
        a.iters[b] = iters + ro.it;
        // bit 1: ws_rows holds this solve's final bound set (the dual active set ran and ended well)
        a.ws_hint[b] = (ro.l0inf ? 1 : 0) | ((!uniq && status == 0) ? 2 : 0);
    }
}

// Level-0 repair kernel: instances with status -2 (flagged by the fast kernel, or by
// the active-set kernel) get y* by BVLS, their pins, and a fresh dual active set. The work itself
// is a separate (noinline) function, so the kernel's entry is only the count read, the counter
// reset and the exit. Measured (r03): with nothing to repair the launch adds ~1-1.5 us to a config-1
// step (A/B with the body compiled out: 36.3 -> 35.4 us; scripts/gpu_ab_empty.sh), the launch
// overhead of any follow-up kernel (scripts/launch_probe2.hip, launch_probe3.hip: registers, LDS,
// scratch, kernarg size and a cold L2 do not change it); rocprofv3's ~5 us duration for it includes
// the dispatch.
// The fused rollout's level-0 repair behind a call (WBQ_ROLL_REPAIR_NOINLINE = 1; round 5's default): the step's
// fast path then keeps more of its registers (round 5, same box: WRITE_SIZE per 20-step launch 730 -> 156 MB).
// Round 4's build of this form faulted on MI355X with no repair running and the cause was not found (DESIGN.md
// 3.5), so the default is the inlined repair again (round 6): on round 6's sources it is also the faster form
// (config 4 24.1 -> 26.0 M QP/s, WRITE_SIZE 142 -> 245 MB per launch, same box: profiles/r06_*).
#ifndef WBQ_ROLL_REPAIR_NOINLINE
#define WBQ_ROLL_REPAIR_NOINLINE 0
#endif
template <int NP, int M0>
__device__ __noinline__ void repair_instance_call(const QppvmArgs &a, double *S, long b, int i, bool rep)
{
    repair_instance<NP, M0>(a, S, b, i, rep);
}

template <int NP, int M0>
__device__ __noinline__ void repair_list(const QppvmArgs &a, int cnt)
{
    constexpr int IPW = kWave / NP;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const ActiveLayout<NP> L(a.ntasks, a.m0);
    const int sub = threadIdx.x / NP;
    const int i = threadIdx.x - sub * NP;
    double *S = smem + sub * L.SIZE;
    for (long e0 = (long)blockIdx.x * IPW; e0 < cnt; e0 += (long)gridDim.x * IPW) {
        const long e = e0 + sub;
        const bool valid = e < cnt;
        const long b = valid ? a.wl[a.B + e] : 0;
        WBQ_STAMP(8);
        WBQ_RTSTAMP(28); // (the constant 100 MHz clock beside the shader-clock stamps: their ratio is the clock)
        __syncthreads(); // the previous instance's LDS is dead
        repair_instance<NP, M0>(a, S, b, i, valid);
        WBQ_RTSTAMP(29);
    }
}

template <int NP, int M0>
__global__ __launch_bounds__(64, 1) void qppvm_repair_kernel(const QppvmArgs a)
{
    constexpr int IPW = kWave / NP;
    const int cnt = a.work[a.epoch * 2 + 1]; // instances flagged for the level-0 repair
    if (blockIdx.x == 0 && threadIdx.x == 0) { // the next solve's counters (its parity was last
        a.work[(a.epoch ^ 1) * 2] = 0;         // used by the previous solve, which has completed)
        a.work[(a.epoch ^ 1) * 2 + 1] = 0;
        if (a.handback) a.work[4 + (a.epoch ^ 1)] = 0; // (the hand-back pass runs after this kernel)
    }
    follow_publish(a.fg, a.work[a.epoch * 2], cnt);
    if ((long)blockIdx.x * IPW >= cnt) return;
    repair_list<NP, M0>(a, cnt);
}

// Waves per SIMD of the n > 32 fast kernel (template W). W = 2 caps it at 256 registers (it
// spills, ~760 B of scratch per lane) but doubles the resident instances: A/B n = 39 config 1
// (one box, profiles/r02_v10_ab_*) 30.3 -> 35.5 M QP/s. W = 1 (512 VGPR + AGPR, no spills) has
// the shorter single-instance latency: config 0's n = 39 plugin tick 73 us vs 110 us with W = 2.
// Batches that fit one wave round at W = 1 (<= 1,024 instances) take W = 1.
constexpr int kNp64OneRound = 1024;

// ====================================================================== fast path
// An instance whose equality-constrained optimum violates a bound needs the dual active
// set: with MERGED (NP = 32, where the active-set layout fits next to the fast one) it runs
// right here, inline; otherwise it parks (u, Q1) in scratch for qppvm_active_kernel
// (status -1). One whose level 0 is infeasible at b0 goes to qppvm_repair_kernel (-2).
// TM: the most tasks this instantiation handles (a.ntasks <= TM): with TM = 2 the stage issues
// 12 J-row loads and 2 pose loads per lane instead of 24 and 3 (TM = 4), which keeps a
// wave's stage under the 63 outstanding vector loads, and the elimination carries 3
// right-hand sides instead of 5.
// MR: rows of M loaded (n <= MR, compile time; the rest of the NP padding rows are identity
// without a load): with n = 39 and MR = 40 the stage issues ~59 loads per lane instead of ~83,
// under the 63 outstanding vector memory operations.
// ROLL (qppvm_rollout_kernel): one step of a fused rollout -- no work-list bookkeeping (the repair is
// inline, INLREP), the launch's counters are reset once by the caller.
template <int NP, int M0, bool MERGED, int TM, int W, int MR, bool INLREP, bool ROLL>
__device__ __forceinline__ void fast_body(const QppvmArgs &a)
{
    constexpr int IPW = kWave / NP;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int T = a.ntasks, n = a.n, m0 = a.m0;
    // the streamed LDL^T (round 6) for the plugin's stack shape: NP = 32, two tasks, six level-0 rows
    constexpr bool kLdl = WBQ_FAST_LDL != 0 && NP == 32 && TM == 2 && M0 == 6 && MR == 32;
    using FL = std::conditional_t<kLdl, LdlLayout, FastLayout<NP>>;
    const FL L(T, m0);
    int tid = threadIdx.x;
    // (a rollout step: the lane index is opaque per step, or the loop-invariant values derived from it
    // -- the identity padding of M, LDS offsets -- are hoisted out of the step loop and spilled across
    // every step. With this and the opaque arguments below: 1,504 -> 560 B of scratch, the hot path's
    // scratch loads per step ~240 -> ~60, and a repair-free 4096 x 20 rollout 1.45 -> 0.75 ms, the
    // time of 20 separate launches, 0.71 ms. (Putting the inline repair behind a noinline call as well
    // removed the rest of the hot path's spills, but the kernel then faulted on MI355X with an illegal
    // memory access even where no repair ran: not used.))
    if constexpr (ROLL) asm volatile("" : "+v"(tid));
    const int sub = tid / NP;
    const int i = tid - sub * NP;
    const long b = (long)blockIdx.x * IPW + sub;
    const bool valid = b < a.B;
    double *S = smem + sub * FastLdsLayout<NP, MERGED>(T, m0).SIZE;
    const bool row = valid && i < n;
    const long bn = valid ? b * n : 0;
    const int ic = i < n ? i : n - 1; // clamped column for unconditional loads
    // INLREP (no follow-up kernel publishes counts): the previous solve's counts, complete by
    // stream order, for the host's choice of the next solve's variant (FollowGrid)
    if constexpr (MERGED && INLREP && !ROLL)
        follow_publish(a.fg, a.work[(a.epoch ^ 1) * 2], a.work[(a.epoch ^ 1) * 2 + 1]);
    // (on-demand follow-up: no follow-up kernel publishes the counts or clears the counters either)
    if constexpr (MERGED && !INLREP && !ROLL)
        if (a.self_book) follow_publish(a.fg, a.work[(a.epoch ^ 1) * 2], a.work[(a.epoch ^ 1) * 2 + 1]);
    WBQ_RTSTAMP(16);
    WBQ_STAMP(0);

    // ---------------------------------------------------------------- 1. stage
    // Every global load is unconditional (clamped offsets, values selected afterwards), so
    // they issue back to back: one HBM round trip.
    // buffer resources start at the wave's first instance b0: per-lane offsets stay small
    const long b0 = (long)blockIdx.x * IPW, lb = valid ? b - b0 : 0, B = a.B;
    const int voff = (int)(8 * (lb * n + ic));
    const double q_i = bload(rsrc_at(a.q, b0, B, n), voff, 0), qd_i = bload(rsrc_at(a.qd, b0, B, n), voff, 0);
    const double qref_i = bload(rsrc_at(a.qref, b0, B, n), voff, 0), h_i0 = bload(rsrc_at(a.h, b0, B, n), voff, 0);
    // the warm-start hint is issued before the bulk loads: vmcnt retires in order, so a load
    // issued after M and waited for early would drain all of M with it
    const unsigned char hint_b = a.ws_hint[valid ? b : 0]; // unconditional: no branch on it here
    // J and the poses first, M last: vmcnt waits are in order, so the task forces (J, poses,
    // qd) can start while M is still streaming in
    double jv[TM * 6];
    {
        const __amdgpu_buffer_rsrc_t Jrs = rsrc_at(a.J, b0, B, (long)T * 6 * n);
        const int joff = (int)(8 * (lb * T * 6 * n + ic));
#pragma unroll
        for (int rr = 0; rr < TM * 6; ++rr) jv[rr] = bload(Jrs, joff, 8 * (rr < T * 6 ? rr : T * 6 - 1) * n);
    }
    constexpr int kPoseIt = (TM * 24 + NP - 1) / NP;
    double pv[kPoseIt];
    {
        const long base = lb * T * 12;
        const __amdgpu_buffer_rsrc_t Prs = rsrc_at(a.pose, b0, B, (long)T * 12);
        const __amdgpu_buffer_rsrc_t Rrs = rsrc_at(a.pose_ref, b0, B, (long)T * 12);
#pragma unroll
        for (int it = 0; it < kPoseIt; ++it) {
            int e = it * NP + i;
            e = e < T * 24 ? e : T * 24 - 1;
            const int t = e / 24, c = e - t * 24;
            const int cc = c < 12 ? c : c - 12;
            const double p0 = bload(Prs, (int)(8 * (base + t * 12 + cc)), 0);
            const double p1 = bload(Rrs, (int)(8 * (base + t * 12 + cc)), 0);
            pv[it] = (c < 12) ? p0 : p1;
        }
    }
    // NP = 64: the M loads issue after the task forces. Overlapped with them, the 40 in-flight rows
    // and the forces' temporaries exceeded the 256 VGPRs of 2 waves per SIMD, and the spill code
    // waited on each M load in turn (vmcnt(0) per row): a serialised stage.
    constexpr bool kForcesFirst = NP == 64;
    // NP = 32: the task-force gains of this lane's task row, loaded before M (a load issued after
    // M and waited for in the forces would wait for all of M)
    const int fr = i < T * 6 ? i : T * 6 - 1;
    double Kc_i = 0.0, Dc_i = 0.0;
    if constexpr (!kForcesFirst) {
        Kc_i = a.Kc[fr];
        Dc_i = a.Dc[fr];
    }
    // (LDL: the joint gains as well -- tau_imp is formed while M streams in)
    double Kq_i = 0.0, Dq_i = 0.0;
    if constexpr (kLdl) {
        Kq_i = a.Kq[ic];
        Dq_i = a.Dq[ic];
    }
    // NP = 32, issue order pinned: the scheduler hoisted the M loads above the J loads and sank a
    // J load into the uniform branch of its LDS store, where it waited with vmcnt(0) -- for all of
    // M -- before the task forces (vmcnt retires in order). Measured (same box): n = 30 config 1
    // 112.1 -> 114.9 M QP/s; the same pinning in the NP = 64 kernel cost 11 %
    if constexpr (!kForcesFirst) __builtin_amdgcn_sched_barrier(0);
    const __amdgpu_buffer_rsrc_t Mrs = rsrc_at(a.M, b0, B, (long)n * n);
    const int moff = (int)(8 * (lb * n * n + ic));
    // M is symmetric: lane i's row is its column, so row r of M read across lanes is
    // contiguous -- coalesced loads straight into the elimination registers.
    // (MR columns per lane: columns past MR are never pivoted and stay zero, block_gj's NC)
    double A[MR];
    if constexpr (!kForcesFirst) {
#pragma unroll
        for (int r = 0; r < MR; ++r) A[r] = bload(Mrs, moff, 8 * (r < n ? r : n - 1) * n);
        __builtin_amdgcn_sched_barrier(0);
    }
    const double h_i = row ? h_i0 : 0.0;
    const bool hint = valid && (hint_b & 1); // the last solve needed the level-0 repair
    const bool warm_gi = valid && (hint_b & 2); // ws_rows holds its final bound active set
    S[L.QD + i] = row ? qd_i : 0.0;
#pragma unroll
    for (int rr = 0; rr < TM * 6; ++rr)
        if (rr < T * 6) S[L.JR + rr * NP + i] = row ? jv[rr] : 0.0;
#pragma unroll
    for (int it = 0; it < kPoseIt; ++it)
        if (it * NP + i < T * 24) S[L.PS + it * NP + i] = valid ? pv[it] : 0.0;
    lds_barrier(); // M keeps streaming in behind the forces
    // task-space force per task row (spring + damper, zero desired twist), QPPVMPlugin.cpp:136-137
    if (i < T * 6) {
        const int t = i / 6, r = i - t * 6;
        // the error first, then the twist: overlapped, the twist's LDS operands and the rotation
        // error's temporaries spilled (a scratch reload issued after M waits for all of M)
        double er, xd;
        if constexpr (kForcesFirst) {
            xd = dot4<MR>(S + L.JR + i * NP, S + L.QD);
            er = cart_error_component(S + L.PS + t * 24, S + L.PS + t * 24 + 12, r);
        } else {
            er = cart_error_component(S + L.PS + t * 24, S + L.PS + t * 24 + 12, r);
            __builtin_amdgcn_sched_barrier(0);
            xd = dot4<MR>(S + L.JR + i * NP, S + L.QD);
        }
        if constexpr (kForcesFirst) {
            Kc_i = a.Kc[i];
            Dc_i = a.Dc[i];
        }
        double F = Kc_i * er - Dc_i * xd;
        // (the row masks packed into one uniform word: a per-lane indexed read of the kernel
        // argument is a vector load, and waiting for it after M's loads waits for all of M)
        if constexpr (kForcesFirst) {
            if (a.select_mode == 1 && !((a.row_mask[t] >> r) & 1)) F = 0.0;
        } else {
            unsigned rm = 0;
#pragma unroll
            for (int tt = 0; tt < kTMax; ++tt) rm |= ((unsigned)a.row_mask[tt] & 63u) << (6 * tt);
            if (a.select_mode == 1 && !((rm >> i) & 1u)) F = 0.0;
        }
        S[L.F + i] = F;
    }
    WBQ_STAMP(15);
    if constexpr (kForcesFirst) {
#pragma unroll
        for (int r = 0; r < MR; ++r) A[r] = bload(Mrs, moff, 8 * (r < n ? r : n - 1) * n);
    }
    constexpr int NT = M0 * (M0 + 1) / 2;
    // (set by either path below; u_imp and u_i by the LDL path only when an instance needs them)
    double Y[M0];               // Y = M G^T (row i): x = tau_imp + Y c needs no second read of M
    double tau_imp_i = 0.0, u_imp = 0.0, u_i = 0.0;
    bool notspd = false;
    double Lm[NT], il[M0], cv[M0]; // factor of G G^T (packed lower, row-major), c = (G G^T)^-1 res
    double eqres = 0.0, rmx = 1.0;
    double w_tau = 0.0;         // (LDL) this lane's entry of Dt^-1 Lt^-1 tau_imp
    if constexpr (kLdl) {
        // ------------------------------- 2'. streamed block LDL^T, forward substitution, Y = M G^T (round 6)
        // M = Lt Dt Lt^T (Lt unit lower by 4 x 4 blocks, Dt block diagonal) by a LEFT-looking sweep: pivot block kb
        // needs only M's columns 4kb..4kb+3 -- the rows this lane loaded kb-th -- and the panels of the blocks
        // before it, so it starts as soon as its rows land while M's later rows are still in flight (vmcnt
        // waits retire in issue order; only LDS-ordering barriers here). The Gauss-Jordan it replaces updated
        // every column at every step, so it could not start before the last row of M (a wave
        // waited ~11k of its ~54k cycles for M, then ran ~18k cycles of elimination).
        //   panel p (LDS): t_j(p) = M[j][blk p] - sum_{q<p} h_j(q) . t_{blk p}(q), rows j >= 4p
        //   D_p = t_{blk p}(p),  h_i(p) = t_i(p) D_p^-1 (rows after block p; lane i keeps it in A[4p..4p+3])
        // The columns B = [G^T | J_t^T F_t - tau_imp | tau_imp] are forward-substituted on the way (Z = Lt^-1 B,
        // right-looking: the pivot rows publish their final rows) and every pivot lane keeps its entries of
        // W = Dt^-1 Z for the last three, so that
        //   res_a = G_a M^-1 (J_t^T F_t - tau_imp) = sum_i Z_i[a] W_i[t(a)]     (one instance sum, no back sweep);
        // u_imp = M^-1 tau_imp = Lt^-T W_tau only when an instance needs u (after the bound check).
        constexpr int BS = LdlLayout::BS, NBLK = LdlLayout::NBLK, NB = LdlLayout::NB, RHS = LdlLayout::RHS;
        tau_imp_i = row ? Kq_i * (qref_i - q_i) - Dq_i * qd_i : 0.0; // (:105-106)
        lds_barrier();                                                 // the task forces
        int rsel[M0]; // (kernel-argument words: SGPRs)
#pragma unroll
        for (int c = 0; c < M0; ++c) rsel[c] = c < m0 ? a.row_selv[c] : 0;
        double Bv[NB];
#pragma unroll
        for (int c = 0; c < M0; ++c) Bv[c] = c < m0 ? S[L.JR + rsel[c] * NP + i] : 0.0;
#pragma unroll
        for (int t = 0; t < TM; ++t) {
            double c_ = 0.0;
            if (t < T)
#pragma unroll
                for (int r = 0; r < 6; ++r) c_ = fma(S[L.JR + (t * 6 + r) * NP + i], S[L.F + t * 6 + r], c_);
            Bv[M0 + t] = t < T ? c_ - tau_imp_i : 0.0; // J_t^T F_t - tau_imp
        }
        Bv[M0 + TM] = tau_imp_i;
        // the Gram G G^T (J only) and its rank-revealing factor while M streams in; the factor waits in LDS
        const int npairs = m0 * (m0 + 1) / 2;
        if (i < npairs) {
            int ra = (int)((sqrtf(8.0f * i + 1.0f) - 1.0f) * 0.5f);
            ra += ((ra + 1) * (ra + 2) / 2 <= i) ? 1 : 0;
            ra -= (ra * (ra + 1) / 2 > i) ? 1 : 0;
            const int ca = i - ra * (ra + 1) / 2;
            int r1 = rsel[0], r2 = rsel[0];
#pragma unroll
            for (int c = 1; c < M0; ++c) {
                r1 = ra == c ? rsel[c] : r1;
                r2 = ca == c ? rsel[c] : r2;
            }
            S[L.GR + ra * kM0Max + ca] = dot4<MR>(S + L.JR + r1 * NP, S + L.JR + r2 * NP);
        }
        lds_barrier();
        {
            double dmx = 0.0;
#pragma unroll
            for (int r = 0; r < M0; ++r) {
#pragma unroll
                for (int c = 0; c <= r; ++c) Lm[r * (r + 1) / 2 + c] = (r < m0) ? S[L.GR + r * kM0Max + c] : 0.0;
                dmx = fmax(dmx, Lm[r * (r + 1) / 2 + r]);
            }
#pragma unroll
            for (int c = 0; c < M0; ++c) {
                double dd = Lm[c * (c + 1) / 2 + c];
#pragma unroll
                for (int k = 0; k < c; ++k) dd = fma(-Lm[c * (c + 1) / 2 + k], Lm[c * (c + 1) / 2 + k], dd);
                const bool indep = c < m0 && dd > 1e-12 * dmx;
                const double ic_ = indep ? frsq(dd) : 0.0;
                il[c] = ic_;
                Lm[c * (c + 1) / 2 + c] = dd * ic_;
#pragma unroll
                for (int r = c + 1; r < M0; ++r) {
                    double t = Lm[r * (r + 1) / 2 + c];
#pragma unroll
                    for (int k = 0; k < c; ++k) t = fma(-Lm[r * (r + 1) / 2 + k], Lm[c * (c + 1) / 2 + k], t);
                    Lm[r * (r + 1) / 2 + c] = t * ic_;
                }
            }
            if (i == 0) {
#pragma unroll
                for (int q = 0; q < NT; ++q) S[L.LF + q] = Lm[q];
#pragma unroll
                for (int c = 0; c < M0; ++c) S[L.LF + NT + c] = il[c];
            }
        }
        WBQ_STAMP(1); // (diagnostic: the forces and the Gram done; the sweep follows M)
        double W3[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int g = 0; g < M0; ++g) Y[g] = 0.0;
#pragma unroll
        for (int kb = 0; kb < NBLK; ++kb) {
            const int k = kb * BS;
            if (k < n) {
                // (a) the earlier blocks' updates first, t_i -= h_i(p) . t_{blk kb}(p): they need the panels and
                //     h only, so they run while this block's rows of M are still in flight. Panel p's 4 x 4 block
                //     (rows k..k+3) is read one panel ahead of its FMAs (the compiler's own schedule waited for
                //     every read in turn), into two accumulator sets (half the dependent chain each).
                double ua[2][BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) ua[0][c] = ua[1][c] = 0.0;
                double pv[2][BS * BS];
                if (kb > 0) {
#pragma unroll
                    for (int e = 0; e < BS * BS; ++e) pv[0][e] = S[L.PL + LdlLayout::pofs(0) + BS * k + e];
                }
#pragma unroll
                for (int p = 0; p < kb; ++p) {
                    if (p + 1 < kb) {
#pragma unroll
                        for (int e = 0; e < BS * BS; ++e)
                            pv[(p + 1) & 1][e] = S[L.PL + LdlLayout::pofs(p + 1) + BS * (k - BS * (p + 1)) + e];
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int c = 0; c < BS; ++c)
#pragma unroll
                        for (int c2 = 0; c2 < BS; ++c2)
                            ua[p & 1][c] = fma(A[BS * p + c2], pv[p & 1][c * BS + c2], ua[p & 1][c]);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // (b) G's columns of this block (rows past m0 read row 0: their Y entries only ever meet c = 0)
                double gk[M0][BS];
#pragma unroll
                for (int g = 0; g < M0; ++g)
#pragma unroll
                    for (int c = 0; c < BS; ++c) gk[g][c] = S[L.JR + rsel[g] * NP + k + c];
                // (c) this block's columns of M -- the first wait for its four rows -- padding -> identity; Y += M G^T
                double tc[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    const double raw = (row && k + c < n) ? A[k + c] : (k + c == i ? 1.0 : 0.0);
#pragma unroll
                    for (int g = 0; g < M0; ++g) Y[g] = fma(raw, gk[g][c], Y[g]);
                    tc[c] = raw - (ua[0][c] + ua[1][c]);
                }
                const int ri = i - k;
                const bool inK = ri >= 0 && ri < BS;
                if (i >= k) { // panel kb, row i
#pragma unroll
                    for (int c = 0; c < BS; ++c) S[L.PL + LdlLayout::pofs(kb) + BS * ri + c] = tc[c];
                }
                if (inK) { // the pivot rows' columns are final now (every earlier block's update is in)
#pragma unroll
                    for (int m = 0; m < NB; ++m) S[L.RH + (kb & 1) * BS * RHS + ri * RHS + m] = Bv[m];
                }
                lds_barrier();
                // D = the pivot block of panel kb: Cholesky (redundant per lane); the pivot rows' columns are read
                // with it (all reads issued before the factor's dependent chain)
                const double *pd = S + L.PL + LdlLayout::pofs(kb);
                const double *zb = S + L.RH + (kb & 1) * BS * RHS;
                double d[BS][BS], il4[BS], zv[BS][NB];
#pragma unroll
                for (int r = 0; r < BS; ++r)
#pragma unroll
                    for (int c = 0; c <= r; ++c) d[r][c] = pd[r * BS + c];
#pragma unroll
                for (int r = 0; r < BS; ++r)
#pragma unroll
                    for (int m = 0; m < NB; ++m) zv[r][m] = zb[r * RHS + m];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    double dd = d[c][c];
#pragma unroll
                    for (int q_ = 0; q_ < c; ++q_) dd = fma(-d[c][q_], d[c][q_], dd);
                    notspd |= !(dd > 0.0);
                    il4[c] = frsq(dd);
#pragma unroll
                    for (int r = c + 1; r < BS; ++r) {
                        double t = d[r][c];
#pragma unroll
                        for (int q_ = 0; q_ < c; ++q_) t = fma(-d[r][q_], d[c][q_], t);
                        d[r][c] = t * il4[c];
                    }
                }
                // y = D^-1 t_i (rows after the block: h_i(kb)), or row ri of D^-1 (the block's own rows)
                double y[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    double v = inK ? (ri == c ? 1.0 : 0.0) : tc[c];
#pragma unroll
                    for (int q_ = 0; q_ < c; ++q_) v = fma(-d[c][q_], y[q_], v);
                    y[c] = v * il4[c];
                }
#pragma unroll
                for (int c = BS - 1; c >= 0; --c) {
                    double v = y[c];
#pragma unroll
                    for (int q_ = c + 1; q_ < BS; ++q_) v = fma(-d[q_][c], y[q_], v);
                    y[c] = v * il4[c];
                }
                const bool later = i >= k + BS;
#pragma unroll
                for (int c = 0; c < BS; ++c) A[k + c] = later ? y[c] : 0.0; // h_i(kb)
#pragma unroll
                for (int m = 0; m < NB; ++m) {
                    double v = Bv[m];
#pragma unroll
                    for (int c = 0; c < BS; ++c) v = fma(-A[k + c], zv[c][m], v);
                    Bv[m] = v;
                }
#pragma unroll
                for (int t = 0; t < 3; ++t) { // W = D^-1 Z on the block's own rows
                    double w = 0.0;
#pragma unroll
                    for (int c = 0; c < BS; ++c) w = fma(y[c], zv[c][M0 + t], w);
                    W3[t] = inK ? w : W3[t];
                }
            }
        }
        WBQ_STAMP(2);
        // ------------------------------------------ 3'. level-0 rows: G u = b0 in least distance from u_imp
        double rv[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) rv[c] = c < m0 ? Bv[c] * ((rsel[c] >= 6) ? W3[1] : W3[0]) : 0.0;
        isum_vec<NP, M0>(rv);
        if (i < m0) { // (the repair path's b0 reads res from LDS)
            double v = 0.0;
#pragma unroll
            for (int c = 0; c < M0; ++c) v = i == c ? rv[c] : v;
            S[L.RES + i] = v;
        }
        w_tau = W3[2];
        double rs[M0];
#pragma unroll
        for (int r = 0; r < M0; ++r) rs[r] = (r < m0) ? rv[r] : 0.0;
#pragma unroll
        for (int q = 0; q < NT; ++q) Lm[q] = S[L.LF + q];
#pragma unroll
        for (int c = 0; c < M0; ++c) il[c] = S[L.LF + NT + c];
#pragma unroll
        for (int c = 0; c < M0; ++c) { // forward: rho = L^-1 res
            double v = rs[c];
#pragma unroll
            for (int k = 0; k < c; ++k) v = fma(-Lm[c * (c + 1) / 2 + k], cv[k], v);
            cv[c] = v * il[c];
        }
#pragma unroll
        for (int c = M0 - 1; c >= 0; --c) { // backward: c = L^-T rho
            double v = cv[c];
#pragma unroll
            for (int k = c + 1; k < M0; ++k) v = fma(-Lm[k * (k + 1) / 2 + c], cv[k], v);
            cv[c] = v * il[c];
        }
        // consistency of the level-0 rows (rows dropped as dependent must still be met, else y* != b0)
#pragma unroll
        for (int r = 0; r < M0; ++r) {
            double v = -rs[r];
#pragma unroll
            for (int c = 0; c < M0; ++c)
                if (r < m0 && c < m0) v = fma(S[L.GR + (r >= c ? r * kM0Max + c : c * kM0Max + r)], cv[c], v);
            eqres = fmax(eqres, fabs(v));
            rmx = fmax(rmx, fabs(rs[r]));
        }
    } else {
        if constexpr (WBQ_FAST_EQ_EARLY == 1) {
            // the Gram G G^T and its factor from J alone, while M is still in flight: lane i's column of the
            // selected J rows, per-lane outer products, instance sums by DPP (no LDS round trips); every
            // lane factors it (rank-revealing Cholesky, dependent rows get a zero column) and lane 0 keeps
            // the Gram (GR, lower triangle) and the factor (LF) for after the elimination
            double g[M0];
    #pragma unroll
            for (int c = 0; c < M0; ++c) g[c] = (c < m0) ? S[L.JR + a.row_sel[c < m0 ? c : 0] * NP + i] : 0.0;
            double gg[NT];
    #pragma unroll
            for (int r = 0; r < M0; ++r)
    #pragma unroll
                for (int c = 0; c <= r; ++c) gg[r * (r + 1) / 2 + c] = g[r] * g[c];
            isum_vec<NP, NT>(gg);
            double Lq[NT], ilq[M0];
            double dmx = 0.0;
    #pragma unroll
            for (int r = 0; r < M0; ++r) {
    #pragma unroll
                for (int c = 0; c <= r; ++c) Lq[r * (r + 1) / 2 + c] = (r < m0) ? gg[r * (r + 1) / 2 + c] : 0.0;
                dmx = fmax(dmx, Lq[r * (r + 1) / 2 + r]);
            }
    #pragma unroll
            for (int c = 0; c < M0; ++c) {
                double dd = Lq[c * (c + 1) / 2 + c];
    #pragma unroll
                for (int k = 0; k < c; ++k) dd = fma(-Lq[c * (c + 1) / 2 + k], Lq[c * (c + 1) / 2 + k], dd);
                const bool indep = c < m0 && dd > 1e-12 * dmx;
                const double ic_ = indep ? frsq(dd) : 0.0;
                ilq[c] = ic_;
                Lq[c * (c + 1) / 2 + c] = dd * ic_;
    #pragma unroll
                for (int r = c + 1; r < M0; ++r) {
                    double t = Lq[r * (r + 1) / 2 + c];
    #pragma unroll
                    for (int k = 0; k < c; ++k) t = fma(-Lq[r * (r + 1) / 2 + k], Lq[c * (c + 1) / 2 + k], t);
                    Lq[r * (r + 1) / 2 + c] = t * ic_;
                }
            }
            if (i == 0) {
    #pragma unroll
                for (int r = 0; r < M0; ++r) {
    #pragma unroll
                    for (int c = 0; c <= r; ++c)
                        if (r < m0) S[L.GR + r * kM0Max + c] = gg[r * (r + 1) / 2 + c];
                    S[L.LF + NT + r] = ilq[r];
                }
    #pragma unroll
                for (int q = 0; q < NT; ++q) S[L.LF + q] = Lq[q];
            }
        }
        // M (still streaming in during the forces): padding rows/columns past n -> identity
    #pragma unroll
        for (int r = 0; r < MR; ++r) A[r] = (row && r < n) ? A[r] : (r == i ? 1.0 : 0.0);
        // Y = M G^T (row i per lane): then x = M u = tau_imp + Y c after the elimination, and M
        // never has to be read again (a re-read of M would double the HBM bytes of the solve)
        if constexpr (WBQ_FAST_Y_CH == 0) {
    #pragma unroll
            for (int c = 0; c < M0; ++c) {
                double v = 0.0;
                if (c < m0) {
                    const int rr = a.row_sel[c];
    #pragma unroll
                    for (int j = 0; j < MR; ++j) v = fma(A[j], S[L.JR + rr * NP + j], v);
                }
                Y[c] = v;
            }
        } else {
            // the same sums (j ascending per row), the G rows read WBQ_FAST_Y_CH columns ahead
            constexpr int YC = WBQ_FAST_Y_CH, NYC = MR / YC;
            static_assert(MR % YC == 0, "WBQ_FAST_Y_CH divides MR");
            int rrs[M0];
    #pragma unroll
            for (int c = 0; c < M0; ++c) {
                rrs[c] = c < m0 ? a.row_sel[c < m0 ? c : 0] : 0;
                Y[c] = 0.0;
            }
            double gb[2][M0][YC];
    #pragma unroll
            for (int ch = 0; ch <= NYC; ++ch) {
                if (ch < NYC) {
    #pragma unroll
                    for (int c = 0; c < M0; ++c)
    #pragma unroll
                        for (int u = 0; u < YC; ++u) gb[ch & 1][c][u] = S[L.JR + rrs[c] * NP + ch * YC + u];
                }
                __builtin_amdgcn_sched_barrier(0);
                if (ch > 0) {
    #pragma unroll
                    for (int c = 0; c < M0; ++c)
    #pragma unroll
                        for (int u = 0; u < YC; ++u)
                            Y[c] = fma(A[(ch - 1) * YC + u], c < m0 ? gb[(ch - 1) & 1][c][u] : 0.0, Y[c]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __syncthreads();
        WBQ_STAMP(1);

        // ------------------------------------------ 2. block Gauss-Jordan, M SPD
        double rhs[1 + TM];
        rhs[0] = row ? a.Kq[ic] * (qref_i - q_i) - a.Dq[ic] * qd_i : 0.0; // tau_imp (:105-106)
        tau_imp_i = rhs[0];
    #pragma unroll
        for (int t = 0; t < TM; ++t) {
            double c = 0.0;
            if (t < T)
    #pragma unroll
                for (int r = 0; r < 6; ++r) c = fma(S[L.JR + (t * 6 + r) * NP + i], S[L.F + t * 6 + r], c);
            rhs[1 + t] = c; // J_t^T F_t
        }
        // (the chunked reads only where the columns leave registers for them: with 64 columns per lane they
        // spilled, 0 -> 528 B of scratch)
        constexpr int kGjCh = MR <= 40 ? WBQ_FAST_GJ_CH : 0;
        notspd = block_gj<NP, 1 + TM, 8, MR, kGjCh, WBQ_FAST_GJ_UNI != 0>(A, rhs, n, i, S + L.PN, S + L.RH);
        u_imp = rhs[0]; // u_imp = M^-1 tau_imp, w_t = M^-1 J_t^T F_t = rhs[1+t]
        double gq[NT], resq[M0]; // (EQ_EARLY == 2) the Gram and res in registers
        if constexpr (!WBQ_FAST_EQ_EARLY) {
    #pragma unroll
            for (int t = 0; t < TM; ++t)
                if (t < T) S[L.WV + t * NP + i] = rhs[1 + t] - u_imp;
            __syncthreads();
        }
        WBQ_STAMP(2);

        // ------------------------------ 3. level-0 rows: G u = b0 in least distance from u_imp
        // res_a = b0_a - G_a u_imp = G_a (w_t(a) - u_imp), and the Gram G G^T: one dot per lane
        if constexpr (WBQ_FAST_EQ_EARLY == 2) {
            // res and the Gram by per-lane products (lane i's column of the selected J rows), one DPP
            // reduction of the NT + M0 sums; no LDS round trip
            double g[M0], v[NT + M0];
    #pragma unroll
            for (int c = 0; c < M0; ++c) {
                const int rr = c < m0 ? a.row_sel[c < m0 ? c : 0] : 0, tt = rr / 6;
                g[c] = c < m0 ? S[L.JR + rr * NP + i] : 0.0;
                double w = rhs[1];
    #pragma unroll
                for (int t = 1; t < TM; ++t) w = tt == t ? rhs[1 + t] : w;
                v[NT + c] = g[c] * (w - u_imp);
            }
    #pragma unroll
            for (int r = 0; r < M0; ++r)
    #pragma unroll
                for (int c = 0; c <= r; ++c) v[r * (r + 1) / 2 + c] = g[r] * g[c];
            isum_vec<NP, NT + M0>(v);
    #pragma unroll
            for (int q = 0; q < NT; ++q) gq[q] = v[q];
    #pragma unroll
            for (int c = 0; c < M0; ++c) resq[c] = v[NT + c];
            if (i < m0) { // (the repair path's b0 reads res from LDS)
                double rv = 0.0;
    #pragma unroll
                for (int c = 0; c < M0; ++c) rv = i == c ? resq[c] : rv;
                S[L.RES + i] = rv;
            }
        } else if constexpr (WBQ_FAST_EQ_EARLY == 1) {
            // (the Gram and its factor are in LDS since the stage) res by per-lane products and DPP sums
            double rp[M0];
    #pragma unroll
            for (int c = 0; c < M0; ++c) {
                const int rr = c < m0 ? a.row_sel[c < m0 ? c : 0] : 0, tt = rr / 6;
                double w = rhs[1];
    #pragma unroll
                for (int t = 1; t < TM; ++t) w = tt == t ? rhs[1 + t] : w;
                rp[c] = c < m0 ? S[L.JR + rr * NP + i] * (w - u_imp) : 0.0;
            }
            isum_vec<NP, M0>(rp);
            if (i == 0) {
    #pragma unroll
                for (int c = 0; c < M0; ++c)
                    if (c < m0) S[L.RES + c] = rp[c];
            }
            __syncthreads();
        } else {
            const int npairs = m0 * (m0 + 1) / 2;
            for (int pp = i; pp < npairs + m0; pp += NP) {
                if (pp < m0) {
                    const int rr = a.row_sel[pp], t = rr / 6;
                    S[L.RES + pp] = dot4<MR>(S + L.JR + rr * NP, S + L.WV + t * NP);
                } else {
                    const int p2 = pp - m0;
                    int ra = (int)((sqrtf(8.0f * p2 + 1.0f) - 1.0f) * 0.5f);
                    ra += ((ra + 1) * (ra + 2) / 2 <= p2) ? 1 : 0;
                    ra -= (ra * (ra + 1) / 2 > p2) ? 1 : 0;
                    const int ca = p2 - ra * (ra + 1) / 2;
                    const int r1 = a.row_sel[ra], r2 = a.row_sel[ca];
                    S[L.GR + ra * kM0Max + ca] = dot4<MR>(S + L.JR + r1 * NP, S + L.JR + r2 * NP);
                }
            }
            __syncthreads();
        }
        // Every lane factors the small Gram redundantly in registers: rank-revealing Cholesky
        // G G^T = L L^T (dependent rows get a zero column), c = L^-T L^-1 res, u = u_imp + G^T c.
        double rs[M0];
        if constexpr (WBQ_FAST_EQ_EARLY == 1) {
    #pragma unroll
            for (int r = 0; r < M0; ++r) {
                rs[r] = (r < m0) ? S[L.RES + r] : 0.0;
                il[r] = S[L.LF + NT + r];
            }
    #pragma unroll
            for (int q = 0; q < NT; ++q) Lm[q] = S[L.LF + q];
        } else {
            double dmx = 0.0;
    #pragma unroll
            for (int r = 0; r < M0; ++r) {
                if constexpr (WBQ_FAST_EQ_EARLY == 2) rs[r] = (r < m0) ? resq[r] : 0.0;
                else rs[r] = (r < m0) ? S[L.RES + r] : 0.0;
    #pragma unroll
                for (int c = 0; c <= r; ++c) {
                    if constexpr (WBQ_FAST_EQ_EARLY == 2) Lm[r * (r + 1) / 2 + c] = (r < m0) ? gq[r * (r + 1) / 2 + c] : 0.0;
                    else Lm[r * (r + 1) / 2 + c] = (r < m0) ? S[L.GR + r * kM0Max + c] : 0.0;
                }
                dmx = fmax(dmx, Lm[r * (r + 1) / 2 + r]);
            }
    #pragma unroll
            for (int c = 0; c < M0; ++c) {
                double dd = Lm[c * (c + 1) / 2 + c];
    #pragma unroll
                for (int k = 0; k < c; ++k) dd = fma(-Lm[c * (c + 1) / 2 + k], Lm[c * (c + 1) / 2 + k], dd);
                const bool indep = c < m0 && dd > 1e-12 * dmx;
                const double ic_ = indep ? frsq(dd) : 0.0;
                il[c] = ic_;
                Lm[c * (c + 1) / 2 + c] = dd * ic_;
    #pragma unroll
                for (int r = c + 1; r < M0; ++r) {
                    double t = Lm[r * (r + 1) / 2 + c];
    #pragma unroll
                    for (int k = 0; k < c; ++k) t = fma(-Lm[r * (r + 1) / 2 + k], Lm[c * (c + 1) / 2 + k], t);
                    Lm[r * (r + 1) / 2 + c] = t * ic_;
                }
            }
        }
    #pragma unroll
        for (int c = 0; c < M0; ++c) { // forward: rho = L^-1 res
            double v = rs[c];
    #pragma unroll
            for (int k = 0; k < c; ++k) v = fma(-Lm[c * (c + 1) / 2 + k], cv[k], v);
            cv[c] = v * il[c];
        }
    #pragma unroll
        for (int c = M0 - 1; c >= 0; --c) { // backward: c = L^-T rho
            double v = cv[c];
    #pragma unroll
            for (int k = c + 1; k < M0; ++k) v = fma(-Lm[k * (k + 1) / 2 + c], cv[k], v);
            cv[c] = v * il[c];
        }
        // consistency of the level-0 rows (rows dropped as dependent must still be met,
        // otherwise y* != b0: level 0 infeasible)
    #pragma unroll
        for (int r = 0; r < M0; ++r) {
            double v = -rs[r];
    #pragma unroll
            for (int c = 0; c < M0; ++c) {
                if constexpr (WBQ_FAST_EQ_EARLY == 2) {
                    if (r < m0 && c < m0) v = fma(gq[r >= c ? r * (r + 1) / 2 + c : c * (c + 1) / 2 + r], cv[c], v);
                } else {
                    if (r < m0 && c < m0) v = fma(S[L.GR + (r >= c ? r * kM0Max + c : c * kM0Max + r)], cv[c], v);
                }
            }
            eqres = fmax(eqres, fabs(v));
            rmx = fmax(rmx, fabs(rs[r]));
        }
        u_i = u_imp;
    #pragma unroll
        for (int c = 0; c < M0; ++c)
            if (c < m0) u_i = fma(S[L.JR + a.row_sel[c] * NP + i], cv[c], u_i);
    }
    WBQ_STAMP(3);

    // ------------------------------------------------------------ 4. bound check
    double x_i = tau_imp_i; // x = M u = tau_imp + M G^T c
#pragma unroll
    for (int c = 0; c < M0; ++c) x_i = fma(Y[c], cv[c], x_i);
    double lo = -kInf, hi = kInf;
    if (row) torque_box(a, ic, q_i, qd_i, h_i, lo, hi);
    int status = 0;
    if (a.limits_crossed) status = 2; // tau_min > tau_max somewhere: infeasible everywhere
    // the JointLimits box can empty per instance (a joint beyond its limit and moving outwards)
    if (a.joint_limits && imax<NP>((row && lo > hi) ? 1.0 : 0.0) > 0.0) status = 2;
    if (notspd) status = 3;           // (instance-uniform: pivots are broadcast values)
    // rows dropped as dependent are not met: y* != b0, level 0 itself is infeasible at b0 and
    // the active-set kernel runs the level-0 repair (BVLS for y*) first
    const bool l0bad = status == 0 && eqres > 1e-9 * rmx;
    double flag = 0.0;
    if (row) {
        const double tol = 1e-10 * fmax(1.0, fmax(fabs(x_i), fmax(fabs(lo), fabs(hi))));
        if (fmax(lo - x_i, x_i - hi) > tol) flag = 1.0;
        if (!isfinite(x_i)) flag = 2.0;
    }
    flag = imax<NP>(flag);
    if (flag >= 2.0 && status == 0) status = 3;
    const bool active = (flag > 0.0 || l0bad) && status == 0 && valid;
    if constexpr (kLdl) {
        // u_imp = M^-1 tau_imp = Lt^-T (Dt^-1 Lt^-1 tau_imp) and u = u_imp + G^T c, only when some instance of
        // the wave needs u: a rollout integrates qdd = u, an active bound or a level-0 repair starts from it
        // (the common path needs x alone). Block kb from the last: u_blk = w_blk - sum_{later rows i} h_i(kb) u_i.
        if (a.integrate || __any(active)) {
            constexpr int BS = LdlLayout::BS, NBLK = LdlLayout::NBLK;
            double uu = 0.0;
#pragma unroll
            for (int kb = NBLK - 1; kb >= 0; --kb) {
                const int k = kb * BS;
                if (k < n) {
                    double s4[BS];
#pragma unroll
                    for (int c = 0; c < BS; ++c) s4[c] = A[k + c] * uu;
                    isum_vec<NP, BS>(s4);
                    const int ri = i - k;
                    double sv = 0.0;
#pragma unroll
                    for (int c = 0; c < BS; ++c) sv = ri == c ? s4[c] : sv;
                    if (ri >= 0 && ri < BS) uu = w_tau - sv;
                }
            }
            u_imp = uu;
            u_i = u_imp;
#pragma unroll
            for (int c = 0; c < M0; ++c)
                if (c < m0) u_i = fma(S[L.JR + a.row_selv[c] * NP + i], cv[c], u_i);
        }
    }
    if (__any(active)) { // b0 = res + G u_imp for the level-0 repair
        S[L.U + i] = u_imp;
        __syncthreads();
        if (active && i < m0) {
            const int rr = a.row_sel[i];
            const double v = S[L.RES + i] + dot4<MR>(S + L.JR + rr * NP, S + L.U);
            a.b0_scr[b * kM0Max + i] = v;
        }
    }

    // level-0 infeasible, or (warm start) it was last time: straight to the repair kernel
    const bool to_rep = l0bad || hint;
    bool rep_inl = false; // INLREP: this instance's level-0 repair runs at the end of this kernel
    if (!active) {
        double tau_i = x_i + h_i;
        if (status != 0) tau_i = h_i; // "SOLVER ERROR!" fallback: tau_qp = 0 (:246-249)
        if (row) a.tau[bn + i] = tau_i;
        rollout_step(a, b, i, row, u_i, status == 0); // qdd = M^-1 (tau - h) = u
        if (valid && i == 0) {
            a.status[b] = status;
            a.iters[b] = 0;
            if (hint_b != 0) a.ws_hint[b] = 0; // level 0 met at b0 inside the bounds: no active bound
        }
    }
    if (__any(active)) {
        // Q1 = G^T L^-T row by row
        double q1[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            double v = (c < m0) ? S[L.JR + a.row_sel[c] * NP + i] : 0.0;
#pragma unroll
            for (int k = 0; k < c; ++k) v = fma(-Lm[c * (c + 1) / 2 + k], q1[k], v);
            q1[c] = v * il[c];
        }
        if (active) a.ui_scr[b * NP + i] = u_imp; // for the level-0 repair
        if constexpr (MERGED) {
            __syncthreads(); // the fast layout is dead: this LDS becomes the active-set layout
            const ActiveLayout<NP> LA(T, m0);
            const bool ga = active && !to_rep;
#pragma unroll
            for (int c = 0; c < NP; ++c) S[LA.QA + c * (NP + 1) + i] = (ga && c < M0 && c < m0) ? q1[c < M0 ? c : 0] : 0.0;
            int st2 = 0, it2 = 0;
            bool inf = false;
            const int wsg = (ga && warm_gi && row) ? (int)a.ws_rows[b * 64 + i] : 0;
            WBQ_STAMP(18); // (diagnostic build: the inline dual active set starts)
            double x2, u2;
            if constexpr (NP == 32 && WBQ_GI_CS != 0) {
                // this lane's column of V = Q1 M = L^-1 G M: forward substitution of Y's row (Y = M G^T)
                double vcol[M0];
#pragma unroll
                for (int c = 0; c < M0; ++c) {
                    double v = (c < m0) ? Y[c] : 0.0;
#pragma unroll
                    for (int k = 0; k < c; ++k) v = fma(-Lm[c * (c + 1) / 2 + k], vcol[k], v);
                    vcol[c] = v * il[c];
                }
                bool bail;
                x2 = cs_solve<NP, M0, 20, 13>(a, S, ga ? b : 0, i, row && ga, ga, lo, hi, u_i, st2, it2, inf, wsg, true, u2,
                                          vcol, bail, x_i);
                inf |= bail; // (the level-0 repair takes a hand-off: its u-space loop settles it)
            } else {
                x2 = gi_solve<NP, M0, 20, 13>(a, S, ga ? b : 0, i, row && ga, ga, lo, hi, u_i, st2, it2, inf, wsg, true);
                u2 = S[LA.U + i];
            }
            WBQ_STAMP(19);
            const bool rep = active && (inf || to_rep);
            if (active && !rep) { // (before the repair below, which reuses the wave's LDS)
                double tau2 = x2 + h_i;
                if (!isfinite(tau2) && st2 == 0) st2 = 3;
                if (st2 != 0) tau2 = h_i;
                if (row) a.tau[bn + i] = tau2;
                rollout_step(a, b, i, row, u2, st2 == 0);
                if (i == 0) {
                    a.status[b] = st2;
                    a.iters[b] = it2;
                    a.ws_hint[b] = st2 == 0 ? 2 : 0; // ws_rows now holds this solve's active set
                }
            }
            // the level-0 repair runs in its own kernel: inlined here its register demand spilled
            // into the fast path
            if constexpr (INLREP) {
                rep_inl = rep;
            } else if (rep && i == 0) {
                a.status[b] = -2; // qppvm_repair_kernel
                wl_push(a, 1, b);
            }
        } else if (active) { // park (u, Q1) for the active-set kernel
            double *us = a.u_scr + b * NP;
            double *qs = a.q1_scr + b * kM0Max * NP;
            us[i] = u_i;
#pragma unroll
            for (int c = 0; c < M0; ++c)
                if (c < m0) qs[c * NP + i] = q1[c];
            if (i == 0) {
                a.status[b] = to_rep ? -2 : -1; // picked up by the active-set / repair kernel
                wl_push(a, to_rep ? 1 : 0, b);
            }
        }
    }
    WBQ_STAMP(5);
    if constexpr (MERGED && !INLREP && !ROLL) {
        if (a.self_book && blockIdx.x == 0 && tid == 0) { // the next solve's counters (published above)
            a.work[(a.epoch ^ 1) * 2] = 0;
            a.work[(a.epoch ^ 1) * 2 + 1] = 0;
        }
    }
    if constexpr (MERGED && INLREP) {
        // one launch per solve: no follow-up kernel resets the next solve's work counters
        if (!ROLL && blockIdx.x == 0 && tid == 0) {
            a.work[(a.epoch ^ 1) * 2] = 0;
            a.work[(a.epoch ^ 1) * 2 + 1] = 0;
        }
        // the level-0 repair at the kernel's top level, after every fast-path value is dead, so
        // its register demand does not reach the fast path (inlined inside the active-set branch
        // it spilled there)
        if (__any(rep_inl)) {
            if (!ROLL && rep_inl && i == 0) atomicAdd(a.work + a.epoch * 2 + 1, 1); // the repair count (grid policy)
            __syncthreads();
#ifdef WBQ_STAMPS
            const unsigned long long rt0_ = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (ROLL && WBQ_ROLL_REPAIR_NOINLINE != 0)
                repair_instance_call<NP, M0>(a, S, rep_inl ? b : 0, i, rep_inl);
            else
                repair_instance<NP, M0>(a, S, rep_inl ? b : 0, i, rep_inl);
#ifdef WBQ_STAMPS
            // (diagnostic: inline repairs' cycles and count summed in slots 6 / 7)
            const unsigned long long rt1_ = __builtin_amdgcn_s_memtime();
            if (tid == 0 && a.stamps) {
                a.stamps[blockIdx.x * kStamps + 6] += rt1_ - rt0_;
                a.stamps[blockIdx.x * kStamps + 7] += 1;
            }
#endif
        }
    }
    WBQ_RTSTAMP(17);
}

template <int NP, int M0, bool MERGED, int TM, int W, int MR, bool INLREP = false>
__global__ __launch_bounds__(64, W) void qppvm_fast_kernel(const QppvmArgs a)
{
    fast_body<NP, M0, MERGED, TM, W, MR, INLREP, false>(a);
}

// MPC rollout in one launch (wbq_rollout): every wave runs its instances'
// `steps` integrating solves back to back -- the fast path, the dual active set and the level-0 repair
// inline -- carrying q, qd (rollout_step) and the warm-start state (ws_hint, ws_rows, ws_state) from
// step to step through its own global rows. The same work as `steps` launches of the inline-repair
// fast kernel; without the per-step launch boundary an instance whose repair runs long delays only its
// own wave instead of every instance's next step (config 4 with per-step launches: the rare repaired
// instance-steps, ~0.3 %, held whole launches for hundreds of microseconds).
// (WBQ_ROLL_W: waves per SIMD of the fused rollout, 2 as the fast kernel; 1 gives its dual active-set loop
// 512 registers -- no spills, LDS reads in flight -- at half the resident instances)
#ifndef WBQ_ROLL_W
#define WBQ_ROLL_W 2
#endif
// (diagnostic: WBQ_ROLL_ARG=a hands the steps the by-value kernel argument itself instead of the laundered
// kernarg-segment reference -- with the repair call, round 4's faulting build)
#ifndef WBQ_ROLL_ARG
#define WBQ_ROLL_ARG as
#endif
template <int NP, int M0, int TM>
__global__ __launch_bounds__(64, WBQ_ROLL_W) void qppvm_rollout_kernel(const QppvmArgs a)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) { // one launch: the next solve's counters (as INLREP)
        a.work[(a.epoch ^ 1) * 2] = 0;
        a.work[(a.epoch ^ 1) * 2 + 1] = 0;
    }
    WBQ_STAMP(28); // (diagnostic: the block's whole rollout, shader clock 28-29, realtime 30-31)
    WBQ_RTSTAMP(30);
#pragma unroll 1
    for (int s = 0; s < a.steps; ++s) {
        // the arguments through an opaque kernarg pointer per step: values loaded from them are not
        // hoisted out of the loop and spilled (1,504 -> 1,056 B of scratch with this alone)
        typedef const __attribute__((address_space(4))) char *KPtr;
        KPtr kp = (KPtr)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const QppvmArgs &as = *(const QppvmArgs *)(const char *)kp;
        fast_body<NP, M0, true, TM, WBQ_ROLL_W, 32, true, true>(WBQ_ROLL_ARG);
        __syncthreads(); // this wave's q, qd and warm-start writes are visible to its next step
    }
    WBQ_STAMP(29);
    WBQ_RTSTAMP(31);
}

template <int NP, typename Lay, typename K>
hipError_t launch_one(K kern, const QppvmArgs &a, unsigned grid, hipStream_t stream, bool nsized = false)
{
    constexpr int IPW = kWave / NP;
    // nsized: the 64-lane active-set kernel's layout with its rows sized by n (ActiveLayout)
    int size = Lay(a.ntasks, a.m0).SIZE;
    if constexpr (std::is_same_v<Lay, ActiveLayout<NP>>)
        if (nsized) size = ActiveLayout<NP>(a.ntasks, a.m0, a.n).SIZE;
    const size_t lds = sizeof(double) * size * IPW;
    if (a.prepare) return ensure_dynamic_lds((const void *)kern, lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWave), lds, stream, a);
    return hipGetLastError();
}

template <int M0>
constexpr bool kInlineRepair = M0 <= 6;

template <int NP, int M0>
hipError_t launch_np(const QppvmArgs &a, hipStream_t stream, hipEvent_t mid)
{
    constexpr int IPW = kWave / NP;
    const unsigned grid = (unsigned)((a.B + IPW - 1) / IPW);
    if (grid == 0) return hipSuccess;
    constexpr bool MERGED = NP == 32; // active-set layout fits next to the fast one
    using Lay = FastLdsLayout<NP, MERGED>;
    if (NP == 32 && a.ntasks <= 2 && a.m0 <= 6 && LdlLayout(a.ntasks, a.m0).SIZE > Lay(a.ntasks, a.m0).SIZE)
        return hipErrorInvalidValue; // (the streamed LDL^T path's layout must fit the instance's LDS)
    hipError_t e;
    if constexpr (NP == 32 && kInlineRepair<M0>) { // a whole rollout in one launch
        if (a.steps > 0 || a.prepare) {
            e = a.ntasks <= 2 ? launch_one<NP, Lay>(qppvm_rollout_kernel<NP, M0, 2>, a, grid, stream)
                              : launch_one<NP, Lay>(qppvm_rollout_kernel<NP, M0, kTMax>, a, grid, stream);
            if (e != hipSuccess || !a.prepare) {
                if (e == hipSuccess && mid) e = hipEventRecord(mid, stream);
                return e;
            }
        }
    }
    if constexpr (NP == 32) {
        // (the inline repair only where it keeps 2 waves per SIMD: M0 <= 6)
        const bool inl = kInlineRepair<M0> && (a.inline_repair || a.prepare);
        const bool sep = !inl || a.prepare;
        e = hipSuccess;
        if constexpr (kInlineRepair<M0>) {
            if (inl)
                e = a.ntasks <= 2
                        ? launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, 2, 2, 32, true>, a, grid, stream)
                        : launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, kTMax, 2, 32, true>, a, grid, stream);
        }
        if (e == hipSuccess && sep)
            e = a.ntasks <= 2 ? launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, 2, 2, 32>, a, grid, stream)
                              : launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, kTMax, 2, 32>, a, grid, stream);
    } else if (a.ntasks > 2) {
        e = launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, kTMax, 1, 64>, a, grid, stream);
    } else {
        // W by batch size (both prepared): 2 waves per SIMD above one wave round
        const bool two = a.B > kNp64OneRound;
        e = hipSuccess;
        if (a.n <= 40) { // CENTAURO-sized (n = 39)
            if (two || a.prepare) e = launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, 2, 2, 40>, a, grid, stream);
            if (e == hipSuccess && (!two || a.prepare))
                e = launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, 2, 1, 40>, a, grid, stream);
        } else {
            if (two || a.prepare) e = launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, 2, 2, 64>, a, grid, stream);
            if (e == hipSuccess && (!two || a.prepare))
                e = launch_one<NP, Lay>(qppvm_fast_kernel<NP, M0, MERGED, 2, 1, 64>, a, grid, stream);
        }
    }
    if (e != hipSuccess) return e;
    if (mid && !a.prepare) { // end of the dominant launch
        e = hipEventRecord(mid, stream);
        if (e != hipSuccess) return e;
    }
    // follow-up kernels: grid-stride over their work lists, grids sized from the last counts seen
    if (MERGED && kInlineRepair<M0> && a.inline_repair && !a.prepare) return hipSuccess; // repaired in the fast kernel
    if (MERGED && a.skip_followup && !a.prepare) return hipSuccess; // on demand: the host completes it
    const unsigned g1 = follow_blocks(a.fg.est[1], IPW, kFollowGrid, a.B);
    if constexpr (MERGED) {
        return launch_one<NP, ActiveLayout<NP>>(qppvm_repair_kernel<NP, M0>, a, g1, stream);
    } else {
        const unsigned g0 = follow_blocks(a.fg.est[0], IPW, kFollowGrid, a.B);
        e = launch_one<NP, ActiveLayout<NP>>(qppvm_active_kernel<NP, M0>, a, g0, stream, true);
        if (e != hipSuccess) return e;
        e = launch_one<NP, ActiveLayout<NP>>(qppvm_repair_kernel<NP, M0>, a, g1, stream);
        if (e != hipSuccess || !(a.handback || a.prepare)) return e;
        // the repaired instances' dual active sets (work list 2), sized like the repair grid
        return launch_one<NP, ActiveLayout<NP>>(qppvm_active_kernel<NP, M0, true>, a, g1, stream, true);
    }
}

}  // namespace

hipError_t launch_qppvm_followup(const QppvmArgs &a, hipStream_t stream)
{
    // (the NP = 32 merged path only: its one follow-up is the repair kernel)
    if (a.n > 32 || a.B <= 0) return hipErrorInvalidValue;
    const unsigned g1 = follow_blocks(a.fg.est[1], 2, kFollowGrid, a.B);
    if (a.m0 <= 6 && a.m_l0 >= a.m0)
        return launch_one<32, ActiveLayout<32>>(qppvm_repair_kernel<32, 6>, a, g1, stream);
    return launch_one<32, ActiveLayout<32>>(qppvm_repair_kernel<32, kM0Max>, a, g1, stream);
}

hipError_t launch_qppvm(const QppvmArgs &a, hipStream_t stream, hipEvent_t mid)
{
    if (a.joint_weight == 1 || a.minnorm) return launch_qppvm_w1m(a, stream, mid);
    // (a middle level, m_l0 < m0, takes the 12-row instantiation: its repair carries the middle step)
    // (both branches: the 6-row instantiation compiles the middle level out, so a split stack of
    // at most 6 rows in total would be solved as one summed level there)
    const bool six = a.m0 <= 6 && a.m_l0 >= a.m0;
    if (a.n <= 32)
        return six ? launch_np<32, 6>(a, stream, mid) : launch_np<32, kM0Max>(a, stream, mid);
    return six ? launch_np<64, 6>(a, stream, mid) : launch_np<64, kM0Max>(a, stream, mid);
}

}  // namespace wbq
