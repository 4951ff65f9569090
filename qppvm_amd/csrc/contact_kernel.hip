// contact_kernel.hip -- batched contact-form (ForceAcc) whole-body QP for gfx950 (MI355X), fp64.
//
// One instance per wave64 block. The math (reference
// src/ForceAcc.cpp; the build's written spec is oracle/wbq_oracle_contact.c):
//   x = [qdd (n); f_c (3) per contact]                                     (:58-72)
//       (wrench_dim 6: w_c = [f_c; m_c], "put 6 for full wrench" :67; every f_c below is then w_c,
//        its box [f_lb, m_lb] <= w_c <= [f_ub, m_ub] and J_c^T w_c runs over all six rows)
//   level 0   min ||J_w qdd - b_w||^2             (waist / pelvis task)       (:118-122)
//   level 1   min ||qdd - b_p||^2 + sum_c ||J_c qdd - b_c||^2 + eps_f ||f||^2 (:83-89, :105-107)
//             s.t. J_w qdd = y0* = b_w (level 0 attained, the generic case)
//   both      M_fb qdd - sum_c J_c[0:3, fb]^T f_c = -h_fb   (DynamicFeasibility, :109-114)
//             f_lb <= f_c <= f_ub for active contacts, f_c = 0 otherwise  (:74-76, :91-95)
//             optional actuated torque rows tau_min <= M_a qdd + h_a - J_ca^T f <= tau_max (a12)
//             optional friction pyramid |f_x| <= mu f_z, |f_y| <= mu f_z per active contact (8f-2)
//   tau = M qdd + h - sum_c J_c^T [f_c; 0]                                  (:206-218)
// with Cartesian acceleration tasks J qdd = Kp e - Kd J qd - Jdot qd and the postural task
// qdd = Kp (q_ref - q) - Kd qd.
//
// Method: Goldfarb-Idnani dual active set carried entirely in constraint space. With
// H = blockdiag(I + sum_c J_c^T J_c, eps_f I) and the m constraint rows A,
//   Gamma = A H^-1 A^T (m x m),  s = A x (m activities),
// one lane per constraint row runs every step: the active-set Gram is Gamma_AA = L L^T with
// T = L^-1 kept in LDS (an add appends one row of T in closed form, a drop re-appends the
// rows after it), and x is rebuilt once at the end from the multipliers,
// x = H^-1 (A^T lambda - g). H^-1 A^T comes from one block Gauss-Jordan on the qdd block of
// H (lane i <-> joint i, the right-hand sides are M's rows and J_w's columns); the force
// block is diagonal. Gamma mixes O(1) acceleration terms with O(1/eps_f) force terms, so the
// active-set arithmetic is only good to ~cond(Gamma) * 1e-16; two steps of iterative
// refinement of (x, lambda) on the final active set, with the residual of the active rows
// taken exactly in x-space, restore full fp64 accuracy (scripts/emulate_contact.py: 1e-5
// relative without, 1e-12 with). A final re-check of every row guards the active set itself.
//
// Torque output: tau_i = (row i of [M | -J_lin^T]) x + h_i from lane i's own M row and
// contact-Jacobian column, held in registers since the stage; only the joint rows that are
// constraints (the 6 floating-base rows, or all with torque rows) are kept in LDS.
//
// Statuses: 0 ok, 1 step cap, 2 infeasible (level 0 not attainable at b_w, or no feasible
// point), 3 numerical. On status != 0: tau = h, x = 0.
#include "wbq_kernels.h"
#include "wbq_device.h"
#include "dual_gi.h"
#include "qppvm_repair.h"
#include "fric_lsi.h"
#include "qr_gi.h"

#include <type_traits>

namespace wbq {
namespace {

// Largest grid of the level-0 repair kernel (grid-stride over its work list; sized per solve from
// the counts of the last solves, FollowGrid in wbq_kernels.h)
constexpr unsigned kContactRepairGrid = 256;

// Per-instance LDS layout in doubles. Compact constraint index ci (= GI lane), NF = wd nc force
// variables (3 forces or the 6-D wrench per contact):
//   ci <  NJ             joint row a = ci (a < 6: dynamic feasibility, an equality;
//                        a >= 6: actuated torque row, only with torque rows, NJ = n)
//   NJ <= ci < NJ + 6    waist row r = ci - NJ (equality, target b_w)
//   NJ + 6 <= ci < NB    force row f = ci - NJ - 6 (box; disabled for inactive contacts)
//   NB <= ci < ME        friction face k = (ci - NB) % 4 of contact (ci - NB) / 4 (with mu > 0):
//                        s f_x - mu f_z <= 0 (k = 0, 1: s = +-1), s f_y - mu f_z <= 0 (k = 2, 3)
// X = H^-1 A_q^T has one column ("slot") per q-bearing row, slot = ci, plus x0 at NJ + 6.
struct ContactLayout {
    int NJ, NR, NF, WD, NB, ME, NX, QS, FS, GS, TS;
    double MU;
    int AQJ, AQW, FFJ, XT, GM, TT, JC, PN, RH, HR, XV, X0, VV, LV, RV, WV, DUM, AC, PS, BT, JD, QD, SIZE;
    // kmr: register slot capacity of the instantiation (0: slot vectors in LDS, as with torque rows)
    __host__ __device__ ContactLayout(int n, int nc, bool tr, int NQ, int NRC, int wd, int nfr, double mu, int kmr)
    {
        NJ = tr ? n : 6;
        NR = NJ + 7;
        WD = wd;
        NF = wd * nc;
        NB = NJ + 6 + NF;
        ME = NB + nfr;
        MU = mu;
        NX = n + NF;
        QS = NQ + 1;          // row stride of NQ-wide rows (odd: lane-per-row reads conflict-free)
        FS = NF + 1;
        GS = ME | 1;
        TS = (NX + 8) | 1;    // the active set never exceeds NX independent rows (+8: chunked dots)
        int o = 0;
        if (!tr) {
            AQJ = o; o += NJ * QS;    // joint constraint rows, acceleration part: M row a
            AQW = o; o += 6 * QS;     // waist rows: J_w row r
        }
        FFJ = o; o += NJ * FS;    // their force part: -J_c[0:3, a] (active contacts)
        XT = o; o += NR * QS;     // X^T: slot s = column s of H^-1 A_q^T over the qdd lanes
        GM = o; o += ME * GS;     // Gamma
        TT = o;                   // T = L^-1 of the active-set Gram, rows of TS
        int ov = 0;               // setup-phase overlays of the TT region
        if (tr) {
            // Torque-row form (LDS-bound occupancy): everything the dual loop does not read lives
            // in the TT region, which the loop only writes after Gamma is assembled. A_q rows
            // (each lane keeps its own row in registers for the loop's activities), task data,
            // the Gauss-Jordan panel; the contact Jacobian rows (dead before the elimination
            // writes X^T) in the X^T region. 64.8 -> 53.3 KB at n = 30, nc = 4: 3 instances per
            // CU instead of 2.
            AQJ = TT + ov; ov += NJ * QS;
            AQW = TT + ov; ov += 6 * QS;
            QD = TT + ov; ov += 64;
            PS = TT + ov; ov += 24 * (1 + nc);
            BT = TT + ov; ov += 6 * (1 + nc);
            JD = TT + ov; ov += 6 * (1 + nc);
            const bool jc_in_xt = 6 * nc * NQ <= NR * QS;
            JC = jc_in_xt ? XT : TT + ov; ov += jc_in_xt ? 0 : 6 * nc * NQ;
            PN = TT + ov; ov += 2 * NQ * kGjBS;   // Gauss-Jordan pivot panel (rows < NQ publish)
            RH = TT + ov; ov += 2 * kGjBS * NRC;  // its right-hand sides
            HR = TT + ov; ov += NQ == 64 ? NQ * QS : 0; // H rows for a second rhs chunk
        } else {
            // The contact Jacobian rows are dead once H is assembled (a barrier precedes the
            // elimination), so the Gauss-Jordan panel reuses them: 22 KB -> 19.6 KB per instance
            // at n = 30, nc = 2, i.e. 8 instances per CU instead of 7
            const int jcs = 6 * nc * NQ, gjs = 2 * NQ * kGjBS + 2 * kGjBS * NRC;
            // (with kmr = 0 the T rows of the loop are written only after these are dead)
            ov = jcs > gjs ? jcs : gjs;
            JC = TT;                  // contact Jacobian rows (steps 1-3)
            PN = TT;                  // Gauss-Jordan pivot panel (rows < NQ publish; step 4)
            RH = TT + 2 * NQ * kGjBS;     // its right-hand sides
            HR = TT;                  // (unused: NQ == 64 && tr only)
        }
        // with torque rows (or kmr = 0) the slot vectors live in LDS: T rows, T columns, Gamma
        // columns (else scratch for the T_E rows and for dual_gi's re-factorisation, KMR rows of
        // KMR + 1; KMR = the register slot capacity of launch_nq)
        const int tt = (tr || kmr == 0) ? NX * TS : (12 * TS > kmr * (kmr + 1) ? 12 * TS : kmr * (kmr + 1));
        o += tt > ov ? tt : ov;
        XV = o; o += 64;          // x
        X0 = o; o += 64;          // x0 = -H^-1 g
        VV = o; o += 72;          // (slot dots read 8 past the active count)
        LV = o; o += 72;
        RV = o; o += 72;
        WV = o; o += 72;
        DUM = o; o += 72;         // row of the lanes that own no slot-vector row
        AC = o; o += 72;          // active constraint (compact index) per slot (+8: chunked gathers)
        if (!tr) {
            PS = o; o += 24 * (1 + nc);      // poses: waist, then contacts ([R|p], ref)
            BT = o; o += 6 * (1 + nc);       // task targets: waist b_w, then b_c
            JD = o; o += 6 * (1 + nc);       // Jdot qd
            QD = o; o += 64;
        }
        SIZE = (o + 1) & ~1;
    }
};

// acceleration part of constraint row ci (nullptr: none, i.e. a force row)
__device__ __forceinline__ const double *row_q(const double *S, const ContactLayout &L, int ci)
{
    if (ci < L.NJ) return S + L.AQJ + ci * L.QS;
    if (ci < L.NJ + 6) return S + L.AQW + (ci - L.NJ) * L.QS;
    return nullptr;
}

// coefficient of friction face k (0..3) on component j (0..2) of its contact's force
__device__ __forceinline__ double fric_coef(int k, int j, double mu)
{
    if (j == 2) return -mu;
    if (j != (k >> 1)) return 0.0;
    return (k & 1) ? -1.0 : 1.0;
}

// force coefficient of row ci on force variable f (FR: the instantiation serves friction rows)
template <bool FR>
__device__ __forceinline__ double fcoef(const double *S, const ContactLayout &L, int ci, int f)
{
    if (ci < L.NJ) return S[L.FFJ + ci * L.FS + f];
    if (ci < L.NJ + 6) return 0.0;
    if (!FR || ci < L.NB) return (ci - L.NJ - 6 == f) ? 1.0 : 0.0;
    const int r = ci - L.NB, c = r >> 2, j = f - L.WD * c;
    return (j >= 0 && j < 3) ? fric_coef(r & 3, j, L.MU) : 0.0;
}

// activity of friction row ci at the force variables xf (= x + n)
__device__ __forceinline__ double fric_activity(const double *xf, const ContactLayout &L, int ci)
{
    const int r = ci - L.NB, c = r >> 2, k = r & 3;
    const double *w = xf + L.WD * c;
    return ((k & 1) ? -1.0 : 1.0) * w[k >> 1] - L.MU * w[2];
}

// activity a_ci . x of constraint row ci at x = XV (n qdd entries, then nf forces); loads
// in chunks of 8 so they issue back to back. NFM: the most force variables of the instantiation
template <int NQ, int NFM, bool FR>
__device__ __forceinline__ double activity(const double *S, const ContactLayout &L, int ci, int n, int nf)
{
    const double *xv = S + L.XV;
    const bool jrow = ci < L.NJ, wrow = !jrow && ci < L.NJ + 6;
    const double *rq = S + (jrow ? L.AQJ + ci * L.QS : (wrow ? L.AQW + (ci - L.NJ) * L.QS : L.AQW));
    double s0 = 0.0, s1 = 0.0; // two accumulators: half the dependent FMA chain
#pragma unroll 1
    for (int j0 = 0; j0 < NQ; j0 += 8) { // chunks of 8 independent loads (entries past n are 0)
        double rv[8], xx[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            rv[u] = rq[j0 + u];
            xx[u] = xv[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            s0 = fma(rv[u], xx[u], s0);
            s1 = fma(rv[u + 1], xx[u + 1], s1);
        }
    }
    const double s = s0 + s1;
    const double *fr = S + L.FFJ + (jrow ? ci : 0) * L.FS;
    double sf0 = 0.0, sf1 = 0.0;
#pragma unroll
    for (int f = 0; f < NFM; ++f) {
        const double t = f < nf ? fr[f] : 0.0, xf = xv[n + (f < nf ? f : 0)];
        if (f & 1) sf1 = fma(t, xf, sf1);
        else sf0 = fma(t, xf, sf0);
    }
    const double sf = sf0 + sf1;
    if (jrow) return s + sf;
    if (wrow) return s;
    if (FR && ci >= L.NB) return fric_activity(xv + n, L, ci);
    return xv[n + ci - L.NJ - 6];
}

// The contact problem for dual_gi: Gamma in LDS, activities from the rows in LDS, and
// x = x0 + H^-1 A^T w with H^-1 A_q^T from the X^T slots and the diagonal force block.
template <int NQ, bool TR, int NFM, bool FR>
struct ContactGi {
    // Gamma mixes O(1) acceleration terms with O(1/eps_f) force terms: a force row's genuine
    // complement can sit ~eps_f below its diagonal, so only roundoff-level ones count as
    // dependent
    static constexpr double kDep = 1e-14;
    static constexpr bool kOwnRowActivity = TR;
    double *S;
    const ContactLayout *L;
    int n, nf, i;
    double ieps;
    int dim; // n + nf
    double aq[TR ? NQ : 1]; // TR: this lane's own A_q row (the LDS rows are overlaid by T)
    __device__ double gamma(int r, int c) const { return S[L->GM + r * L->GS + c]; }
    __device__ double activity(int r) const
    {
        if constexpr (!TR) {
            return wbq::activity<NQ, NFM, FR>(S, *L, r, n, nf);
        } else { // r == this lane's row (dual_gi asks for its own row only)
            const double *xv = S + L->XV;
            const bool jrow = r < L->NJ, wrow = !jrow && r < L->NJ + 6;
            double s0 = 0.0, s1 = 0.0;
#pragma unroll
            for (int j = 0; j < NQ; j += 2) {
                s0 = fma(aq[j], xv[j], s0);
                s1 = fma(aq[j + 1], xv[j + 1], s1);
            }
            const double *fr = S + L->FFJ + (jrow ? r : 0) * L->FS;
            double sf = 0.0;
#pragma unroll
            for (int f = 0; f < NFM; ++f) sf = fma(f < nf ? fr[f] : 0.0, xv[n + (f < nf ? f : 0)], sf);
            if (jrow) return (s0 + s1) + sf;
            if (wrow) return s0 + s1;
            if (FR && r >= L->NB) return fric_activity(xv + n, *L, r);
            return xv[n + r - L->NJ - 6];
        }
    }
    __device__ void rebuild(int pass, int k) const
    {
        if (i >= L->NX) return;
        double dx = 0.0; // slots in chunks of 8 loads
        const int fi = i - n;
        for (int q0 = 0; q0 < k; q0 += 8) {
            int cq[8];
            double wq[8], xq[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                cq[u] = q0 + u < k ? (int)S[L->AC + q0 + u] : 0;
                wq[u] = q0 + u < k ? S[L->RV + q0 + u] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int c = cq[u] < L->NJ + 6 ? cq[u] : 0;
                xq[u] = i < n ? (cq[u] < L->NJ + 6 ? S[L->XT + c * L->QS + i] : 0.0) : fcoef<FR>(S, *L, cq[u], fi < 0 ? 0 : fi);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) dx = fma(wq[u], xq[u], dx);
        }
        if (i >= n) dx *= ieps;
        S[L->XV + i] = (pass == 0 ? (i < n ? S[L->X0 + i] : 0.0) : S[L->XV + i]) + dx;
    }
};

// The contact problem for the QR-form fallback (qr_gi.h): row normals a_ci = [A_q row; force
// coefficients] and H^-1 a_ci = [X^T slot ci; force coefficients / eps_f] (the same data the
// constraint-space loop reads), activities through the ContactGi rows.
template <int NQ, bool TR, int NFM, bool FR>
struct ContactQr {
    const ContactGi<NQ, TR, NFM, FR> *gi;
    double *S;
    const ContactLayout *L;
    int n, nf, i, nx, dim, m;
    double ieps;
    __device__ double own_activity() const { return gi->activity(i); }
    __device__ double own_norm2() const
    {
        double q2 = 0.0;
        if constexpr (TR) {
#pragma unroll
            for (int j = 0; j < NQ; ++j) q2 = fma(gi->aq[j], gi->aq[j], q2);
        } else {
            const double *rq = row_q(S, *L, i);
            if (rq)
                for (int j = 0; j < n; ++j) q2 = fma(rq[j], rq[j], q2);
        }
        for (int f = 0; f < nf; ++f) {
            const double c = fcoef<FR>(S, *L, i, f);
            q2 = fma(c, c, q2);
        }
        return q2;
    }
    __device__ void normal(int p, double sg, double *ap, double *hp) const
    {
        const bool qb = p < L->NJ + 6; // a joint or waist row: it has an acceleration part
        if constexpr (TR) { // the acceleration part lives in row p's own lane (registers)
            if (i == p) {
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    if (j < n) ap[j] = qb ? sg * gi->aq[j] : 0.0;
            }
        } else if (i < n) {
            const double *rq = row_q(S, *L, p);
            ap[i] = rq ? sg * rq[i] : 0.0;
        }
        if (i < n) hp[i] = qb ? sg * S[L->XT + p * L->QS + i] : 0.0;
        if (i >= n && i < nx) {
            const double c = sg * fcoef<FR>(S, *L, p, i - n);
            ap[i] = c;
            hp[i] = c * ieps;
        }
        if (i >= nx) {
            ap[i] = 0.0;
            hp[i] = 0.0;
        }
    }
};

// compact index of equality a (a < 6: dynamic feasibility rows, then the waist rows)
__device__ __forceinline__ int eq_row(int a, int NJ) { return a < 6 ? a : NJ + a - 6; }

// Level 0 of the contact form when the waist task cannot be met at b_w (ForceAcc.cpp:131-137,189:
// QPOases_sot solves waist / (postural + feet), so level 1 keeps the waist at its level-0 optimum
// y0*). With tau = M qdd + h - sum_c J_c^T [f_c; 0], dynamic feasibility is tau_fb = 0 and every
// other row is a box in z = (tau_a, f): qdd = M^-1 (S_a^T tau_a - h + J_c,lin^T f), so level 0 is
//   min 0.5 ||A0 z - (b_w + W^T h)||^2,  lo_z <= z <= hi_z,   W = M^-1 J_w^T,
//   A0 columns: tau_a -> row a of W;  f_ck -> W^T J_c[k]^T
// (without torque rows tau_a is unbounded). BVLS (the QPPVM level-0 repair's, qppvm_repair.h)
// gives z*; y0* = A0 z* - W^T h becomes the waist rows' target, and every variable the level-0
// gradient w = A0^T (b - A0 z*) holds at a bound is pinned there (its torque or force row becomes an
// equality), as oracle/wbq_oracle.c:wbq_ref_qppvm_one pins for the QPPVM form. The oracle
// (oracle/wbq_oracle_contact.c:wbq_ref_contact_one) reaches y0* through a 1e-10 ridge instead:
// the same optimum, to the ridge. Lane roles: joint lane i < n for W; variable lane
// j < n - 6 = tau_{6+j}, then the 3 nc forces; constraint lane ci for the targets and the pins.
// The waist rows and the pins are dependent on the level-0 face: y - y0* = A0 (z - z*) moves only
// along the unpinned columns, so only a pivot basis of their span (wkeep: a mask of waist rows,
// from a pivoted Cholesky of their Gram) is kept as level-1 rows -- the others are implied, and
// keeping them makes the final active set exactly singular.
// Friction rows (mu > 0, FR instantiations) are general rows in z: level 0 is then an LSI over the
// box and the pyramid faces (fric_lsi.h, BVLS generalised to the faces; the oracle keeps the friction
// rows in its level-0 QP, oracle/wbq_oracle_contact.c:413-447), and the faces its multipliers hold
// are pinned as equalities of level 1 like the box sides. (Until round 4 the BVLS ran on the box
// alone and an instance whose level-0 point violated a face ended with status 2)
// Updates this lane's row limits (lo, hi); returns the level-0 iterations, capped = the cap ended it.
template <int NQ, bool FR>
__device__ int contact_level0(const ContactArgs &a, long b, double *S, const ContactLayout &L, int i, double h_i,
                              double &lo, double &hi, bool &capped, int &wkeep)
{
    const int n = a.n, nc = a.nc, wd = L.WD, nf = L.NF, na = n - 6;
    const bool qrow = i < n;
    const int ic = qrow ? i : n - 1;
    const long B = a.B;
    // W = M^-1 J_w^T, lane i holding row i: block Gauss-Jordan on M's rows (re-read: L2) with the
    // J_w columns as right-hand sides; the pivot panel in the T region (not written yet)
    double A[NQ], w[6];
    {
        const __amdgpu_buffer_rsrc_t Mrs = rsrc_at(a.M, b, B, (long)n * n);
        const __amdgpu_buffer_rsrc_t Wrs = rsrc_at(a.Jw, b, B, 6L * n);
#pragma unroll
        for (int r = 0; r < NQ; ++r) A[r] = bload(Mrs, (int)(8 * ic), 8 * (r < n ? r : n - 1) * n);
#pragma unroll
        for (int r = 0; r < 6; ++r) w[r] = bload(Wrs, (int)(8 * ic), 8 * r * n);
#pragma unroll
        for (int r = 0; r < NQ; ++r) A[r] = (qrow && r < n) ? A[r] : (r == i ? 1.0 : 0.0);
#pragma unroll
        for (int r = 0; r < 6; ++r) w[r] = qrow ? w[r] : 0.0;
    }
    wave_sync();
    (void)block_gj<NQ, 6, 6>(A, w, n, i, S + L.PN, S + L.RH);
    // b = b_w + W^T h (the waist targets are the waist rows' limits)
    double bv[6], hw[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        hw[r] = isum<64>(qrow ? w[r] * h_i : 0.0);
        bv[r] = __shfl(lo, L.NJ + r) + hw[r];
    }
    // the columns of A0 on the variable lanes
    const bool tvar = i < na, fvar = i >= na && i < na + nf;
    const int f = fvar ? i - na : 0;
    double acol[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) acol[r] = __shfl(w[r], tvar ? 6 + i : 0);
    {
        const __amdgpu_buffer_rsrc_t Jrs = rsrc_at(a.Jc, b, B, (long)nc * 6 * n);
        for (int ff = 0; ff < nf; ++ff) {
            const int c = ff / wd, k = ff - wd * c;
            const double jv = bload(Jrs, (int)(8 * ic), 8 * (6 * c + k) * n);
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                const double v = isum<64>(qrow ? w[r] * jv : 0.0);
                if (fvar && f == ff) acol[r] = v;
            }
        }
    }
    double zlo = 0.0, zhi = 0.0;
    if (tvar) {
        zlo = a.torque_rows ? a.tau_min[6 + i] : -kInf;
        zhi = a.torque_rows ? a.tau_max[6 + i] : kInf;
    } else if (fvar) {
        const int k = f % wd;
        const bool on = (a.cmask[b] >> (f / wd)) & 1;
        double fl = a.w_lb[0], fu = a.w_ub[0];
#pragma unroll
        for (int kk = 1; kk < 6; ++kk) {
            fl = k == kk ? a.w_lb[kk] : fl;
            fu = k == kk ? a.w_ub[kk] : fu;
        }
        zlo = on ? fl : 0.0; // an inactive contact's forces are fixed at zero
        zhi = on ? fu : 0.0;
    }
    const bool row = tvar || fvar;
    const int maxit = 50 * (na + nf) + 100;
    double xz, mcol[6]; // z_i; the part of this lane's column level 1 can still move along
    int pin, pfm = 0, itz;
    bool capz;
    if (FR && a.nfr > 0) { // box + pyramid faces: the friction groups are the active contacts' forces
        const int fc = fvar ? f / wd : 0, fk = fvar ? f - wd * fc : 3;
        const bool on = (a.cmask[b] >> fc) & 1;
        const int gb = (fvar && fk < 3 && on) ? na + wd * fc : -1;
        const LsiOut lz = fric_lsi<64, 6>(acol, bv, 6, zlo, zhi, row, gb, L.MU, maxit);
        xz = lz.xv;
        pin = lz.pin;
        pfm = lz.pfm;
        itz = lz.it;
        capz = lz.capped;
#pragma unroll
        for (int r = 0; r < 6; ++r) mcol[r] = lz.mcol[r];
    } else {
        const BvlsOut bz = bvls<64, 6>(acol, bv, 6, zlo, zhi, row, true, 0, maxit);
        xz = bz.xv;
        itz = bz.it;
        capz = bz.capped;
        double g = 0.0, abm = 0.0, yv[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) yv[r] = isum<64>(row ? acol[r] * xz : 0.0);
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            abm = fma(acol[r], bv[r], abm);
            g = fma(acol[r], bv[r] - yv[r], g);
        }
        abm = fmax(1.0, imax<64>(row ? fabs(abm) : 0.0));
        pin = (row && g > 1e-9 * abm) ? 1 : ((row && g < -1e-9 * abm) ? -1 : 0);
        const bool mov = row && pin == 0 && zlo != zhi; // columns y can still move along
#pragma unroll
        for (int r = 0; r < 6; ++r) mcol[r] = mov ? acol[r] : 0.0;
    }
    double ys[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) ys[r] = isum<64>(row ? acol[r] * xz : 0.0);
    {
        constexpr int NT = 21;
        double gu[NT];
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
            for (int c = 0; c <= p; ++c) gu[tri(p, c)] = acol[p] * mcol[c];
        isum_vec<64, NT>(gu);
        PivChol<6> pc;
        pc.factor(gu, 6, 1e-10);
        wkeep = 0;
#pragma unroll
        for (int c = 0; c < 6; ++c) wkeep |= (c < pc.k) ? (1 << pc.piv[c]) : 0;
    }
    // constraint lanes: torque row a <-> variable a - 6, force row <-> variable na + its force
    const int ci = i;
    const bool trow = ci >= 6 && ci < L.NJ, frow = ci >= L.NJ + 6 && ci < L.NB;
    const int pin_c = __shfl(pin, trow ? ci - 6 : (frow ? na + ci - L.NJ - 6 : 0));
    if ((trow || frow) && pin_c > 0) lo = hi; // held at the upper limit
    if ((trow || frow) && pin_c < 0) hi = lo; // held at the lower limit
    if (FR && a.nfr > 0) { // friction face r & 3 of contact r >> 2: held at 0 by a positive multiplier
        const bool fface = ci >= L.NB && ci < L.ME;
        const int r = fface ? ci - L.NB : 0;
        const int pf = __shfl(pfm, na + wd * (r >> 2));
        if (fface && ((pf >> (r & 3)) & 1)) lo = hi;
    }
    if (ci >= L.NJ && ci < L.NJ + 6) {
        double y = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) y = (ci - L.NJ == r) ? ys[r] - hw[r] : y;
        lo = hi = y; // the waist rows keep the level-0 optimum y0*
    }
    capped = capz;
    return itz;
}

// The whole solve of instance b by one wave (lane i = threadIdx.x). REPAIR (the follow-up
// kernel): level 0 first (contact_level0: BVLS for y0*, pins), then level 1 with those targets.
// KMR: register slot capacity (12 + the most force variables; 0 = slot vectors in LDS), WD: wrench
// components per contact (3 or 6)
template <int NQ, bool TR, int KMR, int WD, bool REPAIR>
__device__ __forceinline__ void contact_solve(const ContactArgs &a, const long b)
{
    constexpr int NRC = TR ? 40 : 16; // Gauss-Jordan right-hand sides per pass
    // the most contacts this instantiation serves (register slots: KMR = 12 + WD * CM, launch_nq):
    // with 2 the stage issues 12 contact-Jacobian loads per lane instead of 24 (a wave's loads stay
    // under the 63 outstanding vector memory operations, as the QPPVM fast kernel's TM)
    constexpr int CM = (!TR && KMR > 0 && KMR <= 12 + 2 * WD) ? 2 : kCMax;
    constexpr int NFM = WD * CM; // the most force variables
    // friction rows only in the LDS-slot instantiations (their ME exceeds the register slots); the
    // register ones carry none of that code (launch_wd routes mu > 0 to LDS slots)
    constexpr bool FR = TR || KMR == 0;
    extern __shared__ __attribute__((aligned(16))) double S[];
    const int n = a.n, nc = a.nc, nf = WD * nc;
    const ContactLayout L(n, nc, TR, NQ, NRC, WD, FR ? a.nfr : 0, a.mu, TR ? 0 : KMR);
    const int i = threadIdx.x;
    const int cm = a.cmask[b];
    const bool qrow = i < n;
    const int ic = qrow ? i : n - 1;
    WBQ_STAMP(0);

    // ------------------------------------------------------------------ 1. stage
    // unconditional buffer loads (clamped offsets, values selected afterwards): one HBM trip
    // buffer resources start at this block's instance: per-lane offsets stay small
    const long B = a.B;
    const int voff = (int)(8 * ic);
    const double q_i = bload(rsrc_at(a.q, b, B, n), voff, 0), qd_i = bload(rsrc_at(a.qd, b, B, n), voff, 0);
    const double qref_i = bload(rsrc_at(a.qref, b, B, n), voff, 0), h_i0 = bload(rsrc_at(a.h, b, B, n), voff, 0);
    // torque-row variants: M last, its issue order pinned (vmcnt retires in order), so the task
    // targets and H (steps 2-3, no M) run while M streams in, and M enters LDS only before the
    // elimination reads it. Same box: config 2 (torque rows) 5.80 -> 6.17 M QP/s, the variant's
    // spill gone; the register-slot variants lost 4-8 % with it (M live through steps 2-3)
    constexpr bool kMLate = TR;
    double mrow[NQ]; // M is symmetric: lane i's row is its column, so the loads coalesce
    if constexpr (!kMLate) {
        const __amdgpu_buffer_rsrc_t Mrs = rsrc_at(a.M, b, B, (long)n * n);
        const int moff = (int)(8 * ic);
#pragma unroll
        for (int r = 0; r < NQ; ++r) mrow[r] = bload(Mrs, moff, 8 * (r < n ? r : n - 1) * n);
    }
    double jc[6 * CM], jw[6];
    {
        const __amdgpu_buffer_rsrc_t Jrs = rsrc_at(a.Jc, b, B, (long)nc * 6 * n);
        const int joff = (int)(8 * ic);
#pragma unroll
        for (int rr = 0; rr < 6 * CM; ++rr) jc[rr] = bload(Jrs, joff, 8 * (rr < 6 * nc ? rr : 6 * nc - 1) * n);
        const __amdgpu_buffer_rsrc_t Wrs = rsrc_at(a.Jw, b, B, 6L * n);
        const int woff = (int)(8 * ic);
#pragma unroll
        for (int r = 0; r < 6; ++r) jw[r] = bload(Wrs, woff, 8 * r * n);
    }
    constexpr int kPoseIt = (24 * (1 + CM) + 63) / 64;
    double pv[kPoseIt];
#pragma unroll
    for (int it = 0; it < kPoseIt; ++it) {
        int e = it * 64 + i;
        e = e < 24 * (1 + nc) ? e : 24 * (1 + nc) - 1;
        const int t = e / 24, c = e - t * 24;
        if (t == 0) pv[it] = c < 12 ? a.pose_w[b * 12 + c] : a.pose_w_ref[b * 12 + c - 12];
        else pv[it] = c < 12 ? a.pose_c[(b * nc + t - 1) * 12 + c] : a.pose_c_ref[(b * nc + t - 1) * 12 + c - 12];
    }
    double jd = 0.0;
    if (i < 6 * (1 + nc)) jd = i < 6 ? a.jdqd_w[b * 6 + i] : a.jdqd_c[b * nc * 6 + i - 6];
    if constexpr (kMLate) {
        __builtin_amdgcn_sched_barrier(0);
        const __amdgpu_buffer_rsrc_t Mrs = rsrc_at(a.M, b, B, (long)n * n);
        const int moff = (int)(8 * ic);
#pragma unroll
        for (int r = 0; r < NQ; ++r) mrow[r] = bload(Mrs, moff, 8 * (r < n ? r : n - 1) * n);
        __builtin_amdgcn_sched_barrier(0);
    }
    const double h_i = qrow ? h_i0 : 0.0;
#pragma unroll
    for (int rr = 0; rr < 6 * CM; ++rr) jc[rr] = (qrow && rr < 6 * nc) ? jc[rr] : 0.0;
#pragma unroll
    for (int r = 0; r < 6; ++r) jw[r] = qrow ? jw[r] : 0.0;
    if (i < L.NJ) { // joint constraint rows (every joint with torque rows, else the 6 base rows)
        if constexpr (!kMLate) {
#pragma unroll
            for (int r = 0; r < NQ; ++r) S[L.AQJ + i * L.QS + r] = (qrow && r < n) ? mrow[r] : 0.0;
        }
#pragma unroll
        for (int f = 0; f < NFM; ++f)
            if (f < nf) S[L.FFJ + i * L.FS + f] = ((cm >> (f / WD)) & 1) ? -jc[6 * (f / WD) + f % WD] : 0.0;
    }
    if (i < NQ) {
#pragma unroll
        for (int r = 0; r < 6; ++r) S[L.AQW + r * L.QS + i] = jw[r];
#pragma unroll
        for (int rr = 0; rr < 6 * CM; ++rr)
            if (rr < 6 * nc) S[L.JC + rr * NQ + i] = jc[rr];
    }
    S[L.QD + i] = qrow ? qd_i : 0.0;
#pragma unroll
    for (int it = 0; it < kPoseIt; ++it)
        if (it * 64 + i < 24 * (1 + nc)) S[L.PS + it * 64 + i] = pv[it];
    if (i < 6 * (1 + nc)) S[L.JD + i] = jd;
    if constexpr (kMLate) lds_barrier(); // (LDS only: M keeps streaming in)
    else wave_sync();
    WBQ_STAMP(1);

    // ------------------------------------------------- 2. task targets (one lane per row)
    // Cartesian acceleration task: b = Kp e - Kd J qd - Jdot qd (xdd_ref = 0, xd_ref = 0)
    if (i < 6 * (1 + nc)) {
        const int t = i / 6, r = i - 6 * t;
        const double *Jr = t == 0 ? S + L.AQW + r * L.QS : S + L.JC + (6 * (t - 1) + r) * NQ;
        double xd = 0.0;
        for (int j = 0; j < n; ++j) xd = fma(Jr[j], S[L.QD + j], xd);
        const double e = cart_error_component(S + L.PS + 24 * t, S + L.PS + 24 * t + 12, r);
        const double Kp = t == 0 ? a.Kp_w : a.Kp_f, Kd = t == 0 ? a.Kd_w : a.Kd_f;
        S[L.BT + i] = Kp * e - Kd * xd - S[L.JD + i];
    }
    if constexpr (kMLate) lds_barrier();
    else wave_sync();

    // ------------------------------- 3. H row i = e_i + sum_c J_c^T J_c row i, gradient
    double A[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) A[j] = (j == i) ? 1.0 : 0.0;
    double mg = qrow ? a.Kp_p * (qref_i - q_i) - a.Kd_p * qd_i : 0.0; // -g_i = b_p + sum J_c^T b_c
#pragma unroll
    for (int rr = 0; rr < 6 * CM; ++rr) {
        if (rr < 6 * nc) {
            const double v = jc[rr];
            const double *Jr = S + L.JC + rr * NQ;
#pragma unroll
            for (int j = 0; j < NQ; ++j) A[j] = fma(v, Jr[j], A[j]);
            mg = fma(v, S[L.BT + 6 + rr], mg);
        }
    }
    if constexpr (NQ == 64 && TR) {
#pragma unroll
        for (int j = 0; j < NQ; ++j) S[L.HR + i * L.QS + j] = A[j];
    }

    if constexpr (kMLate) { // the joint constraint rows' M part (M arrives here)
        if (i < L.NJ) {
#pragma unroll
            for (int r = 0; r < NQ; ++r) S[L.AQJ + i * L.QS + r] = (qrow && r < n) ? mrow[r] : 0.0;
        }
        lds_barrier();
    }
    WBQ_STAMP(2);
    // ------------- 4. X = H_qq^-1 [M rows 0..NJ-1 | J_w^T | -g]: block Gauss-Jordan, H SPD
    bool notspd = false;
    for (int c0 = 0; c0 < L.NR; c0 += NRC) {
        if constexpr (NQ == 64 && TR) {
            if (c0 > 0) {
#pragma unroll
                for (int j = 0; j < NQ; ++j) A[j] = S[L.HR + i * L.QS + j];
            }
        }
        double rhs[NRC];
#pragma unroll
        for (int m = 0; m < NRC; ++m) {
            const int s = c0 + m;
            double v = 0.0;
            if (s < L.NJ) v = S[L.AQJ + s * L.QS + (i < NQ ? i : 0)]; // M[s][i] = M[i][s]
            else if (s < L.NJ + 6) v = S[L.AQW + (s - L.NJ) * L.QS + (i < NQ ? i : 0)];
            else if (s == L.NJ + 6) v = mg;
            rhs[m] = qrow ? v : 0.0;
        }
        wave_sync();
        notspd |= block_gj<NQ, NRC, NRC>(A, rhs, n, i, S + L.PN, S + L.RH);
        if (i < NQ) {
#pragma unroll
            for (int m = 0; m < NRC; ++m)
                if (c0 + m < L.NR) S[L.XT + (c0 + m) * L.QS + i] = rhs[m];
        }
    }
    wave_sync();
    {
        const double x0 = qrow ? S[L.XT + (L.NJ + 6) * L.QS + i] : 0.0;
        S[L.X0 + i] = x0;
        S[L.XV + i] = x0;
    }

    WBQ_STAMP(3);
    // ------------------------------------------ 5. Gamma row ci, activities, bounds
    const int ci = i;
    const int NJ = L.NJ, ME = L.ME;
    int kind = 0; // 0 disabled, 1 equality, 2 inequality (lo <= a x <= hi)
    double lo = -kInf, hi = kInf;
    if (ci < NJ) {
        if (ci < 6) {
            kind = 1;
            lo = hi = -h_i; // M_fb qdd - J_fb^T f = -h_fb
        } else {
            kind = 2;
            lo = a.tau_min[ci] - h_i;
            hi = a.tau_max[ci] - h_i;
        }
    } else if (ci < NJ + 6) {
        kind = 1;
        lo = hi = S[L.BT + ci - NJ];
    } else if (ci < L.NB) {
        const int f = ci - NJ - 6, c = f / WD, k = f - WD * c;
        if ((cm >> c) & 1) {
            kind = 2;
            lo = a.w_lb[0];
            hi = a.w_ub[0];
#pragma unroll
            for (int kk = 1; kk < WD; ++kk) { // (selects: no dynamic index into the kernel arguments)
                lo = k == kk ? a.w_lb[kk] : lo;
                hi = k == kk ? a.w_ub[kk] : hi;
            }
        }
    } else if (FR && ci < ME) { // friction face: one-sided
        if ((cm >> ((ci - L.NB) >> 2)) & 1) {
            kind = 2;
            hi = 0.0;
        }
    }
    const double ieps = 1.0 / a.eps_f;
    double s_i = 0.0, nrm = 1.0;
    double aq[NQ]; // this lane's acceleration row (kept in registers for the TR loop)
#pragma unroll
    for (int j = 0; j < NQ; ++j) aq[j] = 0.0;
    if (kind != 0) {
        double fc[NFM];
        const double *rq = row_q(S, L, ci);
#pragma unroll
        for (int j = 0; j < NQ; ++j) aq[j] = rq ? rq[j] : 0.0;
#pragma unroll
        for (int f = 0; f < NFM; ++f) fc[f] = f < nf ? fcoef<FR>(S, L, ci, f) : 0.0;
        for (int cl = 0; cl < ME; ++cl) {
            double g = 0.0;
            if (cl < NJ + 6) { // four accumulators: the dot was a 32-long dependent FMA chain per entry
                const double *xt = S + L.XT + cl * L.QS;
                double g4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int j = 0; j < NQ; ++j) g4[j & 3] = fma(aq[j], xt[j], g4[j & 3]);
                g = (g4[0] + g4[1]) + (g4[2] + g4[3]);
            }
            double gf = 0.0;
            if (cl < NJ) {
                const double *fr = S + L.FFJ + cl * L.FS;
#pragma unroll
                for (int f = 0; f < NFM; ++f)
                    if (f < nf) gf = fma(fc[f], fr[f], gf);
            } else if (FR && cl >= L.NB) { // friction row cl: its three force coefficients
                const int r = cl - L.NB, c0 = WD * (r >> 2);
#pragma unroll
                for (int f = 0; f < NFM; ++f) {
                    const int j = f - c0;
                    if (j >= 0 && j < 3) gf = fma(fc[f], fric_coef(r & 3, j, L.MU), gf);
                }
            } else if (cl >= NJ + 6) {
                const int fl = cl - NJ - 6;
#pragma unroll
                for (int f = 0; f < NFM; ++f)
                    if (f == fl) gf = fc[f];
            }
            S[L.GM + ci * L.GS + cl] = fma(gf, ieps, g);
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) s_i = fma(aq[j], S[L.X0 + j], s_i);
    }
    wave_sync();
    if (kind != 0) nrm = sqrt(fmax(S[L.GM + ci * L.GS + ci], 1e-300));
    WBQ_STAMP(4);
    int it0 = 0;
    bool l0cap = false;
    int wkeep = 0x3f; // waist rows kept as level-1 rows (all, except after a level-0 repair)
    const double lo_free = lo, hi_free = hi, s_x0 = s_i; // (a repair retry restarts from these)
    const int kind_free = kind;
    (void)kind_free;
    if constexpr (REPAIR) { // level 0 not attainable at b_w: y0* and the pins first
        if (!notspd && !a.limits_crossed) it0 = contact_level0<NQ, FR>(a, b, S, L, i, h_i, lo, hi, l0cap, wkeep);
        wave_sync();
    }
    const double lo_rep = lo, hi_rep = hi; // the pinned level 1 (the QR fallback's problem)
    const int wkeep_rep = wkeep;

    // ------------------------------------ 6. dual active set in constraint space
    // Slot a (lane a < k) = a-th active row: act (compact row), sgn (normal = sgn * a_act),
    // lam (its multiplier), aeq (an equality, never dropped), row a and column a of
    // T = L^-1 (Gamma_AA = L L^T, signed normals). Lane j (constraint row j) keeps its
    // activity s_j and GA_j[q] = Gamma[j][act_q].
    // without torque rows the active rows are the 12 equalities and independent rows of the
    // force space: k <= 12 + WD nc <= KMR, in registers (KMR = 0: in LDS, as with torque rows)
    constexpr bool SREG = !TR && KMR > 0;
    constexpr int KM = SREG ? KMR : 64;
    using TcolT = typename std::conditional<SREG, SlotVec<KM, true>, TColView>::type;
    using GAT = typename std::conditional<SREG, SlotVec<KM, true>, GAView>::type;
    SlotVec<KM, SREG> Trow;
    TcolT Tcol;
    GAT GA;
    if constexpr (!SREG) {
        Trow.bind(S + (i < L.NX ? L.TT + i * L.TS : L.DUM), L.NX);
        Tcol.bind(S + L.TT + (i < L.NX ? i : 0), L.TS);
        GA.bind(S + L.GM + (ci < ME ? ci : 0) * L.GS, S + L.AC);
    }
    GiState gs; // slots: act = compact row
    // the repair kernel's level 1: the pinned rows and the waist at y0* are exactly dependent on the
    // level-0 face; if that solve fails numerically (status 1 or 3) it runs once more without the
    // pins (the waist rows at y0* alone keep level 1 on the face)
    constexpr int kAttempts = REPAIR ? 2 : 1;
#pragma unroll 1
    for (int attempt = 0; attempt < kAttempts; ++attempt) {
    if (attempt > 0) {
        if (ci < NJ || ci >= NJ + 6) {
            lo = lo_free;
            hi = hi_free;
        }
        wkeep = 0x3f;
        s_i = s_x0;
        wave_sync();
    }
    if constexpr (REPAIR) kind = (ci >= NJ && ci < NJ + 6 && !((wkeep >> (ci - NJ)) & 1)) ? 0 : kind_free;
    // batch row c: the dynamic-feasibility rows, then the kept waist rows; nb of them (12 but
    // after a repair)
    const int nb = REPAIR ? 6 + __popc((unsigned)wkeep) : 12;
    auto brow = [&](int c) {
        if constexpr (!REPAIR) {
            return eq_row(c, NJ);
        } else {
            if (c < 6) return c;
            unsigned m = (unsigned)wkeep;
            for (int j = 6; j < c && j < 12; ++j) m &= m - 1;
            return m ? NJ + __builtin_ctz(m) : NJ;
        }
    };
    Trow.zero_from(0);
    Tcol.zero_from(0);
    GA.zero_from(0);
    gs = GiState();
    gs.status = notspd ? 3 : (a.limits_crossed ? 2 : (l0cap ? 1 : 0));
    // rank cap of the loop: the rows never touch the forces of inactive contacts (their rows
    // are disabled, their joint-row coefficients zero), so the rows span at most
    // n + WD * (active contacts) dimensions, not nx
    const int dim = n + WD * __popc((unsigned)cm & ((1u << nc) - 1u));
    ContactGi<NQ, TR, NFM, FR> pb{S, &L, n, nf, i, ieps, dim};
    if constexpr (TR) {
#pragma unroll
        for (int j = 0; j < NQ; ++j) pb.aq[j] = aq[j];
    }
    const GiVecs gv{L.VV, L.LV, L.RV, L.WV, L.AC, L.TT, SREG ? KMR + 1 : L.TS};
    if (gs.status == 0) {
        // The 12 equality rows in one batch. Lane r < 12 holds row r of Gamma_EE; a
        // right-looking Cholesky runs across the lanes (pivots and columns by readlane), lane
        // c then forward-substitutes column c of T = L^-1 against the broadcast rows of L, and
        // lambda_E = T^T T (e_E - s_E), s += Gamma[:, E] lambda_E.
        // (rows past nb: identity, decoupled, never active)
        const int er = brow(i < nb ? i : 0);
        double g[12];
#pragma unroll
        for (int c = 0; c < 12; ++c)
            g[c] = (i < nb && c < nb) ? S[L.GM + er * L.GS + brow(c)] : ((i == c && i < 12) ? 1.0 : 0.0);
        double gd = 0.0;
#pragma unroll
        for (int c = 0; c < 12; ++c) gd = (i == c && i < nb) ? g[c] : gd;
        const double dmx = imax<64>(gd);
        bool sing = false;
#pragma unroll
        for (int c = 0; c < 12; ++c) {
            const double dcc = bcast(g[c], c);
            sing |= !(dcc > 1e-14 * dmx);
            const double ilc = dcc > 0.0 ? frsq(dcc) : 0.0;
            g[c] = (i > c) ? g[c] * ilc : ((i == c) ? dcc * ilc : g[c]); // L[r][c], r >= c
#pragma unroll
            for (int j = c + 1; j < 12; ++j) {
                const double ljc = bcast(g[c], j);
                if (i >= j) g[j] = fma(-g[c], ljc, g[j]);
            }
        }
        double t[12]; // column i of T (lanes i < 12)
#pragma unroll
        for (int r = 0; r < 12; ++r) {
            double acc = (i == r) ? 1.0 : 0.0;
#pragma unroll
            for (int q = 0; q < r; ++q) acc = fma(-bcast(g[q], r), t[q], acc);
            const double lrr = bcast(g[r], r);
            t[r] = (i < 12 && lrr > 0.0) ? acc / lrr : 0.0;
        }
        // column i of T to lane i's Tcol; rows through LDS (lane c writes T[r][c] into row r
        // of the TT region: the LDS Trow itself, or scratch for the register Trow)
#pragma unroll
        for (int r = 0; r < 12; ++r) {
            const double tr = (i < nb && r < nb) ? t[r] : 0.0;
            Tcol.put(r, i < 12, tr);
            if (i < 12) S[L.TT + r * L.TS + i] = tr;
        }
        const double ye = __shfl(lo - s_i, er); // e_E - s_E (every lane active: sources up to lane NJ + 5)
        if (i < 12) S[L.VV + i] = i < nb ? ye : 0.0;
        S[L.AC + i] = (double)er; // slots 0..nb-1 (the gathered Gamma columns of the LDS variant)
        wave_sync();
        if constexpr (SREG) Trow.load_if(i < nb, S + L.TT + (i < nb ? i : 0) * L.TS, nb);
        const double w = i < nb ? Trow.dot(S + L.VV, nb) : 0.0;
        S[L.LV + i] = w;
        wave_sync();
        const double lm = i < nb ? Tcol.dot(S + L.LV, nb) : 0.0; // lambda_E
        S[L.RV + i] = lm;
        wave_sync();
#pragma unroll
        for (int q = 0; q < 12; ++q)
            GA.put(q, kind != 0, (kind != 0 && q < nb) ? S[L.GM + ci * L.GS + brow(q)] : 0.0);
        if (kind != 0) s_i += GA.dot(S + L.RV, nb);
        if (i < nb) {
            gs.act = er;
            gs.aeq = true;
            gs.lam = lm;
        }
        gs.onact = ci < 6 || (ci >= NJ && ci < NJ + 6 && (!REPAIR || ((wkeep >> (ci - NJ)) & 1)));
        gs.k = nb;
        gs.iters = 1;
        if (sing) gs.status = 3; // dependent equality rows: the spec's level 1 is ill-posed
        wave_sync();
    }
    WBQ_STAMP(9); // (diagnostic build: the equality batch ends here)
    if constexpr (!REPAIR) { // the last solve's active inequality rows on top (dual_gi.h warm_extend)
        if (gs.status == 0 && a.ws_rows) {
            const int wsg = kind == 2 ? (int)a.ws_rows[b * 64 + i] : 0;
            (void)warm_extend<KM>(pb, S, gv, i, Trow, Tcol, GA, kind, lo, hi, s_i, gs, wsg);
        }
    }
    WBQ_STAMP(8);
    dual_gi<KM>(pb, S, gv, i, Trow, Tcol, GA, kind, lo, hi, nrm, s_i, gs, a.max_iter);
    if (gs.status != 1 && gs.status != 3) break;
    }
    int status = gs.status;
    int iters = gs.iters + it0;
    if constexpr (REPAIR) {
        // The constraint-space loop failed on the pinned level 1 (and on the retry without the pins):
        // near a degenerate vertex its Gamma complements cannot tell dependent rows from independent
        // ones. The QR-form loop (qr_gi.h) solves the same pinned problem from x0 with an
        // explicit basis of the active normals. Its LDS follows the layout (a.qr_fallback: it fits).
        if (status != 0 && a.qr_fallback && !notspd && !a.limits_crossed && !l0cap) {
            const int kp = (ci >= NJ && ci < NJ + 6 && !((wkeep_rep >> (ci - NJ)) & 1)) ? 0 : kind_free;
            if (i < L.NX) S[L.XV + i] = i < n ? S[L.X0 + i] : 0.0;
            wave_sync();
            const int dim = n + WD * __popc((unsigned)cm & ((1u << nc) - 1u));
            ContactGi<NQ, TR, NFM, FR> gi{S, &L, n, nf, i, ieps, dim};
            if constexpr (TR) {
#pragma unroll
                for (int j = 0; j < NQ; ++j) gi.aq[j] = aq[j];
            }
            const ContactQr<NQ, TR, NFM, FR> pq{&gi, S, &L, n, nf, i, L.NX, dim, ME, ieps};
            const QrGiLayout Q(L.NX, L.NX);
            int itq = 0;
            status = qr_gi(pq, S + L.XV, S + L.SIZE, Q, L.NX, i, kp, lo_rep, hi_rep, 10 * (L.NX + ME) + 50, itq);
            iters += itq;
            wave_sync();
        }
    }
    if constexpr (!REPAIR) {
        // no step exists: the waist task is not attainable at b_w (the rows are boxes in
        // (tau_a, f), so nothing else can be infeasible) -- the repair kernel solves level 0 first.
        // A loop that ends at the step or rounds cap (1) or on a numerically dependent set (3) goes
        // there too: an unattainable waist target often shows as cycling among nearly dependent rows
        // rather than as a clean "no step", and the repair's pinned level 1 is the robust route
        if ((status == 2 || status == 1 || (status == 3 && !notspd)) && !a.limits_crossed && a.wl) {
            if (i == 0) {
                a.status[b] = -2;
                const int idx = atomicAdd(&a.work[a.epoch * 2 + 1], 1);
                a.wl[idx] = (int)b;
            }
            return;
        }
    }

    // ------------------------------------------------------------------ 7. outputs
    wave_sync();
    WBQ_STAMP(5);
    const bool ok = status == 0;
    if (a.ws_rows) { // the next solve's warm start: this solve's final active set (a repaired solve's
                     // pinned problem is not the next solve's: cold then)
        const int wrec = warm_record(S, GiVecs{L.VV, L.LV, L.RV, L.WV, L.AC, L.TT, L.TS}, i, gs);
        a.ws_rows[b * 64 + i] = (signed char)((ok && !REPAIR && kind == 2) ? wrec : 0);
    }
    double tau_i = h_i;
    if (ok && qrow) { // joint row i: M_i qdd - J_c,i^T f + h_i
        double t = h_i;
        // lane i's own M row and contact-Jacobian column, re-read (L2) rather than held
        const __amdgpu_buffer_rsrc_t Mrs = rsrc_at(a.M, b, B, (long)n * n);
        const int moff = (int)(8 * ic);
        double mr[NQ], jr[NFM]; // unconditional (clamped) loads: one round trip
#pragma unroll
        for (int j = 0; j < NQ; ++j) mr[j] = bload(Mrs, moff, 8 * (j < n ? j : n - 1) * n);
        const __amdgpu_buffer_rsrc_t Jrs = rsrc_at(a.Jc, b, B, (long)nc * 6 * n);
        const int joff = (int)(8 * ic);
#pragma unroll
        for (int f = 0; f < NFM; ++f)
            jr[f] = bload(Jrs, joff, 8 * (6 * (f < nf ? f / WD : 0) + f % WD) * n);
#pragma unroll
        for (int j = 0; j < NQ; ++j) t = fma(j < n ? mr[j] : 0.0, S[L.XV + (j < n ? j : 0)], t);
#pragma unroll
        for (int f = 0; f < NFM; ++f)
            t = fma((f < nf && ((cm >> (f / WD)) & 1)) ? -jr[f] : 0.0, S[L.XV + n + (f < nf ? f : 0)], t);
        tau_i = t;
    }
    const double tmax = imax<64>((qrow && !isfinite(tau_i)) ? 1.0 : 0.0);
    if (ok && tmax > 0.0) status = 3;
    if (status != 0) tau_i = h_i;
    if (qrow) a.tau[b * n + i] = tau_i;
    rollout_step(a, b, i, qrow, S[L.XV + i], status == 0); // qdd = x[0:n]
    if (i < L.NX) a.x[b * L.NX + i] = status == 0 ? S[L.XV + i] : 0.0;
    if (i == 0) {
        a.status[b] = status;
        a.iters[b] = iters;
    }
    WBQ_STAMP(6);
#ifdef WBQ_STAMPS
    if (i == 0 && a.stamps) a.stamps[b * kStamps + 7] = gs.rounds;
#endif
}

template <int NQ, bool TR, int KMR, int WD>
__global__ __launch_bounds__(64, (!TR && KMR > 0 && KMR <= 18) ? 2 : 1) void contact_kernel(const ContactArgs a)
{
    contact_solve<NQ, TR, KMR, WD, false>(a, (long)blockIdx.x);
}

// Level-0 repair: the instances contact_kernel listed (status -2), grid-stride; its own register
// budget (the BVLS of the level-0 step) leaves the main kernel's alone.
template <int NQ, bool TR, int KMR, int WD>
__global__ __launch_bounds__(64, 1) void contact_repair_kernel(const ContactArgs a)
{
    const int cnt = a.work[a.epoch * 2 + 1];
    if (blockIdx.x == 0 && threadIdx.x == 0) { // the next solve's counter (its parity was last used
        a.work[(a.epoch ^ 1) * 2] = 0;         // by the previous solve, which has completed)
        a.work[(a.epoch ^ 1) * 2 + 1] = 0;
    }
    follow_publish(a.fg, 0, cnt);
    for (long e = blockIdx.x; e < cnt; e += gridDim.x) {
        wave_sync(); // the previous instance's LDS is dead
        contact_solve<NQ, TR, KMR, WD, true>(a, uniform_long(a.wl[e]));
    }
}

template <int NQ, bool TR, int KMR, int WD>
hipError_t launch_t(const ContactArgs &a, hipStream_t stream, hipEvent_t mid)
{
    constexpr int NRC = TR ? 40 : 16;
    const ContactLayout L(a.n, a.nc, TR, NQ, NRC, WD, a.nfr, a.mu, TR ? 0 : KMR);
    if (L.NR > NRC * ((NQ == 64 && TR) ? 2 : 1) || L.ME > 64 || L.NX > 64) return hipErrorInvalidValue;
    // the register slot vectors hold every active row
    if (!TR && KMR > 0 && (L.ME > KMR || a.nc * WD > KMR - 12)) return hipErrorInvalidValue;
    const size_t lds = sizeof(double) * L.SIZE;
    // the repair kernel's LDS also holds the QR-form fallback's basis when it fits the device's LDS per
    // workgroup (160 KB on gfx950; queried, so a build for another target keeps the shapes that fit there)
    const size_t lds_qr = lds + sizeof(double) * QrGiLayout(L.NX, L.NX).SIZE;
    const bool qr = lds_qr <= max_workgroup_lds();
    const size_t lds2 = qr ? lds_qr : lds;
    if (a.prepare) {
        const hipError_t e = ensure_dynamic_lds((const void *)contact_kernel<NQ, TR, KMR, WD>, lds);
        return e != hipSuccess ? e : ensure_dynamic_lds((const void *)contact_repair_kernel<NQ, TR, KMR, WD>, lds2);
    }
    hipLaunchKernelGGL((contact_kernel<NQ, TR, KMR, WD>), dim3((unsigned)a.B), dim3(64), lds, stream, a);
    hipError_t e2 = hipGetLastError();
    if (e2 != hipSuccess || !a.wl) return e2;
    if (mid) {
        e2 = hipEventRecord(mid, stream);
        if (e2 != hipSuccess) return e2;
    }
    const unsigned grid = follow_blocks(a.fg.est[1], 1, kContactRepairGrid, a.B);
    ContactArgs a2 = a;
    a2.qr_fallback = qr ? 1 : 0;
    hipLaunchKernelGGL((contact_repair_kernel<NQ, TR, KMR, WD>), dim3(grid), dim3(64), lds2, stream, a2);
    return hipGetLastError();
}

// Variant by problem shape: torque rows -> LDS slot vectors (k up to n + WD nc); otherwise the
// active rows fit register slot vectors of 12 + WD nc (18 for the reference's double support,
// 24 for four contacts or two full wrenches); friction rows (ME > 12 + WD nc) or four full
// wrenches (36 slots) -> LDS slot vectors.
template <int NQ, int WD>
hipError_t launch_wd(const ContactArgs &a, hipStream_t stream, hipEvent_t mid)
{
    if (a.torque_rows) return launch_t<NQ, true, 64, WD>(a, stream, mid);
    if (a.nfr > 0) return launch_t<NQ, false, 0, WD>(a, stream, mid);
    if constexpr (WD == 3)
        return a.nc <= 2 ? launch_t<NQ, false, 18, 3>(a, stream, mid) : launch_t<NQ, false, 24, 3>(a, stream, mid);
    else
        return a.nc <= 2 ? launch_t<NQ, false, 24, 6>(a, stream, mid) : launch_t<NQ, false, 0, 6>(a, stream, mid);
}

template <int NQ>
hipError_t launch_nq(const ContactArgs &a, hipStream_t stream, hipEvent_t mid)
{
    return a.wd == 6 ? launch_wd<NQ, 6>(a, stream, mid) : launch_wd<NQ, 3>(a, stream, mid);
}

}  // namespace

hipError_t launch_contact(const ContactArgs &a, hipStream_t stream, hipEvent_t mid)
{
    if (a.B <= 0) return hipSuccess;
    return a.n <= 32 ? launch_nq<32>(a, stream, mid) : launch_nq<64>(a, stream, mid);
}

}  // namespace wbq
