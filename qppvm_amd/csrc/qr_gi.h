// qr_gi.h -- Goldfarb-Idnani dual active set in QR form: the robust fallback of the contact form's
// level 1 (contact_kernel.hip, repair kernel), one instance per wave64, gfx950, fp64.
//
// The constraint-space loop (dual_gi.h) decides a row's dependency from its Schur complement in
// Gamma = A H^-1 A^T, formed by cancellation against the diagonal: with the contact form's 1 / eps_f
// force scale a dependent row's complement is ~1e-7 against Gamma_pp ~1e8, so near a
// degenerate vertex (the friction pyramid's faces, pinned box sides and torque rows all active) the
// loop can add a row that is dependent to roundoff, or reject one that is not, and end with status 1
// or 2 where the problem is solvable. This loop keeps an explicit basis of the active normals instead:
// covectors v_q, orthonormal in the H^-1 metric, each carried with z_q = H^-1 v_q (x-space vectors),
// and R with a_act(q) = sum_j R[j][q] v_j. A row's residual w = a_p - sum_q u_q v_q (u_q = z_q . a_p,
// two Gram-Schmidt passes) and H^-1 w = H^-1 a_p - sum_q u_q z_q give its complement zz = w . H^-1 w
// to roundoff of |a_p|, not of Gamma_pp; the primal direction is H^-1 w, the dual one r = R^-1 u.
// A drop deletes a column of R and restores the triangle by Givens rotations on R's rows and the
// basis pairs. Activities are recomputed from x at every outer step, and x is refined on the active
// rows there and at the end (A_A H^-1 A_A^T = R^T R, so dx = sum_q (R^-T r_A)_q z_q).
// Row selection, the dependency scale |a_p|^2 and the skip of a dependent row violated only to the
// roundoff of the rows it depends on follow the oracle's dense dual method
// (oracle/wbq_oracle_contact.c:wbq_ref_dual_qp); numpy statement: scripts/qr_gi.py solve_metric.
//
// Lane roles: lane j <-> coordinate j of x-space vectors (j < nx), lane ci <-> constraint row ci
// (activities, selection, its normal's owner), lane q <-> active slot q (u, r, lambda, R's row q).
// The problem P supplies (every lane calls each, wave-uniformly):
//   P.nx, P.dim (rank cap), P.m (rows)
//   double P.own_activity() const      -- lane ci: a_ci . x at x = S[XV]
//   double P.own_norm2() const         -- lane ci: |a_ci|^2
//   void P.normal(int p, double sg, double *ap, double *hp) const
//                                      -- writes sg a_p and sg H^-1 a_p into LDS vectors (all lanes)
#pragma once
#include "wbq_device.h"
#include "dual_gi.h" // bcast

namespace wbq {

// LDS of the fallback (doubles): basis covectors V, their H^-1 images Z (rows of stride VS), R (rows
// of stride RS), and per-lane vectors. kq = the most active rows, nx = the x-space dimension.
struct QrGiLayout {
    int VS, RS, V, Z, R, AP, HP, W, HW, U, U2, RR, LAM, ACT, SG, SV, Y, SIZE;
    __host__ __device__ QrGiLayout(int kq, int nx)
    {
        VS = nx | 1;
        RS = kq | 1;
        int o = 0;
        V = o; o += kq * VS;
        Z = o; o += kq * VS;
        R = o; o += kq * RS;
        AP = o; o += 64;
        HP = o; o += 64;
        W = o; o += 64;
        HW = o; o += 64;
        U = o; o += 64;
        U2 = o; o += 64;
        RR = o; o += 64;
        LAM = o; o += 64;
        ACT = o; o += 64;
        SG = o; o += 64;
        SV = o; o += 64;
        Y = o; o += 64;
        SIZE = (o + 1) & ~1;
    }
};

// Returns the status (0 solved, 1 step cap, 2 infeasible); x in X[0, nx) (LDS), which starts at the
// unconstrained minimum x0. SQ: the fallback's LDS (QrGiLayout offsets). Lane i's row: kind (0 off,
// 1 equality, 2 inequality; lo == hi also an equality), lo, hi.
template <typename P>
__device__ int qr_gi(const P &pb, double *X, double *SQ, const QrGiLayout &Q, int kq, int i, int kind, double lo,
                     double hi, int maxit, int &iters)
{
    double *S = SQ;
    constexpr double kInfT = 1.0e300;
    const int nx = pb.nx, m = pb.m;
    const bool rowi = i < m && kind != 0;
    const bool eqrow = rowi && (kind == 1 || lo == hi);
    const double an2 = rowi ? pb.own_norm2() : 0.0;
    const double anrm = sqrt(fmax(an2, 1e-300));
    bool onact = false, skipped = false;
    int k = 0, it = 0;
    int status = -1; // running
    auto refine = [&]() {
        // x on the active rows: r_A = sg (b - a . x) per slot, y = R^-T r_A, x += sum_q y_q z_q
        for (int pass = 0; pass < 2 && k > 0; ++pass) {
            S[Q.SV + i] = rowi ? pb.own_activity() : 0.0;
            __syncthreads();
            const int c = i < k ? (int)S[Q.ACT + i] : 0;
            const double loc = __shfl(lo, c), hic = __shfl(hi, c); // (every lane active)
            double acc = 0.0;
            if (i < k) {
                const double sg = S[Q.SG + i];
                acc = sg * ((sg > 0.0 ? loc : hic) - S[Q.SV + c]);
            }
            double y = 0.0;
            for (int q = 0; q < k; ++q) { // forward substitution with R^T (lower), one slot per step
                const double yq = bcast(acc, q) / S[Q.R + q * Q.RS + q];
                if (i == q) y = yq;
                if (i > q && i < k) acc = fma(-S[Q.R + q * Q.RS + i], yq, acc);
            }
            S[Q.Y + i] = y;
            __syncthreads();
            if (i < nx) {
                double dx = 0.0;
                for (int q = 0; q < k; ++q) dx = fma(S[Q.Y + q], S[Q.Z + q * Q.VS + i], dx);
                X[i] += dx;
            }
            __syncthreads();
        }
    };
#pragma unroll 1
    for (;;) {
        refine();
        const double s = rowi ? pb.own_activity() : 0.0;
        // next row: the lowest equality not yet active, else the most violated inequality side
        const unsigned long long eqm = __ballot(eqrow && !onact && !skipped);
        int p = -1;
        double sg = 1.0;
        if (eqm) {
            p = __builtin_ctzll(eqm);
            sg = bcast((lo - s) >= 0.0 ? 1.0 : -1.0, p);
        } else {
            double v = 0.0, vs = 1.0;
            if (rowi && kind == 2 && !onact && !skipped) {
                const double tol = 1e-10 * fmax(1.0, fmax(fabs(s), fmax(fin_abs(lo), fin_abs(hi))));
                if (lo - s > tol) {
                    v = (lo - s) / anrm;
                    vs = 1.0;
                }
                if (s - hi > tol && (s - hi) / anrm > v) {
                    v = (s - hi) / anrm;
                    vs = -1.0;
                }
            }
            int idx = i;
            iargmax<64>(v, idx);
            if (v > 0.0) {
                p = idx;
                sg = bcast(vs, p);
            }
        }
        if (p < 0) {
            status = 0;
            break;
        }
        const double bnd = sg > 0.0 ? bcast(lo, p) : bcast(hi, p);
        const double an2p = bcast(an2, p);
        pb.normal(p, sg, S + Q.AP, S + Q.HP);
        __syncthreads();
        double lamp = 0.0;
        bool done = false;
#pragma unroll 1
        while (!done) {
            if (++it > maxit) {
                status = 1;
                break;
            }
            // u = Z a_p, w = a_p - u V, H^-1 w = H^-1 a_p - u Z, and a second pass
            double wj = i < nx ? S[Q.AP + i] : 0.0, hj = i < nx ? S[Q.HP + i] : 0.0;
#pragma unroll 1
            for (int pass = 0; pass < 2; ++pass) {
                if (i < k) {
                    double d = 0.0;
                    for (int j = 0; j < nx; ++j) d = fma(S[Q.Z + i * Q.VS + j], pass ? S[Q.W + j] : S[Q.AP + j], d);
                    S[(pass ? Q.U2 : Q.U) + i] = d;
                }
                __syncthreads();
                if (i < nx) {
                    for (int q = 0; q < k; ++q) {
                        const double uq = S[(pass ? Q.U2 : Q.U) + q];
                        wj = fma(-uq, S[Q.V + q * Q.VS + i], wj);
                        hj = fma(-uq, S[Q.Z + q * Q.VS + i], hj);
                    }
                }
                S[Q.W + i] = wj;
                __syncthreads();
            }
            if (i < k) S[Q.U + i] += S[Q.U2 + i];
            const double zz = isum<64>(i < nx ? wj * hj : 0.0);
            __syncthreads();
            // r = R^-1 u (back substitution, one slot per step)
            double acc = i < k ? S[Q.U + i] : 0.0, r = 0.0;
            for (int q = k - 1; q >= 0; --q) {
                const double rq = bcast(acc, q) / S[Q.R + q * Q.RS + q];
                if (i == q) r = rq;
                if (i < q) acc = fma(-S[Q.R + i * Q.RS + q], rq, acc);
            }
            // slack of p at the current x (lane p's own row)
            const double sp = bcast(rowi ? pb.own_activity() : 0.0, p);
            const double slack = sg * (bnd - sp);
            // ratio test over the active inequalities (equalities and pinned rows are never dropped)
            const double rmax = imax<64>(i < k ? fabs(r) : 0.0);
            double cand = kInfT;
            const int cs = i < k ? (int)S[Q.ACT + i] : 0;
            const bool ceq = __shfl(eqrow ? 1 : 0, cs) != 0; // (every lane active)
            if (i < k && !ceq && r > 1e-12 * fmax(rmax, 1e-300)) cand = S[Q.LAM + i] / r;
            int blk = i;
            iargmin<64>(cand, blk);
            const double t1 = cand;
            const bool indep = zz > 1e-14 * an2p && k < pb.dim && k < kq;
            const double t2 = indep ? slack / zz : kInfT;
            if (t1 >= kInfT && t2 >= kInfT) {
                // dependent, nothing to drop: skip a violation at the roundoff of the rows p depends on
                // (the oracle's rule), else infeasible
                const double ps = isum<64>(i < nx ? fabs(S[Q.AP + i] * X[i]) : 0.0);
                if (lamp == 0.0 && slack <= 1e-9 * (1.0 + fabs(bnd) + ps)) {
                    if (i == p) skipped = true;
                    break;
                }
                status = 2;
                done = true;
                break;
            }
            const double t = fmin(t1, t2);
            if (indep && i < nx) X[i] = fma(t, hj, X[i]);
            if (i < k) S[Q.LAM + i] -= t * r;
            lamp += t;
            __syncthreads();
            if (t2 <= t1) { // add p: v_k = w / |w|, z_k = H^-1 w / |w|, R column k = [u; |w|]
                const double nz = sqrt(zz), inz = 1.0 / nz;
                if (i < nx) {
                    S[Q.V + k * Q.VS + i] = wj * inz;
                    S[Q.Z + k * Q.VS + i] = hj * inz;
                }
                if (i < k) S[Q.R + i * Q.RS + k] = S[Q.U + i];
                if (i == k) {
                    S[Q.R + k * Q.RS + k] = nz;
                    S[Q.ACT + k] = (double)p;
                    S[Q.SG + k] = sg;
                    S[Q.LAM + k] = lamp;
                }
                if (i == p) onact = true;
                ++k;
                __syncthreads();
                break;
            }
            // drop slot blk (wave-uniform): its row leaves the active set, the slots after it move up
            const int cb = (int)S[Q.ACT + blk];
            if (i == cb) onact = false;
            double a0 = 0.0, a1 = 0.0, a2 = 0.0;
            if (i >= blk && i + 1 < k) {
                a0 = S[Q.ACT + i + 1];
                a1 = S[Q.SG + i + 1];
                a2 = S[Q.LAM + i + 1];
            }
            // R without column blk: lane q shifts its row
            if (i < k)
                for (int c = blk; c + 1 < k; ++c) S[Q.R + i * Q.RS + c] = S[Q.R + i * Q.RS + c + 1];
            __syncthreads();
            if (i >= blk && i + 1 < k) {
                S[Q.ACT + i] = a0;
                S[Q.SG + i] = a1;
                S[Q.LAM + i] = a2;
            }
            // Givens on rows q, q + 1 of R (columns q.. k-2) and on the basis pairs (v, z)
            for (int q = blk; q + 1 < k; ++q) {
                const double ra = S[Q.R + q * Q.RS + q], rb = S[Q.R + (q + 1) * Q.RS + q];
                const double h = sqrt(fma(ra, ra, rb * rb));
                const double c = h > 0.0 ? ra / h : 1.0, sn = h > 0.0 ? rb / h : 0.0;
                __syncthreads();
                if (i >= q && i + 1 < k) {
                    const double x0 = S[Q.R + q * Q.RS + i], x1 = S[Q.R + (q + 1) * Q.RS + i];
                    S[Q.R + q * Q.RS + i] = fma(c, x0, sn * x1);
                    S[Q.R + (q + 1) * Q.RS + i] = fma(-sn, x0, c * x1);
                }
                if (i < nx) {
                    const double v0 = S[Q.V + q * Q.VS + i], v1 = S[Q.V + (q + 1) * Q.VS + i];
                    S[Q.V + q * Q.VS + i] = fma(c, v0, sn * v1);
                    S[Q.V + (q + 1) * Q.VS + i] = fma(-sn, v0, c * v1);
                    const double z0 = S[Q.Z + q * Q.VS + i], z1 = S[Q.Z + (q + 1) * Q.VS + i];
                    S[Q.Z + q * Q.VS + i] = fma(c, z0, sn * z1);
                    S[Q.Z + (q + 1) * Q.VS + i] = fma(-sn, z0, c * z1);
                }
                __syncthreads();
            }
            --k;
            __syncthreads();
        }
        if (done || status >= 0) break;
    }
    if (status == 0) refine();
    iters = it;
    return status;
}

}  // namespace wbq
