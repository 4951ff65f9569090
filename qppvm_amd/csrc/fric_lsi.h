// fric_lsi.h -- level 0 of the contact form over the box AND the linearised friction pyramid
// (SURVEY.md 8f-2), the least-squares problem with inequalities (LSI)
//   min 0.5 ||A z - b||^2   s.t.  lo <= z <= hi,   s f_x - mu f_z <= 0,  s f_y - mu f_z <= 0
// for every active contact's force (f_x, f_y, f_z) (z = (tau_a, w), contact_kernel.hip:
// contact_level0). The oracle solves the same level 0 as a ridge QP in x-space
// (oracle/wbq_oracle_contact.c:wbq_ref_contact_one, friction rows in Z.C); this is a primal active set
// in the pattern of BVLS (qppvm_repair.h:bvls, Stark-Parker), generalised to the pyramid faces:
// * a lane owns one variable (its A column). A variable outside a friction group has BVLS's box
//   state; the three force components of an active contact form a group whose active constraints
//   (box sides of its components, pyramid faces) span N_c, with Q_c R_c = N_c (Gram-Schmidt, <= 3
//   normals) and the projector P_c = I - Q_c Q_c^T onto the group's free directions;
// * inner loop: minimum-norm least-squares step dz = P A^T w, (A P A^T) w = b - A z (6 x 6, pivoted
//   Cholesky as BVLS), interpolated back at the first blocking box side or face (it joins the set);
// * outer loop: multipliers -- a single variable's is BVLS's w_j = a_j^T (b - A z); a group's solve
//   N_c lambda = w_c (R_c lambda = Q_c^T w_c) -- and the most violated constraint leaves the set
//   (Stark-Parker's exclusion when it re-enters at once);
// * at the optimum the constraints with positive multipliers are the pins level 1 holds.
// tests/fric_lsi_ref.py is the numpy statement of the same steps (checked against the
// oracle on the level-0-infeasible sweep with mu 0.3 / 0.5: y0* to 1e-7 relative).
#pragma once
#include "qppvm_repair.h"

namespace wbq {

// Orthonormal basis of a friction group's active normals: box side of component k (st3[k] = +-1,
// normal +-e_k), then faces 0..3 (fm bits; face f = s f_{f>>1} - mu f_z, s = (f & 1) ? -1 : 1).
// Normals are taken in that order, at most three; one numerically dependent on the earlier ones is
// skipped (the ratio test never adds a dependent one, so this is roundoff insurance).
struct FricBasis {
    double q[3][3]; // rows q_s (s < d)
    double r[3][3]; // R (upper): n_s = sum_{t <= s} r[t][s] q_t
    double nn[3];   // |n_s|
    int code[3];    // 0..2 box side of component code, 3..6 face code - 3
    int d;
};

__device__ __forceinline__ void fric_normal(int code, int sgn, double mu, double (&v)[3])
{
    v[0] = v[1] = v[2] = 0.0;
    if (code < 3) {
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k] = k == code ? (double)sgn : 0.0;
    } else {
        const int f = code - 3;
        v[0] = (f >> 1) == 0 ? ((f & 1) ? -1.0 : 1.0) : 0.0;
        v[1] = (f >> 1) == 1 ? ((f & 1) ? -1.0 : 1.0) : 0.0;
        v[2] = -mu;
    }
}

__device__ __forceinline__ void fric_basis(const int (&st3)[3], int fm, double mu, FricBasis &B)
{
    B.d = 0;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        B.nn[s] = 0.0;
        B.code[s] = -1;
#pragma unroll
        for (int k = 0; k < 3; ++k) B.q[s][k] = B.r[s][k] = 0.0;
    }
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        const bool on = c < 3 ? (st3[c] == 1 || st3[c] == -1) : ((fm >> (c - 3)) & 1);
        if (!on || B.d >= 3) continue;
        double v[3];
        fric_normal(c, c < 3 ? st3[c] : 1, mu, v);
        const double n0 = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        double rc[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int pass = 0; pass < 2; ++pass)
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                if (s >= B.d) continue;
                const double t = B.q[s][0] * v[0] + B.q[s][1] * v[1] + B.q[s][2] * v[2];
                rc[s] += t;
#pragma unroll
                for (int k = 0; k < 3; ++k) v[k] = fma(-t, B.q[s][k], v[k]);
            }
        const double nv = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        if (!(nv > 1e-12 * n0)) continue;
        const double iv = 1.0 / nv;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            if (s != B.d) continue;
#pragma unroll
            for (int k = 0; k < 3; ++k) B.q[s][k] = v[k] * iv;
#pragma unroll
            for (int t = 0; t < 3; ++t) B.r[t][s] = t < s ? rc[t] : (t == s ? nv : 0.0);
            B.nn[s] = n0;
            B.code[s] = c;
        }
        ++B.d;
    }
}

// row k of the projector onto the free directions, P = I - sum_s q_s q_s^T
__device__ __forceinline__ void fric_prow(const FricBasis &B, int k, double (&p)[3])
{
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double v = j == k ? 1.0 : 0.0;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            double qk = 0.0;
#pragma unroll
            for (int kk = 0; kk < 3; ++kk) qk = kk == k ? B.q[s][kk] : qk;
            v = fma(-qk, B.q[s][j], v);
        }
        p[j] = v;
    }
}

// multipliers of the active normals: N lambda = w (w = -gradient of the group), R lambda = Q^T w
__device__ __forceinline__ void fric_lambda(const FricBasis &B, const double (&w)[3], double (&lam)[3])
{
    double y[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) y[s] = B.q[s][0] * w[0] + B.q[s][1] * w[1] + B.q[s][2] * w[2];
#pragma unroll
    for (int s = 2; s >= 0; --s) {
        double v = y[s];
#pragma unroll
        for (int t = s + 1; t < 3; ++t) v = fma(-B.r[s][t], lam[t], v);
        lam[s] = s < B.d ? v / B.r[s][s] : 0.0;
    }
}

struct LsiOut {
    double xv;      // z_i
    int it;         // iterations (inner steps)
    bool capped;    // the iteration cap ended it
    int pin;        // this lane's box side held by a positive multiplier (+1 hi, -1 lo, 0 none)
    int pfm;        // group lanes: pyramid faces held by a positive multiplier (bit f)
    double mcol[6]; // this lane's part of the columns level 1 can still move along (P' A^T, P' from
                    // the held constraints; a single variable: a_i unless held or fixed)
};

// Lane i: variable lane (row) with column acol, box [lo, hi]; gb >= 0: the lane is component
// k = i - gb (< 3) of the friction group starting at lane gb (every lane of the wave agrees on the
// groups). M0 = 6 rows, b every lane alike.
template <int NP, int M0>
__device__ __forceinline__ LsiOut fric_lsi(const double (&acol)[M0], const double (&b0v)[M0], int m0, double lo,
                                           double hi, bool row, int gb, double mu, int maxit)
{
    constexpr int NT = M0 * (M0 + 1) / 2;
    const int i = threadIdx.x & (NP - 1);
    const bool grp = gb >= 0;
    const int k = grp ? i - gb : 0;
    const int src0 = grp ? gb : i, src1 = grp ? gb + 1 : i, src2 = grp ? gb + 2 : i;
    LsiOut out;
    out.it = 0;
    out.capped = false;
    out.pin = 0;
    out.pfm = 0;
    // the group's three columns, once
    double gcol[3][M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) {
        gcol[0][c] = __shfl(acol[c], src0);
        gcol[1][c] = __shfl(acol[c], src1);
        gcol[2][c] = __shfl(acol[c], src2);
    }
    double xv = row ? fmin(fmax(0.0, lo), hi) : 0.0;
    int st = row ? 0 : 2; // 0 free, -1 at lo, +1 at hi, 2 padding lane
    if (row && lo == hi) st = -1;
    int fm = 0;     // active faces of the group (all lanes of a group alike)
    int ex = -1;    // excluded own constraint (code 0 box, 1 / 2 face 2k / 2k + 1), until progress
    int freed = -1; // constraint id (lane * 4 + code) released by the last KKT pick
    double abm = 0.0;
#pragma unroll
    for (int c = 0; c < M0; ++c) abm = fma(acol[c], b0v[c], abm);
    const double wtb = fabs(abm);
    abm = fmax(1.0, imax<NP>(wtb));
    int it = 0;
    auto group_state = [&](FricBasis &B) {
        int st3[3];
        st3[0] = __shfl(st, src0);
        st3[1] = __shfl(st, src1);
        st3[2] = __shfl(st, src2);
        fric_basis(st3, fm, mu, B);
    };
    bool outer = true;
    while (outer) {
        for (;;) {
            ++it;
            FricBasis B;
            group_state(B);
            double prow[3];
            fric_prow(B, k, prow);
            const bool fr1 = !grp && st == 0; // a free single variable
            double pcol[M0];
#pragma unroll
            for (int c = 0; c < M0; ++c)
                pcol[c] = grp ? fma(prow[0], gcol[0][c], fma(prow[1], gcol[1][c], prow[2] * gcol[2][c]))
                              : (fr1 ? acol[c] : 0.0);
            double rv[M0], gp[NT];
#pragma unroll
            for (int c = 0; c < M0; ++c) rv[c] = row ? acol[c] * xv : 0.0;
#pragma unroll
            for (int p = 0; p < M0; ++p)
#pragma unroll
                for (int c = 0; c <= p; ++c) gp[tri(p, c)] = acol[p] * pcol[c];
            isum_vec<NP, M0>(rv);
            isum_vec<NP, NT>(gp);
            const double kfree = isum<NP>(grp ? (k == 0 ? prow[0] : (k == 1 ? prow[1] : prow[2])) : (fr1 ? 1.0 : 0.0));
            if (!(kfree > 0.5)) break; // nothing can move
#pragma unroll
            for (int c = 0; c < M0; ++c) rv[c] = b0v[c] - rv[c];
            double wv[M0];
            if (!chol_solve_full<M0>(gp, m0, rv, wv, kCholFastTol<M0>)) {
                PivChol<M0> pc;
                pc.factor(gp, m0, 1e-12);
                pc.solve(rv, m0, wv);
            }
            double aw = 0.0;
#pragma unroll
            for (int c = 0; c < M0; ++c) aw = fma(acol[c], wv[c], aw);
            const double aw0 = __shfl(aw, src0), aw1 = __shfl(aw, src1), aw2 = __shfl(aw, src2);
            const double dz = grp ? fma(prow[0], aw0, fma(prow[1], aw1, prow[2] * aw2)) : (fr1 ? aw : 0.0);
            // ratio test: own box side (a component not at a bound), then the lane's two faces
            const double fz = __shfl(xv, src2), dfz = __shfl(dz, src2);
            double al = kInf;
            int code = 0, side = 0;
            if (row && st == 0 && lo != hi) {
                const double zn = xv + dz;
                if (dz < 0.0 && zn < lo) {
                    al = fmax(0.0, (lo - xv) / dz);
                    side = -1;
                } else if (dz > 0.0 && zn > hi) {
                    al = fmax(0.0, (hi - xv) / dz);
                    side = 1;
                }
                if (!(al < 1.0)) al = kInf;
            }
            if (grp && k < 2) {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int f = 2 * k + s;
                    if ((fm >> f) & 1) continue;
                    const double sg = s ? -1.0 : 1.0;
                    const double ph = fma(sg, xv, -mu * fz), dph = fma(sg, dz, -mu * dfz);
                    // (a roundoff-level approach is no block: the face would be dependent)
                    if (dph > 1e-13 * (fabs(dz) + mu * fabs(dfz)) && ph + dph > 0.0) {
                        const double af = fmax(0.0, -ph) / dph;
                        if (af < 1.0 && af < al) {
                            al = af;
                            code = 1 + s;
                        }
                    }
                }
            }
            int jb = i;
            double alm = al;
            iargmin<NP>(alm, jb);
            if (alm >= kInf) { // the step stays feasible: take it
                xv += dz;
                freed = -1;
                ex = -1;
                break;
            }
            const int cb = __shfl(code, jb), gbb = __shfl(gb, jb), kb = __shfl(k, jb);
            const double alpha = fmax(alm, 0.0);
            if (jb * 4 + cb == freed && alpha == 0.0) {
                // the constraint just released wants back through: re-add it, exclude it
                if (cb == 0 && i == jb) {
                    st = side;
                    xv = st < 0 ? lo : hi;
                }
                if (cb > 0 && grp && gb == gbb) fm |= 1 << (2 * kb + cb - 1);
                if (i == jb) ex = cb;
                freed = -1;
                break;
            }
            ex = -1; // progress: exclusions expire
            const double zt = xv + dz; // the full step's target
            xv = fma(alpha, dz, xv);
            if (!grp && fr1 && i != jb) { // BVLS: single variables that land on a bound stop there
                const double tl = 1e-14 * fmax(1.0, fabs(lo)), tu = 1e-14 * fmax(1.0, fabs(hi));
                if (xv <= lo + tl && zt < lo) st = -1;
                else if (xv >= hi - tu && zt > hi) st = 1;
            }
            if (cb == 0 && i == jb) st = side;
            if (st == -1) xv = lo;
            if (st == 1) xv = hi;
            if (cb > 0 && grp && gb == gbb) fm |= 1 << (2 * kb + cb - 1);
            freed = -1;
            if (it >= maxit) break;
        }
        // KKT: w = A^T (b - A z); single variables as BVLS, groups through their multipliers
        double rf[M0];
#pragma unroll
        for (int c = 0; c < M0; ++c) rf[c] = row ? acol[c] * xv : 0.0;
        isum_vec<NP, M0>(rf);
        double w = 0.0, wx = 0.0;
#pragma unroll
        for (int c = 0; c < M0; ++c) {
            w = fma(acol[c], b0v[c] - rf[c], w);
            wx = fma(acol[c], rf[c], wx);
        }
        const double wtol = 1e-11 * fmax(abm, imax<NP>(fmax(wtb, fabs(wx))));
        FricBasis B;
        group_state(B);
        double lam[3];
        {
            const double wg[3] = {__shfl(w, src0), __shfl(w, src1), __shfl(w, src2)};
            fric_lambda(B, wg, lam);
        }
        double v = -kInf;
        int vcode = 0;
        if (!grp) {
            if ((st == -1 || st == 1) && ex != 0 && lo != hi) v = st < 0 ? w : -w;
        } else {
            // the lane's own constraints: its box side (code 0) and faces 2k, 2k + 1 (codes 1, 2)
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                if (s >= B.d) continue;
                const int c = B.code[s];
                int own = -1;
                if (c < 3 && c == k && lo != hi) own = 0;
                if (c >= 3 && ((c - 3) >> 1) == k) own = 1 + ((c - 3) & 1);
                if (own < 0 || own == ex) continue;
                const double vv = -lam[s] * B.nn[s];
                if (vv > v) {
                    v = vv;
                    vcode = own;
                }
            }
        }
        int best = i;
        double vb = v;
        iargmax<NP>(vb, best);
        if (!(vb > wtol)) {
            outer = false;
        } else if (it >= maxit) {
            out.capped = true;
            outer = false;
        } else {
            const int cb = __shfl(vcode, best), gbb = __shfl(gb, best), kb = __shfl(k, best);
            if (cb == 0 && i == best) st = 0; // exclusions persist until the inner loop makes progress
            if (cb > 0 && grp && gb == gbb) fm &= ~(1 << (2 * kb + cb - 1));
            freed = best * 4 + cb;
        }
    }
    // pins: the constraints held by a positive multiplier at the optimum, and the directions the
    // remaining ones leave (level 1's waist rows keep only a basis of what these columns span)
    double rf[M0];
#pragma unroll
    for (int c = 0; c < M0; ++c) rf[c] = row ? acol[c] * xv : 0.0;
    isum_vec<NP, M0>(rf);
    double w = 0.0;
#pragma unroll
    for (int c = 0; c < M0; ++c) w = fma(acol[c], b0v[c] - rf[c], w);
    const double pintol = 1e-9 * abm;
    if (!grp) {
        if (row && lo != hi) out.pin = w > pintol ? 1 : (w < -pintol ? -1 : 0);
        if (row && lo == hi) out.pin = -1;
        const bool mov = row && out.pin == 0;
#pragma unroll
        for (int c = 0; c < M0; ++c) out.mcol[c] = mov ? acol[c] : 0.0;
    } else {
        FricBasis B;
        group_state(B);
        double lam[3];
        const double wg[3] = {__shfl(w, src0), __shfl(w, src1), __shfl(w, src2)};
        fric_lambda(B, wg, lam);
        int st3h[3] = {0, 0, 0}, fmh = 0;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            if (s >= B.d) continue;
            const int c = B.code[s];
            const bool held = lam[s] * B.nn[s] > pintol;
            if (c < 3) {
                int sd = __shfl(st, c == 0 ? src0 : (c == 1 ? src1 : src2));
                const double l0 = __shfl(lo, c == 0 ? src0 : (c == 1 ? src1 : src2));
                const double h0 = __shfl(hi, c == 0 ? src0 : (c == 1 ? src1 : src2));
                if (held || l0 == h0) {
#pragma unroll
                    for (int kk = 0; kk < 3; ++kk) st3h[kk] = kk == c ? sd : st3h[kk];
                    if (c == k) out.pin = sd;
                }
            } else if (held) {
                fmh |= 1 << (c - 3);
            }
        }
        out.pfm = fmh;
        FricBasis Bh;
        fric_basis(st3h, fmh, mu, Bh);
        double prow[3];
        fric_prow(Bh, k, prow);
#pragma unroll
        for (int c = 0; c < M0; ++c) out.mcol[c] = fma(prow[0], gcol[0][c], fma(prow[1], gcol[1][c], prow[2] * gcol[2][c]));
    }
    out.xv = xv;
    out.it = it;
    return out;
}

}  // namespace wbq
