/*
 * wbq_oracle_contact.c -- CPU restatement (TEST INFRASTRUCTURE ONLY) of the contact-form
 * whole-body QP of the reference's ForceAcc plugin.
 *
 * Parity status: unpinned against the reference binaries (OpenSoT/qpOASES absent, SURVEY
 * 8c). Pinned instead to tests/golden/make_golden_contact.py (an independent numpy
 * restatement whose answers carry a KKT certificate).
 *
 * Reference anchors (files under /root/reference):
 *   src/ForceAcc.cpp:58-72    decision vector x = [qddot (n); f_c (3) per contact] (:67 "put 6 for
 *                             full wrench": wrench_dim = 6, x = [qddot; w_c (6) per contact])
 *   src/ForceAcc.cpp:74-95    wrench w_c = [f_c; 0_3], box lb=(-1000,-1000,10,-1,-1,-1) ub=(1000,..,1)
 *   src/ForceAcc.cpp:83-89    feet acceleration Cartesian tasks (world frame)
 *   src/ForceAcc.cpp:105-107  postural acceleration task
 *   src/ForceAcc.cpp:109-114  DynamicFeasibility: floating-base rows of M qdd + h = sum J_c^T w_c
 *   src/ForceAcc.cpp:118-122  waist (pelvis) acceleration Cartesian task, ref p_init - 0.1 z
 *   src/ForceAcc.cpp:131-133  stack waist / (postural + feet) << dyn_feas << wrench bounds
 *   src/ForceAcc.cpp:135-137  QPOases_sot(.., eps_regularisation = 1e4)
 *   src/ForceAcc.cpp:196-219  tau = ID(q, qd, qdd) - sum J_c^T w_c = M qdd + h - sum J_c^T w_c
 *
 * The build's written spec (each [upstream] choice a named option):
 *   Cartesian acceleration task  J qdd = Kp e - Kd J qd - Jdot qd   (xdd_ref = 0, xd_ref = 0)
 *   postural task                qdd  = Kp (q_ref - q) - Kd qd
 *   level 0   min ||J_w qdd - b_w||^2
 *   level 1   min ||qdd - b_p||^2 + sum_c ||J_c qdd - b_c||^2 + eps_f ||f||^2
 *             s.t. J_w qdd = y0* (level-0 optimality)
 *   both      dynamic feasibility (6 equality rows), force box (inactive contacts: f = 0),
 *             optional actuated torque rows tau_min <= M_a qdd + h_a - J_{c,a}^T f <= tau_max
 *             (row a12, an extension: the reference ForceAcc has none), optional linearised
 *             friction pyramid |f_x| <= mu f_z, |f_y| <= mu f_z per active contact (SURVEY 8f-2;
 *             the reference has no cone, ForceAcc.cpp:74-76)
 * With wrench_dim = 6 every "f" above is the 6-D wrench w_c and J_c^T w_c uses all six Jacobian rows.
 * eps_f is the minimum-norm tie-break on the contact forces: with 3+ contacts the forces
 * have an internal null space no task sees; the reference leaves it to qpOASES' Hessian
 * regularisation, which this makes explicit.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "wbq_oracle.h"

static double cmaxd(double a, double b) { return a > b ? a : b; }

/* |bound|, 0 for an unbounded side (+-1e300): tolerances scale with finite bounds only */
static double fin(double v) { return fabs(v) < 1e299 ? fabs(v) : 0.0; }

int wbq_ref_contact_wd(const wbq_ref_contact_desc *d) { return d->wrench_dim == 6 ? 6 : 3; }

/* Solve A x = b (A N x N destroyed, b overwritten), LU with partial pivoting. */
static int lu(int N, double *A, double *b)
{
    double amax = 0.0;
    for (int i = 0; i < N * N; ++i) amax = cmaxd(amax, fabs(A[i]));
    const double tiny = 1e-14 * cmaxd(amax, 1e-300);
    for (int k = 0; k < N; ++k) {
        int p = k;
        for (int i = k + 1; i < N; ++i)
            if (fabs(A[i * N + k]) > fabs(A[p * N + k])) p = i;
        if (fabs(A[p * N + k]) <= tiny) return -1;
        if (p != k) {
            for (int j = 0; j < N; ++j) {
                const double t = A[k * N + j];
                A[k * N + j] = A[p * N + j];
                A[p * N + j] = t;
            }
            const double t = b[k];
            b[k] = b[p];
            b[p] = t;
        }
        for (int i = k + 1; i < N; ++i) {
            const double f = A[i * N + k] / A[k * N + k];
            if (f == 0.0) continue;
            for (int j = k + 1; j < N; ++j) A[i * N + j] -= f * A[k * N + j];
            b[i] -= f * b[k];
        }
    }
    for (int i = N - 1; i >= 0; --i) {
        double t = b[i];
        for (int j = i + 1; j < N; ++j) t -= A[i * N + j] * b[j];
        b[i] = t / A[i * N + i];
    }
    return 0;
}

/* Step of the dual method for the active normals A (k x n, row-major): solves
 *   [H A^T; A 0] [z; r] = [np; 0]
 * so that z = primal direction (H-orthogonal to the active normals), r = dual direction. */
static int gi_direction(int n, const double *H, int k, const double *A, const double *np, double *z, double *r)
{
    const int N = n + k;
    double *K = (double *)calloc((size_t)N * N, sizeof(double));
    double *rhs = (double *)calloc((size_t)N, sizeof(double));
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) K[i * N + j] = H[i * n + j];
        rhs[i] = np[i];
    }
    for (int a = 0; a < k; ++a)
        for (int j = 0; j < n; ++j) {
            K[(n + a) * N + j] = A[a * n + j];
            K[j * N + n + a] = A[a * n + j];
        }
    const int rc = lu(N, K, rhs);
    if (rc == 0) {
        memcpy(z, rhs, sizeof(double) * n);
        memcpy(r, rhs + n, sizeof(double) * k);
    }
    free(K);
    free(rhs);
    return rc;
}

int wbq_ref_dual_qp(int n, const double *H, const double *g, int me, const double *E, const double *e, int mi,
                    const double *C, const double *clo, const double *chi, double *x, int *iters)
{
    const int kmax = me + mi;
    double *A = (double *)malloc(sizeof(double) * (size_t)(kmax + 1) * n); /* active normals */
    double *ab = (double *)malloc(sizeof(double) * (kmax + 1));            /* their rhs */
    double *lam = (double *)malloc(sizeof(double) * (kmax + 1));
    int *kind = (int *)malloc(sizeof(int) * (kmax + 1)); /* -1 equality, else inequality row */
    double *z = (double *)malloc(sizeof(double) * n);
    double *r = (double *)malloc(sizeof(double) * (kmax + 1));
    double *np = (double *)malloc(sizeof(double) * n);
    double *Hc = (double *)malloc(sizeof(double) * n * n);
    int k = 0, it = 0, status = WBQ_REF_MAXITER;
    const int maxit = 10 * (n + kmax) + 50;
    int *onrow = (int *)calloc((size_t)(mi > 0 ? mi : 1), sizeof(int)); /* row active (either side) */

    /* unconstrained minimum x = -H^-1 g */
    memcpy(Hc, H, sizeof(double) * n * n);
    for (int i = 0; i < n; ++i) x[i] = -g[i];
    if (lu(n, Hc, x) != 0) {
        status = WBQ_REF_NUMERICAL;
        goto out;
    }
    int eq_next = 0;
    for (;;) {
        /* pick the constraint to add: equalities first (in order), then the most violated
         * inequality side (violation scaled by the row norm) */
        double bp = 0.0;
        int pk = -2; /* -1 equality, >= 0 inequality row */
        if (eq_next < me) {
            const double *er = E + (size_t)eq_next * n;
            double s = -e[eq_next];
            for (int j = 0; j < n; ++j) s += er[j] * x[j];
            const double sg = s > 0.0 ? -1.0 : 1.0; /* orient so that s_p <= 0 */
            for (int j = 0; j < n; ++j) np[j] = sg * er[j];
            bp = sg * e[eq_next];
            pk = -1;
            ++eq_next;
        } else {
            double best = 0.0;
            int bj = -1, bside = 0;
            for (int j = 0; j < mi; ++j) {
                if (onrow[j]) continue;
                const double *cr = C + (size_t)j * n;
                double s = 0.0, nn = 0.0;
                for (int i = 0; i < n; ++i) {
                    s += cr[i] * x[i];
                    nn += cr[i] * cr[i];
                }
                nn = sqrt(cmaxd(nn, 1e-300));
                const double vlo = clo[j] - s, vhi = s - chi[j];
                const double tl = 1e-10 * cmaxd(1.0, cmaxd(fabs(s), fin(clo[j])));
                const double th = 1e-10 * cmaxd(1.0, cmaxd(fabs(s), fin(chi[j])));
                if (vlo > tl && vlo / nn > best) best = vlo / nn, bj = j, bside = 1;
                if (vhi > th && vhi / nn > best) best = vhi / nn, bj = j, bside = -1;
            }
            if (bj < 0) {
                status = WBQ_REF_OK;
                break;
            }
            const double *cr = C + (size_t)bj * n;
            for (int i = 0; i < n; ++i) np[i] = bside * cr[i];
            bp = bside > 0 ? clo[bj] : -chi[bj];
            pk = bj;
        }
        double lamp = 0.0;
        for (;;) { /* steps for this constraint until it is added */
            if (++it > maxit) goto out;
            if (gi_direction(n, H, k, A, np, z, r) != 0) {
                status = WBQ_REF_NUMERICAL;
                goto out;
            }
            double zz = 0.0, sp = -bp, nn = 0.0;
            for (int i = 0; i < n; ++i) {
                zz += z[i] * np[i];
                sp += np[i] * x[i];
                nn += np[i] * np[i];
            }
            double rmax = 0.0;
            for (int a = 0; a < k; ++a) rmax = cmaxd(rmax, fabs(r[a]));
            double t1 = INFINITY;
            int blk = -1;
            for (int a = 0; a < k; ++a)
                if (kind[a] >= 0 && r[a] > 1e-12 * cmaxd(rmax, 1e-300) && lam[a] / r[a] < t1) t1 = lam[a] / r[a], blk = a;
            const double t2 = (zz > 1e-14 * nn) ? -sp / zz : INFINITY;
            if (!isfinite(t1) && !isfinite(t2)) {
                /* p depends on the active normals and nothing can be dropped. A violation at the
                 * roundoff of the rows it depends on (a degenerate face: the level-1 problem after a
                 * level-0 repair holds the waist rows at y0*, which the active bounds already imply)
                 * is not an inconsistency: p is met as far as the data determine it, so it is
                 * skipped for this pass. A first step only: once partial steps moved x for p its
                 * multiplier is in play and the rows are genuinely inconsistent. */
                double ps = 0.0;
                for (int i = 0; i < n; ++i) ps += fabs(np[i] * x[i]);
                if (lamp == 0.0 && -sp <= 1e-9 * (1.0 + fabs(bp) + ps)) {
                    if (pk >= 0) onrow[pk] = 2; /* skipped: no multiplier, not re-selected */
                    break;
                }
                status = WBQ_REF_INFEASIBLE;
                goto out;
            }
            const double t = t1 < t2 ? t1 : t2;
            if (isfinite(t2) || t1 < t2)
                for (int i = 0; i < n; ++i) x[i] += t * z[i];
            for (int a = 0; a < k; ++a) lam[a] -= t * r[a];
            lamp += t;
            if (t2 <= t1) { /* add p */
                memcpy(A + (size_t)k * n, np, sizeof(double) * n);
                ab[k] = bp;
                lam[k] = lamp;
                kind[k] = pk;
                if (pk >= 0) onrow[pk] = 1;
                ++k;
                break;
            }
            /* drop the blocking inequality, keep p */
            onrow[kind[blk]] = 0;
            for (int a = blk; a + 1 < k; ++a) {
                memcpy(A + (size_t)a * n, A + (size_t)(a + 1) * n, sizeof(double) * n);
                ab[a] = ab[a + 1];
                lam[a] = lam[a + 1];
                kind[a] = kind[a + 1];
            }
            --k;
        }
    }
    if (status == WBQ_REF_OK) {
        /* the incremental x must meet every row: a degenerate active set whose steps drifted is a
         * numerical failure, never a silent success */
        for (int j = 0; j < me && status == WBQ_REF_OK; ++j) {
            double s = 0.0;
            for (int i = 0; i < n; ++i) s += E[(size_t)j * n + i] * x[i];
            if (fabs(s - e[j]) > 1e-8 * cmaxd(1.0, cmaxd(fabs(s), fabs(e[j])))) status = WBQ_REF_NUMERICAL;
        }
        for (int j = 0; j < mi && status == WBQ_REF_OK; ++j) {
            double s = 0.0;
            for (int i = 0; i < n; ++i) s += C[(size_t)j * n + i] * x[i];
            const double sc = 1e-8 * cmaxd(1.0, cmaxd(fabs(s), cmaxd(fin(clo[j]), fin(chi[j]))));
            if (clo[j] - s > sc || s - chi[j] > sc) status = WBQ_REF_NUMERICAL;
        }
    }
out:
    if (iters) *iters = it;
    free(A);
    free(ab);
    free(lam);
    free(kind);
    free(z);
    free(r);
    free(np);
    free(Hc);
    free(onrow);
    return status;
}

/* Problem of one level: H [nx][nx], g [nx], E [12][nx], e [12], C [mi][nx], clo/chi [mi]. */
typedef struct {
    int nx, me, mi;
    double *H, *g, *E, *e, *C, *clo, *chi;
} level_qp;

static void level_alloc(level_qp *L, int nx, int me, int mi)
{
    L->nx = nx;
    L->me = me;
    L->mi = mi;
    L->H = (double *)calloc((size_t)nx * nx, sizeof(double));
    L->g = (double *)calloc((size_t)nx, sizeof(double));
    L->E = (double *)calloc((size_t)me * nx, sizeof(double));
    L->e = (double *)calloc((size_t)me, sizeof(double));
    L->C = (double *)calloc((size_t)(mi > 0 ? mi : 1) * nx, sizeof(double));
    L->clo = (double *)calloc((size_t)(mi > 0 ? mi : 1), sizeof(double));
    L->chi = (double *)calloc((size_t)(mi > 0 ? mi : 1), sizeof(double));
}

static void level_free(level_qp *L)
{
    free(L->H);
    free(L->g);
    free(L->E);
    free(L->e);
    free(L->C);
    free(L->clo);
    free(L->chi);
}

/* Cartesian acceleration task rhs: b = Kp e - Kd J qd - Jdot qd (ForceAcc.cpp:83-89,118-122) */
static void cart_acc_rhs(int n, const double *J, const double *jdqd, const double *pose, const double *pose_ref,
                         double Kp, double Kd, const double *qd, double b[6])
{
    double e[6];
    wbq_ref_cart_error(pose, pose_ref, e);
    for (int r = 0; r < 6; ++r) {
        double xd = 0.0;
        for (int j = 0; j < n; ++j) xd += J[r * n + j] * qd[j];
        b[r] = Kp * e[r] - Kd * xd - jdqd[r];
    }
}

int wbq_ref_contact_assemble(const wbq_ref_contact_desc *d, const wbq_ref_contact_instance *in, double *H1,
                             double *g1, double *E, double *e, double *C, double *clo, double *chi, double *bw)
{
    const int n = d->n, nc = d->nc, nfb = d->n_fb, wd = wbq_ref_contact_wd(d), nx = n + wd * nc;
    const int nfr = d->mu > 0.0 ? 4 * nc : 0;
    const int mi = wd * nc + nfr + (d->torque_rows ? n - nfb : 0);
    double bc[6];
    memset(H1, 0, sizeof(double) * nx * nx);
    memset(g1, 0, sizeof(double) * nx);
    /* postural (ForceAcc.cpp:105-107): H += I, g -= b_p */
    for (int i = 0; i < n; ++i) {
        H1[i * nx + i] += 1.0;
        g1[i] -= d->Kp_p * (in->qref[i] - in->q[i]) - d->Kd_p * in->qd[i];
    }
    /* feet Cartesian acceleration tasks (:83-89): H += J^T J, g -= J^T b */
    for (int c = 0; c < nc; ++c) {
        const double *J = in->Jc + (size_t)c * 6 * n;
        cart_acc_rhs(n, J, in->jdqd_c + 6 * c, in->pose_c + 12 * c, in->pose_c_ref + 12 * c, d->Kp_f, d->Kd_f, in->qd,
                     bc);
        for (int i = 0; i < n; ++i) {
            for (int j = 0; j < n; ++j) {
                double s = 0.0;
                for (int r = 0; r < 6; ++r) s += J[r * n + i] * J[r * n + j];
                H1[i * nx + j] += s;
            }
            double s = 0.0;
            for (int r = 0; r < 6; ++r) s += J[r * n + i] * bc[r];
            g1[i] -= s;
        }
    }
    /* min-norm tie-break on the forces */
    for (int k = n; k < nx; ++k) H1[k * nx + k] = d->eps_f;
    /* waist task (level 0; appears on level 1 as J_w qdd = y0*) */
    cart_acc_rhs(n, in->Jw, in->jdqd_w, in->pose_w, in->pose_w_ref, d->Kp_w, d->Kd_w, in->qd, bw);
    memset(E, 0, sizeof(double) * 12 * nx);
    for (int r = 0; r < 6; ++r) {
        for (int j = 0; j < n; ++j) E[r * nx + j] = in->Jw[r * n + j];
        e[r] = bw[r];
    }
    /* DynamicFeasibility (:109-114): M_fb qdd - sum_c J_c[0:3, fb]^T f_c = -h_fb */
    for (int r = 0; r < nfb; ++r) {
        double *er = E + (size_t)(6 + r) * nx;
        for (int j = 0; j < n; ++j) er[j] = in->M[r * n + j];
        for (int c = 0; c < nc; ++c)
            for (int k = 0; k < wd; ++k) er[n + wd * c + k] = -in->Jc[((size_t)c * 6 + k) * n + r];
        e[6 + r] = -in->h[r];
    }
    /* force box (:74-76,91-95); inactive contacts fixed at zero */
    memset(C, 0, sizeof(double) * (size_t)(mi > 0 ? mi : 1) * nx);
    for (int c = 0; c < nc; ++c) {
        const int on = (in->contact_mask >> c) & 1;
        for (int k = 0; k < wd; ++k) {
            const int row = wd * c + k;
            C[row * nx + n + wd * c + k] = 1.0;
            clo[row] = on ? (k < 3 ? d->f_lb[k] : d->m_lb[k - 3]) : 0.0;
            chi[row] = on ? (k < 3 ? d->f_ub[k] : d->m_ub[k - 3]) : 0.0;
        }
    }
    /* friction pyramid: s_x f_x - mu f_z <= 0 (faces +x, -x), s_y f_y - mu f_z <= 0 (+y, -y);
     * an inactive contact's rows are left unbounded (its forces are fixed at zero) */
    for (int c = 0; c < nfr / 4; ++c) {
        const int on = (in->contact_mask >> c) & 1;
        for (int k = 0; k < 4; ++k) {
            const int row = wd * nc + 4 * c + k;
            double *cr = C + (size_t)row * nx + n + wd * c;
            cr[k < 2 ? 0 : 1] = (k & 1) ? -1.0 : 1.0;
            cr[2] = -d->mu;
            clo[row] = -1e300;
            chi[row] = on ? 0.0 : 1e300;
        }
    }
    /* a12: actuated torque rows tau_min - h_a <= M_a qdd - sum_c J_c[0:3, a]^T f_c <= tau_max - h_a */
    if (d->torque_rows)
        for (int a = nfb; a < n; ++a) {
            const int row = wd * nc + nfr + (a - nfb);
            double *cr = C + (size_t)row * nx;
            for (int j = 0; j < n; ++j) cr[j] = in->M[a * n + j];
            for (int c = 0; c < nc; ++c)
                for (int k = 0; k < wd; ++k) cr[n + wd * c + k] = -in->Jc[((size_t)c * 6 + k) * n + a];
            clo[row] = d->tau_min[a] - in->h[a];
            chi[row] = d->tau_max[a] - in->h[a];
        }
    return mi;
}

int wbq_ref_contact_one(const wbq_ref_contact_desc *d, const wbq_ref_contact_instance *in, double *tau,
                        double *x, int *iters, int *l0_repaired)
{
    const int n = d->n, nc = d->nc, wd = wbq_ref_contact_wd(d), nx = n + wd * nc;
    const int mi = wd * nc + (d->mu > 0.0 ? 4 * nc : 0) + (d->torque_rows ? n - d->n_fb : 0);
    level_qp L;
    level_alloc(&L, nx, 12, mi);
    double bw[6];
    int it1 = 0, it0 = 0, status;
    wbq_ref_contact_assemble(d, in, L.H, L.g, L.E, L.e, L.C, L.clo, L.chi, bw);
    if (l0_repaired) *l0_repaired = 0;
    /* level 0 attained at b_w (the generic case): level 1 with J_w qdd = b_w */
    status = wbq_ref_dual_qp(nx, L.H, L.g, L.me, L.E, L.e, L.mi, L.C, L.clo, L.chi, x, &it1);
    /* an unattainable waist target shows as "no step" (infeasible), but near the degenerate face it
     * can also end the active set numerically (status 3) or cycling (1): every failure tries level 0
     * first (the GPU routes the same statuses to its repair kernel, contact_kernel.hip) */
    if (status != WBQ_REF_OK) {
        /* level 0 not attainable at b_w: y0* from the level-0 QP (its Hessian J_w^T J_w is
         * singular; a relative 1e-10 ridge only picks among level-0 optima), then level 1 */
        level_qp Z;
        level_alloc(&Z, nx, 6, mi);
        double dmx = 1.0;
        for (int i = 0; i < n; ++i)
            for (int r = 0; r < 6; ++r) dmx = cmaxd(dmx, in->Jw[r * n + i] * in->Jw[r * n + i]);
        for (int i = 0; i < n; ++i) {
            for (int j = 0; j < n; ++j) {
                double s = 0.0;
                for (int r = 0; r < 6; ++r) s += in->Jw[r * n + i] * in->Jw[r * n + j];
                Z.H[i * nx + j] = s;
            }
            double s = 0.0;
            for (int r = 0; r < 6; ++r) s += in->Jw[r * n + i] * bw[r];
            Z.g[i] = -s;
        }
        for (int k = 0; k < nx; ++k) Z.H[k * nx + k] += 1e-10 * dmx;
        memcpy(Z.E, L.E + 6 * nx, sizeof(double) * 6 * nx);
        memcpy(Z.e, L.e + 6, sizeof(double) * 6);
        memcpy(Z.C, L.C, sizeof(double) * (size_t)(mi > 0 ? mi : 1) * nx);
        memcpy(Z.clo, L.clo, sizeof(double) * (mi > 0 ? mi : 1));
        memcpy(Z.chi, L.chi, sizeof(double) * (mi > 0 ? mi : 1));
        status = wbq_ref_dual_qp(nx, Z.H, Z.g, Z.me, Z.E, Z.e, Z.mi, Z.C, Z.clo, Z.chi, x, &it0);
        if (status == WBQ_REF_OK) {
            for (int r = 0; r < 6; ++r) {
                double s = 0.0;
                for (int j = 0; j < n; ++j) s += in->Jw[r * n + j] * x[j];
                L.e[r] = s;
            }
            if (l0_repaired) *l0_repaired = 1;
            status = wbq_ref_dual_qp(nx, L.H, L.g, L.me, L.E, L.e, L.mi, L.C, L.clo, L.chi, x, &it1);
        }
        level_free(&Z);
    }
    if (status == WBQ_REF_OK) {
        /* ForceAcc.cpp:206-218: tau = M qdd + h - sum_c J_c^T w_c (w_c = [f_c; 0] or the 6-D wrench) */
        for (int i = 0; i < n; ++i) {
            double s = in->h[i];
            for (int j = 0; j < n; ++j) s += in->M[i * n + j] * x[j];
            for (int c = 0; c < nc; ++c)
                for (int k = 0; k < wd; ++k) s -= in->Jc[((size_t)c * 6 + k) * n + i] * x[n + wd * c + k];
            tau[i] = s;
        }
    } else {
        for (int i = 0; i < n; ++i) tau[i] = in->h[i];
    }
    if (iters) *iters = it0 + it1;
    level_free(&L);
    return status;
}

void wbq_ref_contact_batch(const wbq_ref_contact_desc *d, int B, const double *M, const double *h, const double *q,
                           const double *qd, const double *qref, const double *Jw, const double *jdqd_w,
                           const double *pose_w, const double *pose_w_ref, const double *Jc, const double *jdqd_c,
                           const double *pose_c, const double *pose_c_ref, const int32_t *cmask, double *tau,
                           double *x, int32_t *status, int32_t *iters, int32_t *l0_repaired)
{
    const int n = d->n, nc = d->nc, nx = n + wbq_ref_contact_wd(d) * nc;
    for (int b = 0; b < B; ++b) {
        wbq_ref_contact_instance in;
        in.M = M + (size_t)b * n * n;
        in.h = h + (size_t)b * n;
        in.q = q + (size_t)b * n;
        in.qd = qd + (size_t)b * n;
        in.qref = qref + (size_t)b * n;
        in.Jw = Jw + (size_t)b * 6 * n;
        in.jdqd_w = jdqd_w + (size_t)b * 6;
        in.pose_w = pose_w + (size_t)b * 12;
        in.pose_w_ref = pose_w_ref + (size_t)b * 12;
        in.Jc = Jc + (size_t)b * nc * 6 * n;
        in.jdqd_c = jdqd_c + (size_t)b * nc * 6;
        in.pose_c = pose_c + (size_t)b * nc * 12;
        in.pose_c_ref = pose_c_ref + (size_t)b * nc * 12;
        in.contact_mask = cmask[b];
        int it = 0, rep = 0;
        const int st = wbq_ref_contact_one(d, &in, tau + (size_t)b * n, x + (size_t)b * nx, &it, &rep);
        status[b] = st;
        iters[b] = it;
        if (l0_repaired) l0_repaired[b] = rep;
    }
}
