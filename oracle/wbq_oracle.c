/*
 * wbq_oracle.c -- CPU restatement of the QPPVM per-tick solve (TEST INFRASTRUCTURE ONLY).
 * See wbq_oracle.h for scope, parity status and the reference lines each step follows.
 *
 * Plain C99, fp64, single-threaded, dense linear algebra written here (no Eigen /
 * LAPACK in the image). Algorithms:
 *   - task assembly in the reference's x-space form (explicit M^-1 via Cholesky);
 *   - level 0: Stark & Parker BVLS (bounded-variable least squares); only y* = A0 x0*
 *     is unique and only y* is handed to level 1 (the OpenSoT hierarchy constrains
 *     level 1 with A0 x = A0 x0*);
 *   - level 1: primal active-set QP on the simple bounds with the level-0 optimality
 *     equalities kept in every KKT system (LU with partial pivoting).
 */
#include "wbq_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ helpers */

static double dmax(double a, double b) { return a > b ? a : b; }
static double dmin(double a, double b) { return a < b ? a : b; }

/* In-place Cholesky A = L L^T (lower, row-major N x N). Returns 0 on success. */
static int chol(int N, double *A)
{
    for (int j = 0; j < N; ++j) {
        double s = A[j * N + j];
        for (int k = 0; k < j; ++k) s -= A[j * N + k] * A[j * N + k];
        if (!(s > 0.0)) return -1;
        double Ljj = sqrt(s);
        A[j * N + j] = Ljj;
        for (int i = j + 1; i < N; ++i) {
            double t = A[i * N + j];
            for (int k = 0; k < j; ++k) t -= A[i * N + k] * A[j * N + k];
            A[i * N + j] = t / Ljj;
        }
        for (int k = j + 1; k < N; ++k) A[j * N + k] = 0.0;
    }
    return 0;
}

/* Inverse of an SPD matrix through its Cholesky factor. Returns 0 on success. */
static int spd_inverse(int N, const double *A, double *Ainv)
{
    double *L = (double *)malloc(sizeof(double) * N * N);
    double *col = (double *)malloc(sizeof(double) * N);
    memcpy(L, A, sizeof(double) * N * N);
    int rc = chol(N, L);
    if (rc == 0) {
        for (int c = 0; c < N; ++c) {
            /* solve L y = e_c, then L^T x = y */
            for (int i = 0; i < N; ++i) {
                double t = (i == c) ? 1.0 : 0.0;
                for (int k = 0; k < i; ++k) t -= L[i * N + k] * col[k];
                col[i] = t / L[i * N + i];
            }
            for (int i = N - 1; i >= 0; --i) {
                double t = col[i];
                for (int k = i + 1; k < N; ++k) t -= L[k * N + i] * col[k];
                col[i] = t / L[i * N + i];
            }
            for (int i = 0; i < N; ++i) Ainv[i * N + c] = col[i];
        }
        /* symmetrise the rounding */
        for (int i = 0; i < N; ++i)
            for (int j = i + 1; j < N; ++j) {
                double s = 0.5 * (Ainv[i * N + j] + Ainv[j * N + i]);
                Ainv[i * N + j] = s;
                Ainv[j * N + i] = s;
            }
    }
    free(L);
    free(col);
    return rc;
}

/* Solve A x = b in place (A N x N destroyed, b overwritten) by LU with partial pivoting.
 * Returns 0, or -1 when a pivot falls below rtol * max|A|. */
static int lu_solve(int N, double *A, double *b, double rtol)
{
    double amax = 0.0;
    for (int i = 0; i < N * N; ++i) amax = dmax(amax, fabs(A[i]));
    const double tiny = rtol * dmax(amax, 1e-300);
    for (int k = 0; k < N; ++k) {
        int p = k;
        double pv = fabs(A[k * N + k]);
        for (int i = k + 1; i < N; ++i)
            if (fabs(A[i * N + k]) > pv) {
                pv = fabs(A[i * N + k]);
                p = i;
            }
        if (pv <= tiny) return -1;
        if (p != k) {
            for (int j = 0; j < N; ++j) {
                double t = A[k * N + j];
                A[k * N + j] = A[p * N + j];
                A[p * N + j] = t;
            }
            double t = b[k];
            b[k] = b[p];
            b[p] = t;
        }
        const double inv = 1.0 / A[k * N + k];
        for (int i = k + 1; i < N; ++i) {
            const double f = A[i * N + k] * inv;
            if (f == 0.0) continue;
            A[i * N + k] = f;
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

/* One-sided Jacobi (Hestenes) SVD of X (R x C, row-major, C <= R is not required):
 * orthogonalises the columns, X V = U diag(sig). On return X holds U diag(sig) (columns
 * not normalised), V (C x C) the right singular vectors, sig the column norms. Singular
 * values come out to relative accuracy, unlike eigenvalues of the Gram X^T X. */
static void jacobi_svd(int R, int C, double *X, double *V, double *sig)
{
    for (int i = 0; i < C * C; ++i) V[i] = 0.0;
    for (int i = 0; i < C; ++i) V[i * C + i] = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        int rotated = 0;
        for (int p = 0; p < C; ++p)
            for (int q = p + 1; q < C; ++q) {
                double al = 0.0, be = 0.0, ga = 0.0;
                for (int k = 0; k < R; ++k) {
                    al += X[k * C + p] * X[k * C + p];
                    be += X[k * C + q] * X[k * C + q];
                    ga += X[k * C + p] * X[k * C + q];
                }
                if (fabs(ga) <= 1e-15 * sqrt(al * be) || ga == 0.0) continue;
                rotated = 1;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
                for (int k = 0; k < R; ++k) {
                    const double xp = X[k * C + p], xq = X[k * C + q];
                    X[k * C + p] = c * xp - sn * xq;
                    X[k * C + q] = sn * xp + c * xq;
                }
                for (int k = 0; k < C; ++k) {
                    const double vp = V[k * C + p], vq = V[k * C + q];
                    V[k * C + p] = c * vp - sn * vq;
                    V[k * C + q] = sn * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    for (int j = 0; j < C; ++j) {
        double s2 = 0.0;
        for (int k = 0; k < R; ++k) s2 += X[k * C + j] * X[k * C + j];
        sig[j] = sqrt(s2);
    }
}

/* Minimum-norm least squares over the columns F of A (m x n): z = pinv(A_F) r, via the SVD
 * of A_F^T (k x m): A_F^T V = U S  =>  A_F = V S U^T  =>  pinv(A_F) = U S^-1 V^T. */
static void minnorm_ls_floor(int m, int n, const double *A, const int *F, int k, const double *r, double *z,
                             double floor);
static void minnorm_ls(int m, int n, const double *A, const int *F, int k, const double *r,
                       double *z)
{
    minnorm_ls_floor(m, n, A, F, k, r, z, 0.0);
}

/* Same, singular values also dropped below an absolute floor (a matrix that is zero up to roundoff
 * has no directions: a relative cut would keep its roundoff). */
static void minnorm_ls_floor(int m, int n, const double *A, const int *F, int k, const double *r, double *z,
                             double floor)
{
    double *X = (double *)malloc(sizeof(double) * (k > 0 ? k : 1) * m);
    double *V = (double *)malloc(sizeof(double) * m * m);
    double *sig = (double *)malloc(sizeof(double) * m);
    double *t = (double *)malloc(sizeof(double) * m);
    for (int c = 0; c < k; ++c)
        for (int a = 0; a < m; ++a) X[c * m + a] = A[a * n + F[c]];
    jacobi_svd(k, m, X, V, sig);
    double smax = 0.0;
    for (int j = 0; j < m; ++j) smax = dmax(smax, sig[j]);
    for (int j = 0; j < m; ++j) {
        double s = 0.0;
        for (int a = 0; a < m; ++a) s += V[a * m + j] * r[a];
        /* U_j = X_j / sig_j, and z = sum_j U_j (V_j . r) / sig_j  => X_j (V_j . r) / sig_j^2 */
        t[j] = (sig[j] > 1e-13 * smax && sig[j] > floor) ? s / (sig[j] * sig[j]) : 0.0;
    }
    for (int c = 0; c < k; ++c) {
        double s = 0.0;
        for (int j = 0; j < m; ++j) s += X[c * m + j] * t[j];
        z[c] = s;
    }
    free(X);
    free(V);
    free(sig);
    free(t);
}

/* ------------------------------------------------------------ task assembly */

void wbq_ref_cart_error(const double pose[12], const double pose_ref[12], double e[6])
{
    /* position error p_ref - p */
    e[0] = pose_ref[3] - pose[3];
    e[1] = pose_ref[7] - pose[7];
    e[2] = pose_ref[11] - pose[11];
    /* Re = Rref * R^T */
    double Re[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += pose_ref[i * 4 + k] * pose[j * 4 + k];
            Re[i * 3 + j] = s;
        }
    /* Shepperd's method; sign fixed so that the scalar part is >= 0 (the reference's
     * quaternion error flips q when dot(q, qd) < 0 [upstream cartesian_utils]). */
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
    e[3] = sg * qx;
    e[4] = sg * qy;
    e[5] = sg * qz;
}

int wbq_ref_assemble(const wbq_ref_desc *d, const wbq_ref_instance *in, double *A0, double *b0,
                     double *H1, double *g1, double *lb, double *ub)
{
    const int n = d->n;
    double *Minv = (double *)malloc(sizeof(double) * n * n);
    double *JMi = (double *)malloc(sizeof(double) * 6 * n);
    double *c = (double *)malloc(sizeof(double) * n);
    double *W = (double *)malloc(sizeof(double) * n * n);
    double *tmp = (double *)malloc(sizeof(double) * n * n);
    double *timp = (double *)malloc(sizeof(double) * n);
    double *b1 = (double *)malloc(sizeof(double) * n);
    int m0 = 0;
    if (spd_inverse(n, in->M, Minv) != 0) {
        m0 = -WBQ_REF_NUMERICAL;
        goto done;
    }
    /* ---- level 0: Cartesian impedance tasks (QPPVMPlugin.cpp:129-152), summed (:177); with a middle
     * level (task_level, the elbow tasks :154-166,178) its tasks' rows follow the level-0 rows */
    for (int tt = 0; tt < 2 * d->ntasks; ++tt) {
        const int t = tt % d->ntasks;
        if ((d->task_level[t] != 0) != (tt >= d->ntasks)) continue;
        const double *J = in->J + (size_t)t * 6 * n;
        double e[6], xdot[6], F[6], b6[6];
        wbq_ref_cart_error(in->pose + 12 * t, in->pose_ref + 12 * t, e);
        for (int r = 0; r < 6; ++r) {
            double s = 0.0;
            for (int j = 0; j < n; ++j) s += J[r * n + j] * in->qd[j];
            xdot[r] = s;
            /* spring + damper with zero desired twist */
            F[r] = d->Kc[6 * t + r] * e[r] - d->Dc[6 * t + r] * xdot[r];
            if (d->select_mode == WBQ_REF_SELECT_TASK && !((d->row_mask[t] >> r) & 1)) F[r] = 0.0;
        }
        /* A6 = J M^-1 (useInertiaMatrix(true), :139,:151) */
        for (int r = 0; r < 6; ++r)
            for (int j = 0; j < n; ++j) {
                double s = 0.0;
                for (int k = 0; k < n; ++k) s += J[r * n + k] * Minv[k * n + j];
                JMi[r * n + j] = s;
            }
        /* b6 = J M^-1 J^T F */
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int r = 0; r < 6; ++r) s += J[r * n + j] * F[r];
            c[j] = s;
        }
        for (int r = 0; r < 6; ++r) {
            double s = 0.0;
            for (int j = 0; j < n; ++j) s += JMi[r * n + j] * c[j];
            b6[r] = s;
        }
        for (int r = 0; r < 6; ++r) {
            if (!((d->row_mask[t] >> r) & 1)) continue;
            memcpy(A0 + (size_t)m0 * n, JMi + (size_t)r * n, sizeof(double) * n);
            b0[m0] = b6[r];
            ++m0;
        }
    }
    /* ---- level 1: joint impedance task (QPPVMPlugin.cpp:114-118): A1 = M^-1, b1 = M^-1 tau_imp */
    for (int j = 0; j < n; ++j)
        timp[j] = d->Kq[j] * (in->qref[j] - in->q[j]) - d->Dq[j] * in->qd[j];
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += Minv[i * n + j] * timp[j];
        b1[i] = s;
    }
    if (d->no_joint_task) {
        /* no joint task (QPPVMPlugin.cpp:177-178 in place of :179): the last level's optima are
         * decided by qpOASES' eps I regularisation (:188), eps -> 0: min 0.5 ||x||^2 */
        for (int i = 0; i < n * n; ++i) H1[i] = (i % (n + 1) == 0) ? 1.0 : 0.0;
        for (int i = 0; i < n; ++i) g1[i] = 0.0;
        goto bounds;
    }
    /* W1 */
    if (d->joint_weight == WBQ_REF_WEIGHT_INERTIA)
        memcpy(W, in->M, sizeof(double) * n * n);
    else
        for (int i = 0; i < n * n; ++i) W[i] = (i % (n + 1) == 0) ? 1.0 : 0.0;
    /* H1 = A1^T W A1, g1 = -A1^T W b1 (A1 = M^-1 symmetric) */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int k = 0; k < n; ++k) s += W[i * n + k] * Minv[k * n + j];
            tmp[i * n + j] = s; /* W A1 */
        }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int k = 0; k < n; ++k) s += Minv[k * n + i] * tmp[k * n + j];
            H1[i * n + j] = s;
        }
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {
            const double s = 0.5 * (H1[i * n + j] + H1[j * n + i]);
            H1[i * n + j] = H1[j * n + i] = s;
        }
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int k = 0; k < n; ++k) s += tmp[k * n + i] * b1[k];
        g1[i] = -s;
    }
bounds:
    /* ---- torque limits shifted by -h (QPPVMPlugin.cpp:66-67, 203-205), and with the JointLimits
     * toggle (:169-171) the joint-limit barrier Kjl (q_lim - q) - Djl qd on tau as well */
    for (int j = 0; j < n; ++j) {
        double lo = d->tau_min[j], hi = d->tau_max[j];
        if (d->joint_limits) {
            const double bl = d->Kjl[j] * (d->q_min[j] - in->q[j]) - d->Djl[j] * in->qd[j];
            const double bu = d->Kjl[j] * (d->q_max[j] - in->q[j]) - d->Djl[j] * in->qd[j];
            lo = bl > lo ? bl : lo;
            hi = bu < hi ? bu : hi;
        }
        lb[j] = lo - in->h[j];
        ub[j] = hi - in->h[j];
    }
done:
    free(Minv);
    free(JMi);
    free(c);
    free(W);
    free(tmp);
    free(timp);
    free(b1);
    return m0;
}

/* ---------------------------------------------------------------- level 0 */

int wbq_ref_level0(int m, int n, const double *A, const double *b, const double *lb,
                   const double *ub, double *x, int *state, int *iters)
{
    int *F = (int *)malloc(sizeof(int) * n);
    int *excl = (int *)calloc((size_t)n, sizeof(int));
    double *r = (double *)malloc(sizeof(double) * m);
    double *z = (double *)malloc(sizeof(double) * n);
    double *w = (double *)malloc(sizeof(double) * n);
    int status = WBQ_REF_MAXITER, it = 0;
    const int maxit = 50 * n + 100;

    for (int i = 0; i < n; ++i) {
        if (lb[i] > ub[i]) {
            status = WBQ_REF_INFEASIBLE;
            goto out;
        }
        if (state[i] < 0)
            x[i] = lb[i];
        else if (state[i] > 0)
            x[i] = ub[i];
        else
            x[i] = dmin(dmax(0.0, lb[i]), ub[i]);
        if (lb[i] == ub[i]) {
            state[i] = -1;
            x[i] = lb[i];
        }
    }
    double Abmax = 0.0;
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int a = 0; a < m; ++a) s += A[a * n + i] * b[a];
        Abmax = dmax(Abmax, fabs(s));
    }
    const double wtol = 1e-11 * dmax(1.0, Abmax);
    int freed = -1; /* variable freed by the last KKT step */

    while (it < maxit) {
        /* inner loop: solve on the free set, interpolate back into the box */
        for (;;) {
            ++it;
            int k = 0;
            for (int i = 0; i < n; ++i)
                if (state[i] == 0) F[k++] = i;
            if (k == 0) break;
            for (int a = 0; a < m; ++a) {
                double s = b[a];
                for (int i = 0; i < n; ++i)
                    if (state[i] != 0) s -= A[a * n + i] * x[i];
                r[a] = s;
            }
            minnorm_ls(m, n, A, F, k, r, z);
            double alpha = 1.0;
            int jblk = -1;
            for (int c = 0; c < k; ++c) {
                const int i = F[c];
                const double step = z[c] - x[i];
                if (z[c] < lb[i] && step < 0.0) {
                    const double a = (lb[i] - x[i]) / step;
                    if (a < alpha) alpha = a, jblk = c;
                } else if (z[c] > ub[i] && step > 0.0) {
                    const double a = (ub[i] - x[i]) / step;
                    if (a < alpha) alpha = a, jblk = c;
                }
            }
            if (jblk < 0) {
                for (int c = 0; c < k; ++c) x[F[c]] = z[c];
                freed = -1;
                for (int i = 0; i < n; ++i) excl[i] = 0; /* progress: exclusions expire */
                break;
            }
            if (alpha < 0.0) alpha = 0.0;
            if (F[jblk] == freed && alpha == 0.0) {
                /* the variable just freed wants to go back through its bound: the KKT sign was
                 * rounding noise (Stark-Parker); re-bind it and exclude it from this round */
                const int i = F[jblk];
                excl[i] = 1;
                state[i] = (z[jblk] < lb[i]) ? -1 : 1;
                x[i] = state[i] < 0 ? lb[i] : ub[i];
                freed = -1;
                break;
            }
            for (int i = 0; i < n; ++i) excl[i] = 0; /* progress: exclusions expire */
            for (int c = 0; c < k; ++c) {
                const int i = F[c];
                x[i] += alpha * (z[c] - x[i]);
                const double tl = 1e-14 * dmax(1.0, fabs(lb[i]));
                const double tu = 1e-14 * dmax(1.0, fabs(ub[i]));
                if (c == jblk) {
                    state[i] = (z[c] < lb[i]) ? -1 : 1;
                } else if (x[i] <= lb[i] + tl && z[c] < lb[i]) {
                    state[i] = -1;
                } else if (x[i] >= ub[i] - tu && z[c] > ub[i]) {
                    state[i] = 1;
                }
                if (state[i] < 0) x[i] = lb[i];
                if (state[i] > 0) x[i] = ub[i];
            }
            freed = -1;
            if (it >= maxit) break;
        }
        /* KKT on the bound variables: w = A^T (b - A x) */
        for (int a = 0; a < m; ++a) {
            double s = b[a];
            for (int i = 0; i < n; ++i) s -= A[a * n + i] * x[i];
            r[a] = s;
        }
        int best = -1;
        double bestv = wtol;
        for (int i = 0; i < n; ++i) {
            double s = 0.0;
            for (int a = 0; a < m; ++a) s += A[a * n + i] * r[a];
            w[i] = s;
            if (state[i] == 0 || excl[i] || lb[i] == ub[i]) continue;
            const double v = (state[i] < 0) ? s : -s;
            if (v > bestv) bestv = v, best = i;
        }
        if (best < 0) {
            status = WBQ_REF_OK;
            break;
        }
        state[best] = 0; /* exclusions persist until the inner loop makes progress */
        freed = best;
    }
out:
    if (iters) *iters = it;
    free(F);
    free(excl);
    free(r);
    free(z);
    free(w);
    return status;
}

int wbq_ref_task_rows(const wbq_ref_desc *d, int *m_l0)
{
    int m = 0, m0 = 0;
    for (int t = 0; t < d->ntasks; ++t)
        for (int r = 0; r < 6; ++r)
            if ((d->row_mask[t] >> r) & 1) {
                ++m;
                if (d->task_level[t] == 0) ++m0;
            }
    if (m_l0) *m_l0 = m0;
    return m;
}

/* ----------------------------------------------------------- middle level */

/* Free-set step of the middle level: d = argmin ||A_F d - r|| over d in null(E_F), minimum norm.
 * With E_F^T = U S V^T (one-sided Jacobi), P = I - U U^T projects onto null(E_F) and the minimum-norm
 * solution of (A_F P) t = r lies in range(P A_F^T), so d = t already meets E_F d = 0. Returns 0 when
 * null(E_F) is empty (d = 0): then P is zero up to roundoff, which the solve must not amplify. */
static int mid_step(int me, const double *E, int m, int n, const double *A, const int *F, int k, const double *r,
                    double *d)
{
    const int mq = me > 0 ? me : 1, kq = k > 0 ? k : 1;
    double *X = (double *)malloc(sizeof(double) * kq * mq);
    double *V = (double *)malloc(sizeof(double) * mq * mq);
    double *sig = (double *)malloc(sizeof(double) * mq);
    double *P = (double *)malloc(sizeof(double) * kq * kq);
    double *B = (double *)malloc(sizeof(double) * m * kq);
    int *all = (int *)malloc(sizeof(int) * kq);
    for (int c = 0; c < k; ++c)
        for (int a = 0; a < me; ++a) X[c * me + a] = E[a * n + F[c]];
    for (int i = 0; i < k * k; ++i) P[i] = (i % (k + 1) == 0) ? 1.0 : 0.0;
    int rank = 0;
    if (me > 0 && k > 0) {
        jacobi_svd(k, me, X, V, sig);
        double smax = 0.0;
        for (int j = 0; j < me; ++j) smax = dmax(smax, sig[j]);
        for (int j = 0; j < me; ++j) {
            if (!(sig[j] > 1e-12 * smax)) continue;
            ++rank;
            for (int a = 0; a < k; ++a)
                for (int c = 0; c < k; ++c) P[a * k + c] -= X[a * me + j] * X[c * me + j] / (sig[j] * sig[j]);
        }
    }
    double amax = 0.0;
    for (int a = 0; a < m; ++a)
        for (int c = 0; c < k; ++c) amax = dmax(amax, fabs(A[a * n + F[c]]));
    if (rank >= k || k == 0) {
        for (int c = 0; c < k; ++c) d[c] = 0.0;
        free(X);
        free(V);
        free(sig);
        free(P);
        free(B);
        free(all);
        return 0;
    }
    for (int a = 0; a < m; ++a)
        for (int c = 0; c < k; ++c) {
            double s = 0.0;
            for (int q = 0; q < k; ++q) s += A[a * n + F[q]] * P[q * k + c];
            B[a * k + c] = s;
        }
    for (int c = 0; c < k; ++c) all[c] = c;
    minnorm_ls_floor(m, k, B, all, k, r, d, 1e-12 * amax * sqrt((double)k));
    free(X);
    free(V);
    free(sig);
    free(P);
    free(B);
    free(all);
    return 1;
}

/* multipliers of the bound variables at x: w = A^T (b - A x) - E^T nu, nu the least-squares fit of the
 * free variables' gradient by the equality rows (E_F^T nu = A_F^T (b - A x)) */
static void mid_multipliers(int me, const double *E, int m, int n, const double *A, const double *b,
                            const double *x, const int *F, int k, double *w)
{
    const int mq = me > 0 ? me : 1, kq = k > 0 ? k : 1;
    double *r = (double *)malloc(sizeof(double) * m);
    double *Et = (double *)malloc(sizeof(double) * kq * mq);
    double *gF = (double *)malloc(sizeof(double) * kq);
    double *nu = (double *)calloc((size_t)mq, sizeof(double));
    int *all = (int *)malloc(sizeof(int) * mq);
    for (int a = 0; a < m; ++a) {
        double s = b[a];
        for (int j = 0; j < n; ++j) s -= A[a * n + j] * x[j];
        r[a] = s;
    }
    for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int a = 0; a < m; ++a) s += A[a * n + j] * r[a];
        w[j] = s;
    }
    if (me > 0 && k > 0) {
        for (int c = 0; c < k; ++c) {
            gF[c] = w[F[c]];
            for (int a = 0; a < me; ++a) Et[c * me + a] = E[a * n + F[c]];
        }
        for (int a = 0; a < me; ++a) all[a] = a;
        minnorm_ls(k, me, Et, all, me, gF, nu);
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int a = 0; a < me; ++a) s += E[a * n + j] * nu[a];
            w[j] -= s;
        }
    }
    free(r);
    free(Et);
    free(gF);
    free(nu);
    free(all);
}

int wbq_ref_level_mid(int me, const double *E, int m, int n, const double *A, const double *b, const double *lb,
                      const double *ub, double *x, int *state, double *w_out, int *iters)
{
    int *F = (int *)malloc(sizeof(int) * n);
    int *excl = (int *)calloc((size_t)n, sizeof(int));
    double *r = (double *)malloc(sizeof(double) * m);
    double *dz = (double *)malloc(sizeof(double) * n);
    double *w = (double *)malloc(sizeof(double) * n);
    int status = WBQ_REF_MAXITER, it = 0;
    const int maxit = 50 * n + 100;
    for (int i = 0; i < n; ++i) {
        if (lb[i] == ub[i]) state[i] = -1;
        if (state[i] < 0) x[i] = lb[i];
        if (state[i] > 0) x[i] = ub[i];
    }
    double Abmax = 0.0, xmax = 1.0;
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int a = 0; a < m; ++a) s += A[a * n + i] * b[a];
        Abmax = dmax(Abmax, fabs(s));
        xmax = dmax(xmax, fabs(x[i]));
    }
    const double wtol = 1e-11 * dmax(1.0, Abmax);
    int freed = -1;
    while (it < maxit) {
        for (;;) { /* inner loop: step on the free set inside null(E_F), interpolate back into the box */
            ++it;
            int k = 0;
            for (int i = 0; i < n; ++i)
                if (state[i] == 0) F[k++] = i;
            if (k == 0) break;
            for (int a = 0; a < m; ++a) {
                double s = b[a];
                for (int i = 0; i < n; ++i) s -= A[a * n + i] * x[i];
                r[a] = s;
            }
            if (!mid_step(me, E, m, n, A, F, k, r, dz)) break; /* no direction left on the free set */
            double dmx = 0.0;
            for (int c = 0; c < k; ++c) dmx = dmax(dmx, fabs(dz[c]));
            if (dmx <= 1e-15 * xmax) break; /* stationary on the free set */
            double alpha = 1.0;
            int jblk = -1;
            for (int c = 0; c < k; ++c) {
                const int i = F[c];
                if (dz[c] < 0.0 && x[i] + dz[c] < lb[i]) {
                    const double a = (lb[i] - x[i]) / dz[c];
                    if (a < alpha) alpha = a, jblk = c;
                } else if (dz[c] > 0.0 && x[i] + dz[c] > ub[i]) {
                    const double a = (ub[i] - x[i]) / dz[c];
                    if (a < alpha) alpha = a, jblk = c;
                }
            }
            if (jblk < 0) {
                for (int c = 0; c < k; ++c) x[F[c]] += dz[c];
                freed = -1;
                for (int i = 0; i < n; ++i) excl[i] = 0;
                break;
            }
            if (alpha < 0.0) alpha = 0.0;
            if (F[jblk] == freed && alpha == 0.0) { /* Stark-Parker: re-bind, exclude */
                const int i = F[jblk];
                excl[i] = 1;
                state[i] = dz[jblk] < 0.0 ? -1 : 1;
                x[i] = state[i] < 0 ? lb[i] : ub[i];
                freed = -1;
                break;
            }
            for (int i = 0; i < n; ++i) excl[i] = 0;
            for (int c = 0; c < k; ++c) x[F[c]] += alpha * dz[c];
            {
                const int i = F[jblk];
                state[i] = dz[jblk] < 0.0 ? -1 : 1;
                x[i] = state[i] < 0 ? lb[i] : ub[i];
            }
            freed = -1;
            if (it >= maxit) break;
        }
        int k = 0;
        for (int i = 0; i < n; ++i)
            if (state[i] == 0) F[k++] = i;
        mid_multipliers(me, E, m, n, A, b, x, F, k, w);
        int best = -1;
        double bestv = wtol;
        for (int i = 0; i < n; ++i) {
            if (state[i] == 0 || excl[i] || lb[i] == ub[i]) continue;
            const double v = (state[i] < 0) ? w[i] : -w[i];
            if (v > bestv) bestv = v, best = i;
        }
        if (best < 0) {
            status = WBQ_REF_OK;
            break;
        }
        state[best] = 0;
        freed = best;
    }
    if (w_out) memcpy(w_out, w, sizeof(double) * n);
    if (iters) *iters = it;
    free(F);
    free(excl);
    free(r);
    free(dz);
    free(w);
    return status;
}

/* ---------------------------------------------------------------- level 1 */

int wbq_ref_level1(int n, const double *H, const double *g, int me, const double *Aeq,
                   const double *beq, const double *lb, const double *ub, double *x, int *state,
                   int *iters)
{
    /* Primal active set from a feasible point. The level-0 optimality rows Aeq x = beq are
     * reduced, on the current free set, to an orthonormal independent combination
     * (eigen-decomposition of Aeq_F Aeq_F^T): they become dependent when level 0 pins
     * variables to bounds. */
    const int N = n + me;
    const int mq = me > 0 ? me : 1;
    double *K = (double *)malloc(sizeof(double) * N * N);
    double *rhs = (double *)malloc(sizeof(double) * N);
    double *p = (double *)malloc(sizeof(double) * n);
    double *grad = (double *)malloc(sizeof(double) * n);
    double *Gm = (double *)malloc(sizeof(double) * mq * (n > mq ? n : mq));
    double *V = (double *)malloc(sizeof(double) * mq * mq);
    double *lam = (double *)malloc(sizeof(double) * mq);
    double *E2 = (double *)malloc(sizeof(double) * mq * n);
    double *r2 = (double *)malloc(sizeof(double) * mq);
    double *nu = (double *)malloc(sizeof(double) * mq);
    int *F = (int *)malloc(sizeof(int) * n);
    int status = WBQ_REF_MAXITER, it = 0, stationary = 0;
    const int maxit = 20 * n + 50;
    double scale = 1.0, gmax = 1.0;
    for (int i = 0; i < n; ++i) {
        scale = dmax(scale, fabs(x[i]));
        gmax = dmax(gmax, fabs(g[i]));
    }
    for (int i = 0; i < n; ++i) {
        if (lb[i] == ub[i]) state[i] = -1;
        if (state[i] < 0) x[i] = lb[i];
        if (state[i] > 0) x[i] = ub[i];
    }
    while (it++ < maxit) {
        int k = 0;
        for (int i = 0; i < n; ++i)
            if (state[i] == 0) F[k++] = i;
        /* independent equality rows on F */
        int r = 0;
        if (me > 0) {
            /* SVD of Aeq_F^T (k x me): the left singular vectors of Aeq_F are the columns of V */
            for (int c = 0; c < k; ++c)
                for (int a = 0; a < me; ++a) Gm[c * me + a] = Aeq[a * n + F[c]];
            jacobi_svd(k, me, Gm, V, lam);
            double lmax = 0.0;
            for (int a = 0; a < me; ++a) lmax = dmax(lmax, lam[a]);
            for (int e = 0; e < me; ++e) {
                if (!(lam[e] > 1e-12 * lmax) || lmax <= 0.0) continue;
                for (int c = 0; c < n; ++c) {
                    double t = 0.0;
                    for (int a = 0; a < me; ++a) t += V[a * me + e] * Aeq[a * n + c];
                    E2[r * n + c] = t;
                }
                double t = 0.0;
                for (int a = 0; a < me; ++a) t += V[a * me + e] * beq[a];
                r2[r] = t;
                ++r;
            }
        }
        const int NK = k + r;
        /* KKT on the free set: [H_FF E2_F^T; E2_F 0] [xF; nu] = [-g_F - H_FB x_B; r2 - E2_B x_B] */
        for (int a = 0; a < k; ++a) {
            for (int c = 0; c < k; ++c) K[a * NK + c] = H[F[a] * n + F[c]];
            for (int e = 0; e < r; ++e) K[a * NK + k + e] = E2[e * n + F[a]];
            double s = -g[F[a]];
            for (int j = 0; j < n; ++j)
                if (state[j] != 0) s -= H[F[a] * n + j] * x[j];
            rhs[a] = s;
        }
        for (int e = 0; e < r; ++e) {
            for (int c = 0; c < k; ++c) K[(k + e) * NK + c] = E2[e * n + F[c]];
            for (int f = 0; f < r; ++f) K[(k + e) * NK + k + f] = 0.0;
            double s = r2[e];
            for (int j = 0; j < n; ++j)
                if (state[j] != 0) s -= E2[e * n + j] * x[j];
            rhs[k + e] = s;
        }
        if (NK > 0 && lu_solve(NK, K, rhs, 1e-15) != 0) {
            status = WBQ_REF_NUMERICAL;
            break;
        }
        double pmax = 0.0;
        for (int a = 0; a < k; ++a) {
            p[a] = rhs[a] - x[F[a]];
            pmax = dmax(pmax, fabs(p[a]));
        }
        for (int e = 0; e < r; ++e) nu[e] = rhs[k + e];
        if (stationary || pmax <= 1e-13 * scale) {
            stationary = 0;
            /* stationary on the working set: bound multipliers grad_i = lambda_lo - lambda_hi */
            int best = -1;
            double bestv = 0.0, numax = 0.0;
            for (int i = 0; i < n; ++i) {
                double s = g[i], t = 0.0;
                for (int j = 0; j < n; ++j) s += H[i * n + j] * x[j];
                for (int e = 0; e < r; ++e) t += E2[e * n + i] * nu[e];
                grad[i] = s + t;
                numax = dmax(numax, fabs(t));
            }
            const double tol = 1e-10 * dmax(gmax, numax);
            for (int i = 0; i < n; ++i) {
                if (state[i] == 0 || lb[i] == ub[i]) continue;
                const double v = (state[i] < 0) ? -grad[i] : grad[i]; /* >0 means wrong sign */
                if (v > tol && v > bestv) bestv = v, best = i;
            }
            if (best < 0) {
                status = WBQ_REF_OK;
                break;
            }
            state[best] = 0;
            continue;
        }
        double alpha = 1.0;
        int jblk = -1;
        for (int a = 0; a < k; ++a) {
            const int i = F[a];
            if (p[a] < 0.0 && x[i] + p[a] < lb[i]) {
                const double t = (lb[i] - x[i]) / p[a];
                if (t < alpha) alpha = t, jblk = a;
            } else if (p[a] > 0.0 && x[i] + p[a] > ub[i]) {
                const double t = (ub[i] - x[i]) / p[a];
                if (t < alpha) alpha = t, jblk = a;
            }
        }
        if (alpha < 0.0) alpha = 0.0;
        for (int a = 0; a < k; ++a) x[F[a]] += alpha * p[a];
        stationary = (jblk < 0);
        if (jblk >= 0) {
            const int i = F[jblk];
            state[i] = (p[jblk] < 0.0) ? -1 : 1;
            x[i] = state[i] < 0 ? lb[i] : ub[i];
        }
    }
    if (iters) *iters = it;
    free(K);
    free(rhs);
    free(p);
    free(grad);
    free(Gm);
    free(V);
    free(lam);
    free(E2);
    free(r2);
    free(nu);
    free(F);
    return status;
}

/* ----------------------------------------------------------- whole chain */

int wbq_ref_qppvm_one(const wbq_ref_desc *d, const wbq_ref_instance *in, double *tau, double *y0,
                      int *iters)
{
    const int n = d->n;
    int m_l0 = 0;
    const int m0max = wbq_ref_task_rows(d, &m_l0);
    double *A0 = (double *)malloc(sizeof(double) * (m0max + 1) * n);
    double *b0 = (double *)malloc(sizeof(double) * (m0max + 1));
    double *y = (double *)malloc(sizeof(double) * (m0max + 1));
    double *H1 = (double *)malloc(sizeof(double) * n * n);
    double *g1 = (double *)malloc(sizeof(double) * n);
    double *lb = (double *)malloc(sizeof(double) * n);
    double *ub = (double *)malloc(sizeof(double) * n);
    double *x = (double *)malloc(sizeof(double) * n);
    int *state = (int *)calloc((size_t)n, sizeof(int));
    int it0 = 0, it1 = 0, status;

    const int m0 = wbq_ref_assemble(d, in, A0, b0, H1, g1, lb, ub);
    if (m0 < 0) {
        status = -m0;
        goto fallback;
    }
    {
        /* level 0 over its own rows (the first m_l0; all of them in the reference stack) */
        const int ml = m0 - (m0max - m_l0);
        status = wbq_ref_level0(ml, n, A0, b0, lb, ub, x, state, &it0);
        if (status != WBQ_REF_OK) goto fallback;
        for (int a = 0; a < ml; ++a) {
            double s = 0.0;
            for (int j = 0; j < n; ++j) s += A0[a * n + j] * x[j];
            y[a] = s;
        }
        /* Variables the level-0 gradient w = A0^T (b0 - y*) pins to a bound sit at that bound
         * in every level-0 optimum, hence everywhere in level 1's feasible set: fix them. */
        double wmax = 1.0;
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int a = 0; a < ml; ++a) s += A0[a * n + j] * b0[a];
            wmax = dmax(wmax, fabs(s));
        }
        for (int j = 0; j < n; ++j) {
            double w = 0.0;
            for (int a = 0; a < ml; ++a) w += A0[a * n + j] * (b0[a] - y[a]);
            if (w > 1e-9 * wmax) lb[j] = ub[j];
            else if (w < -1e-9 * wmax) ub[j] = lb[j];
            if (x[j] < lb[j]) x[j] = lb[j];
            if (x[j] > ub[j]) x[j] = ub[j];
        }
        if (ml < m0) {
            /* the middle level (the elbow tasks): its optimum y1* keeping level 0 at y0*, then the
             * variables its multipliers hold at a bound are fixed too */
            const int m1 = m0 - ml;
            double *w = (double *)malloc(sizeof(double) * n);
            int itm = 0;
            status = wbq_ref_level_mid(ml, A0, m1, n, A0 + (size_t)ml * n, b0 + ml, lb, ub, x, state, w, &itm);
            it0 += itm;
            if (status == WBQ_REF_OK) {
                for (int a = ml; a < m0; ++a) {
                    double s = 0.0;
                    for (int j = 0; j < n; ++j) s += A0[a * n + j] * x[j];
                    y[a] = s;
                }
                double wm = 1.0;
                for (int j = 0; j < n; ++j) {
                    double s = 0.0;
                    for (int a = ml; a < m0; ++a) s += A0[a * n + j] * b0[a];
                    wm = dmax(wm, fabs(s));
                }
                for (int j = 0; j < n; ++j) {
                    if (lb[j] == ub[j] || state[j] == 0) continue;
                    if (state[j] < 0 && w[j] < -1e-9 * wm) ub[j] = lb[j];
                    if (state[j] > 0 && w[j] > 1e-9 * wm) lb[j] = ub[j];
                }
            }
            free(w);
            if (status != WBQ_REF_OK) goto fallback;
        }
    }
    if (y0) memcpy(y0, y, sizeof(double) * m0);
    status = wbq_ref_level1(n, H1, g1, m0, A0, y, lb, ub, x, state, &it1);
    if (status != WBQ_REF_OK) goto fallback;
    for (int j = 0; j < n; ++j) tau[j] = x[j] + in->h[j];
    goto done;
fallback:
    /* QPPVMPlugin.cpp:246-249: "SOLVER ERROR!" -> tau_qp = 0 -> tau = h */
    for (int j = 0; j < n; ++j) tau[j] = in->h[j];
done:
    if (iters) *iters = it0 + it1;
    free(A0);
    free(b0);
    free(y);
    free(H1);
    free(g1);
    free(lb);
    free(ub);
    free(x);
    free(state);
    return status;
}

void wbq_ref_qppvm_batch(const wbq_ref_desc *d, int B, const double *M, const double *J,
                         const double *pose, const double *pose_ref, const double *q,
                         const double *qd, const double *qref, const double *h, double *tau,
                         int32_t *status, int32_t *iters)
{
    const size_t n = (size_t)d->n, T = (size_t)d->ntasks;
    for (int b = 0; b < B; ++b) {
        wbq_ref_instance in;
        in.M = M + (size_t)b * n * n;
        in.J = J + (size_t)b * T * 6 * n;
        in.pose = pose + (size_t)b * T * 12;
        in.pose_ref = pose_ref + (size_t)b * T * 12;
        in.q = q + (size_t)b * n;
        in.qd = qd + (size_t)b * n;
        in.qref = qref + (size_t)b * n;
        in.h = h + (size_t)b * n;
        int it = 0;
        const int st = wbq_ref_qppvm_one(d, &in, tau + (size_t)b * n, NULL, &it);
        if (status) status[b] = st;
        if (iters) iters[b] = it;
    }
}
