/* wbq_oracle_rbd.c -- CPU restatement of the rigid-body quantities the hot path consumes
 * (TEST INFRASTRUCTURE ONLY: the checker of qppvm_amd/csrc/rbd_kernel.hip, never the product).
 *
 * The reference takes them from XBotInterface's ModelInterface (RBDL backend, [upstream]):
 *   M(q)             getInertiaMatrix          (QPPVMPlugin.cpp:114-118 via the tasks, ForceAcc.cpp:208)
 *   h(q, qd)         computeNonlinearTerm      (QPPVMPlugin.cpp:65, :312)
 *   J_e(q), pose_e   getJacobian / getPose     (QPPVMPlugin.cpp:272, the Cartesian tasks :129-152)
 *   ID(q, qd, qdd)   computeInverseDynamics    (ForceAcc.cpp:208-217) = M qdd + h
 * This restatement uses the textbook recursions in LINK coordinates (Featherstone, "Rigid Body
 * Dynamics Algorithms", 2008: RNEA Table 5.1, CRBA Table 6.2); the GPU kernel uses world-frame
 * sums over ancestor sets instead, so the two share no algorithm.
 *
 * Model: a kinematic tree of n revolute or prismatic joints, one per link, parent[i] < i (-1 =
 * fixed base). Link i's frame is the joint frame: T_i = X_fixed[i] * Rot(axis[i], q_i) (revolute)
 * or X_fixed[i] * Trans(axis[i] q_i) (prismatic) relative to the parent link frame; motion subspace
 * S_i = [axis; 0] or [0; axis]. Task frame t = link task_link[t] * task_offset[t]. Spatial vectors
 * [angular; linear]. */
#include <math.h>
#include <string.h>

#include "wbq_oracle.h"

typedef struct {
    double R[9], p[3];
} se3;

static void rot_axis(const double *a, double q, double *R)
{
    const double c = cos(q), s = sin(q), v = 1.0 - c;
    const double x = a[0], y = a[1], z = a[2];
    R[0] = c + x * x * v;     R[1] = x * y * v - z * s; R[2] = x * z * v + y * s;
    R[3] = y * x * v + z * s; R[4] = c + y * y * v;     R[5] = y * z * v - x * s;
    R[6] = z * x * v - y * s; R[7] = z * y * v + x * s; R[8] = c + z * z * v;
}

static se3 compose(const se3 *A, const se3 *B) /* A * B */
{
    se3 C;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c)
            C.R[3 * r + c] = A->R[3 * r] * B->R[c] + A->R[3 * r + 1] * B->R[3 + c] + A->R[3 * r + 2] * B->R[6 + c];
        C.p[r] = A->R[3 * r] * B->p[0] + A->R[3 * r + 1] * B->p[1] + A->R[3 * r + 2] * B->p[2] + A->p[r];
    }
    return C;
}

static void cross3(const double *a, const double *b, double *c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

/* motion transform child <- parent for the child pose T (child in parent): [R^T, 0; -R^T [p]x, R^T] */
static void xform_motion(const se3 *T, const double *v, double *out)
{
    double w[3], l[3], px[3];
    for (int r = 0; r < 3; ++r) w[r] = T->R[r] * v[0] + T->R[3 + r] * v[1] + T->R[6 + r] * v[2];
    /* linear: R^T (v_l - p x w_parent) */
    cross3(T->p, v, px);
    for (int r = 0; r < 3; ++r) l[r] = T->R[r] * (v[3] - px[0]) + T->R[3 + r] * (v[4] - px[1]) + T->R[6 + r] * (v[5] - px[2]);
    memcpy(out, w, sizeof w);
    memcpy(out + 3, l, sizeof l);
}

/* force transform parent <- child (the transpose of xform_motion): [R n + p x R f; R f] */
static void xform_force_T(const se3 *T, const double *f, double *out)
{
    double n[3], ff[3], px[3];
    for (int r = 0; r < 3; ++r) {
        n[r] = T->R[3 * r] * f[0] + T->R[3 * r + 1] * f[1] + T->R[3 * r + 2] * f[2];
        ff[r] = T->R[3 * r] * f[3] + T->R[3 * r + 1] * f[4] + T->R[3 * r + 2] * f[5];
    }
    cross3(T->p, ff, px);
    for (int r = 0; r < 3; ++r) {
        out[r] = n[r] + px[r];
        out[3 + r] = ff[r];
    }
}

static void crm(const double *v, const double *m, double *out) /* v x m (motion) */
{
    double a[3], b[3], c[3];
    cross3(v, m, a);
    cross3(v, m + 3, b);
    cross3(v + 3, m, c);
    for (int r = 0; r < 3; ++r) {
        out[r] = a[r];
        out[3 + r] = b[r] + c[r];
    }
}

static void crf(const double *v, const double *f, double *out) /* v x* f (force) */
{
    double a[3], b[3], c[3];
    cross3(v, f, a);
    cross3(v + 3, f + 3, b);
    cross3(v, f + 3, c);
    for (int r = 0; r < 3; ++r) {
        out[r] = a[r] + b[r];
        out[3 + r] = c[r];
    }
}

/* spatial inertia of link i about its frame origin, link coordinates (6 x 6, row-major) */
static void link_inertia(const wbq_ref_rbd_model *m, int i, double *I)
{
    const double ms = m->mass[i], *c = m->com + 3 * i, *in = m->inertia + 6 * i;
    const double Ic[9] = {in[0], in[3], in[4], in[3], in[1], in[5], in[4], in[5], in[2]};
    const double cx[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
    memset(I, 0, 36 * sizeof(double));
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            double cc = 0.0; /* (cx cx^T)_rk */
            for (int t = 0; t < 3; ++t) cc += cx[3 * r + t] * cx[3 * k + t];
            I[6 * r + k] = Ic[3 * r + k] + ms * cc;
            I[6 * r + 3 + k] = ms * cx[3 * r + k];
            I[6 * (3 + r) + k] = ms * cx[3 * k + r];
            I[6 * (3 + r) + 3 + k] = r == k ? ms : 0.0;
        }
}

static void mat6_vec(const double *A, const double *v, double *out)
{
    for (int r = 0; r < 6; ++r) {
        double s = 0.0;
        for (int k = 0; k < 6; ++k) s += A[6 * r + k] * v[k];
        out[r] = s;
    }
}

static int prismatic(const wbq_ref_rbd_model *m, int i) { return m->jtype && m->jtype[i] == 1; }

/* motion subspace of joint i in its link frame */
static void subspace(const wbq_ref_rbd_model *m, int i, double *S)
{
    const double *a = m->axis + 3 * i;
    const int pr = prismatic(m, i);
    for (int r = 0; r < 3; ++r) {
        S[r] = pr ? 0.0 : a[r];
        S[3 + r] = pr ? a[r] : 0.0;
    }
}

static double dot6(const double *a, const double *b)
{
    double s = 0.0;
    for (int k = 0; k < 6; ++k) s += a[k] * b[k];
    return s;
}

static void local_transforms(const wbq_ref_rbd_model *m, const double *q, se3 *T)
{
    for (int i = 0; i < m->n; ++i) {
        se3 F, Jq;
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) F.R[3 * r + c] = m->X_fixed[12 * i + 4 * r + c];
            F.p[r] = m->X_fixed[12 * i + 4 * r + 3];
        }
        if (prismatic(m, i)) {
            for (int k = 0; k < 9; ++k) Jq.R[k] = (k % 4 == 0) ? 1.0 : 0.0;
            for (int r = 0; r < 3; ++r) Jq.p[r] = m->axis[3 * i + r] * q[i];
        } else {
            rot_axis(m->axis + 3 * i, q[i], Jq.R);
            Jq.p[0] = Jq.p[1] = Jq.p[2] = 0.0;
        }
        T[i] = compose(&F, &Jq);
    }
}

/* Inverse dynamics tau = M(q) qdd + h(q, qd) by RNEA in link coordinates. */
void wbq_ref_rnea(const wbq_ref_rbd_model *m, const double *q, const double *qd, const double *qdd, double *tau)
{
    const int n = m->n;
    se3 T[WBQ_REF_RBD_MAX];
    double v[WBQ_REF_RBD_MAX][6], a[WBQ_REF_RBD_MAX][6], f[WBQ_REF_RBD_MAX][6];
    local_transforms(m, q, T);
    const double a0[6] = {0, 0, 0, -m->gravity[0], -m->gravity[1], -m->gravity[2]};
    const double v0[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        const int p = m->parent[i];
        double S[6], t[6], c[6], I[36], Iv[6];
        subspace(m, i, S);
        xform_motion(&T[i], p < 0 ? v0 : v[p], v[i]);
        for (int k = 0; k < 6; ++k) v[i][k] += S[k] * qd[i];
        xform_motion(&T[i], p < 0 ? a0 : a[p], a[i]);
        for (int k = 0; k < 6; ++k) t[k] = S[k] * qd[i];
        crm(v[i], t, c);
        for (int k = 0; k < 6; ++k) a[i][k] += S[k] * qdd[i] + c[k];
        link_inertia(m, i, I);
        mat6_vec(I, a[i], f[i]);
        mat6_vec(I, v[i], Iv);
        crf(v[i], Iv, t);
        for (int k = 0; k < 6; ++k) f[i][k] += t[k];
    }
    for (int i = n - 1; i >= 0; --i) {
        double S[6];
        subspace(m, i, S);
        tau[i] = dot6(S, f[i]);
        const int p = m->parent[i];
        if (p >= 0) {
            double fp[6];
            xform_force_T(&T[i], f[i], fp);
            for (int k = 0; k < 6; ++k) f[p][k] += fp[k];
        }
    }
}

/* Joint-space inertia by CRBA in link coordinates (M row-major n x n). */
void wbq_ref_crba(const wbq_ref_rbd_model *m, const double *q, double *M)
{
    const int n = m->n;
    se3 T[WBQ_REF_RBD_MAX];
    static double Ic[WBQ_REF_RBD_MAX][36];
    local_transforms(m, q, T);
    for (int i = 0; i < n; ++i) link_inertia(m, i, Ic[i]);
    memset(M, 0, sizeof(double) * n * n);
    for (int i = n - 1; i >= 0; --i) {
        const int p = m->parent[i];
        if (p >= 0) { /* Ic_p += X^T Ic_i X, X = motion transform p -> i */
            double X[36], XtI[36];
            for (int c = 0; c < 6; ++c) {
                double e[6] = {0, 0, 0, 0, 0, 0}, col[6];
                e[c] = 1.0;
                xform_motion(&T[i], e, col);
                for (int r = 0; r < 6; ++r) X[6 * r + c] = col[r];
            }
            for (int r = 0; r < 6; ++r)
                for (int c = 0; c < 6; ++c) {
                    double s = 0.0;
                    for (int k = 0; k < 6; ++k) s += X[6 * k + r] * Ic[i][6 * k + c];
                    XtI[6 * r + c] = s;
                }
            for (int r = 0; r < 6; ++r)
                for (int c = 0; c < 6; ++c) {
                    double s = 0.0;
                    for (int k = 0; k < 6; ++k) s += XtI[6 * r + k] * X[6 * k + c];
                    Ic[p][6 * r + c] += s;
                }
        }
    }
    for (int i = 0; i < n; ++i) {
        double S[6], F[6];
        subspace(m, i, S);
        mat6_vec(Ic[i], S, F);
        M[i * n + i] = dot6(S, F);
        int j = i;
        while (m->parent[j] >= 0) {
            double Fp[6];
            xform_force_T(&T[j], F, Fp);
            memcpy(F, Fp, sizeof F);
            j = m->parent[j];
            double Sj[6];
            subspace(m, j, Sj);
            const double v = dot6(Sj, F);
            M[i * n + j] = v;
            M[j * n + i] = v;
        }
    }
}

static se3 task_offset(const wbq_ref_rbd_model *m, int t)
{
    se3 X;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) X.R[3 * r + c] = m->task_offset ? m->task_offset[12 * t + 4 * r + c] : (r == c);
        X.p[r] = m->task_offset ? m->task_offset[12 * t + 4 * r + 3] : 0.0;
    }
    return X;
}

/* World pose [R | p] row-major 3 x 4 and the geometric Jacobian (rows: linear velocity of the
 * frame origin, angular velocity; world frame) of the frame Xo attached to link e. */
static void frame_kinematics(const wbq_ref_rbd_model *m, const double *q, int e, const se3 *Xo, double *pose, double *J)
{
    const int n = m->n;
    se3 T[WBQ_REF_RBD_MAX], W[WBQ_REF_RBD_MAX];
    local_transforms(m, q, T);
    for (int i = 0; i < n; ++i) W[i] = m->parent[i] < 0 ? T[i] : compose(&W[m->parent[i]], &T[i]);
    const se3 We = compose(&W[e], Xo);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) pose[4 * r + c] = We.R[3 * r + c];
        pose[4 * r + 3] = We.p[r];
    }
    memset(J, 0, sizeof(double) * 6 * n);
    for (int j = e; j >= 0; j = m->parent[j]) {
        double a[3], d[3], lin[3];
        for (int r = 0; r < 3; ++r)
            a[r] = W[j].R[3 * r] * m->axis[3 * j] + W[j].R[3 * r + 1] * m->axis[3 * j + 1] + W[j].R[3 * r + 2] * m->axis[3 * j + 2];
        if (prismatic(m, j)) {
            for (int r = 0; r < 3; ++r) {
                J[r * n + j] = a[r];
                J[(3 + r) * n + j] = 0.0;
            }
            continue;
        }
        for (int r = 0; r < 3; ++r) d[r] = We.p[r] - W[j].p[r];
        cross3(a, d, lin);
        for (int r = 0; r < 3; ++r) {
            J[r * n + j] = lin[r];
            J[(3 + r) * n + j] = a[r];
        }
    }
}

void wbq_ref_link_kinematics(const wbq_ref_rbd_model *m, const double *q, int e, double *pose, double *J)
{
    const se3 I = {{1, 0, 0, 0, 1, 0, 0, 0, 1}, {0, 0, 0}};
    frame_kinematics(m, q, e, &I, pose, J);
}

/* Jdot qd of task frame t: the link-coordinate forward pass with qdd = 0 and no gravity gives the
 * task link's spatial velocity v = [w; v_O] and acceleration a = [dw; a_O] at its origin; the frame
 * origin p (link coordinates) then has classical acceleration a_O + dw x p + w x (v_O + w x p). */
void wbq_ref_task_jdqd(const wbq_ref_rbd_model *m, const double *q, const double *qd, int t, double *jdqd)
{
    const int n = m->n, e = m->task_link[t];
    se3 T[WBQ_REF_RBD_MAX], W[WBQ_REF_RBD_MAX];
    double v[WBQ_REF_RBD_MAX][6], a[WBQ_REF_RBD_MAX][6];
    local_transforms(m, q, T);
    for (int i = 0; i < n; ++i) W[i] = m->parent[i] < 0 ? T[i] : compose(&W[m->parent[i]], &T[i]);
    const double z6[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i <= e; ++i) {
        const int p = m->parent[i];
        double S[6], sq[6], c[6];
        subspace(m, i, S);
        xform_motion(&T[i], p < 0 ? z6 : v[p], v[i]);
        for (int k = 0; k < 6; ++k) v[i][k] += S[k] * qd[i];
        xform_motion(&T[i], p < 0 ? z6 : a[p], a[i]);
        for (int k = 0; k < 6; ++k) sq[k] = S[k] * qd[i];
        crm(v[i], sq, c);
        for (int k = 0; k < 6; ++k) a[i][k] += c[k];
    }
    const se3 Xo = task_offset(m, t);
    const double *w = v[e], *vo = v[e] + 3, *dw = a[e], *ao = a[e] + 3, *p = Xo.p;
    double t1[3], t2[3], vp[3], t3[3], lin[3];
    cross3(dw, p, t1);
    cross3(w, p, t2);
    for (int r = 0; r < 3; ++r) vp[r] = vo[r] + t2[r];
    cross3(w, vp, t3);
    for (int r = 0; r < 3; ++r) lin[r] = ao[r] + t1[r] + t3[r];
    for (int r = 0; r < 3; ++r) {
        jdqd[r] = W[e].R[3 * r] * lin[0] + W[e].R[3 * r + 1] * lin[1] + W[e].R[3 * r + 2] * lin[2];
        jdqd[3 + r] = W[e].R[3 * r] * dw[0] + W[e].R[3 * r + 1] * dw[1] + W[e].R[3 * r + 2] * dw[2];
    }
}

/* Everything the QPPVM solve consumes for one instance, in the wbq input layout. */
void wbq_ref_rbd_one(const wbq_ref_rbd_model *m, const double *q, const double *qd, double *M, double *h,
                     double *J, double *pose)
{
    double zero[WBQ_REF_RBD_MAX];
    memset(zero, 0, sizeof zero);
    wbq_ref_crba(m, q, M);
    wbq_ref_rnea(m, q, qd, zero, h);
    for (int t = 0; t < m->ntasks; ++t) {
        const se3 Xo = task_offset(m, t);
        frame_kinematics(m, q, m->task_link[t], &Xo, pose + 12 * t, J + (size_t)6 * m->n * t);
    }
}
