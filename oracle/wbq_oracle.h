/*
 * wbq_oracle.h -- CPU restatement (TEST INFRASTRUCTURE ONLY) of the per-tick
 * torque solve that ADVRHumanoids/qppvm's QPPVMPlugin delegates to
 * OpenSoT + qpOASES.
 *
 * This is the *checker*: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product path (qppvm_amd, libwbq.so) never
 * links or calls it.
 *
 * Parity status: the reference cannot be built or run anywhere in this
 * pipeline (OpenSoT, qpOASES, XBotInterface, XCM, Eigen are absent; SURVEY.md
 * 8c), and the reference holds no tests or golden data. The oracle is
 * therefore pinned to closed-form known-answer tests and to an independent
 * numpy/scipy restatement (tests/golden/make_golden.py), NOT to reference
 * outputs: "parity unpinned" against the reference binaries.
 *
 * The formulation deliberately follows the reference's *task* form (x-space,
 * A = J M^-1 formed explicitly, H = A^T W A, qpOASES-style primal active set)
 * so that it is an independent computation path from the GPU kernels, which
 * work in the transformed u = M^-1 x space with a dual active-set method.
 *
 * Reference anchors (files under /root/reference):
 *   src/QPPVMPlugin.cpp:56-67    effort limits, tau_min = -tau_max, bounds shifted by -h
 *   src/QPPVMPlugin.cpp:99-118   joint impedance task K=5, D=2, useInertiaMatrix(true)
 *   src/QPPVMPlugin.cpp:129-152  two Cartesian impedance tasks Kc=700, Dc=70, rows {0,1,2}
 *   src/QPPVMPlugin.cpp:177-179  stack ((ee_right + ee_left) / joint_task) << torque_limits
 *   src/QPPVMPlugin.cpp:188      QPOases_sot(stack, bounds, eps_regularisation = 1.0)
 *   src/QPPVMPlugin.cpp:203-205  bounds re-shifted each tick
 *   src/QPPVMPlugin.cpp:246-256  solve; on failure tau_qp = 0; tau = tau_qp + h
 */
#ifndef WBQ_ORACLE_H
#define WBQ_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WBQ_REF_MAX_TASKS 4

/* select_mode: how OpenSoT::Indices::range(0,2) (QPPVMPlugin.cpp:134,147) restricts
 * a 6-D Cartesian impedance task.  [upstream semantics unverifiable offline]
 *   0 = SUBTASK: the full 6-D task (A6, b6) is built, then rows are selected
 *       (OpenSoT SubTask semantics).
 *   1 = TASK:    the task-space force F is masked before J^T F. */
#define WBQ_REF_SELECT_SUBTASK 0
#define WBQ_REF_SELECT_TASK 1

/* joint_weight: weight of the joint impedance task on level 1 (W1). */
#define WBQ_REF_WEIGHT_IDENTITY 0
#define WBQ_REF_WEIGHT_INERTIA 1

/* statuses (shared with the product ABI, include/wbq.h) */
#define WBQ_REF_OK 0
#define WBQ_REF_MAXITER 1
#define WBQ_REF_INFEASIBLE 2
#define WBQ_REF_NUMERICAL 3

typedef struct {
    int n;                           /* joint DoF */
    int ntasks;                      /* Cartesian tasks summed on level 0 */
    int row_mask[WBQ_REF_MAX_TASKS]; /* bit r keeps row r of task t (reference: 0x7) */
    int select_mode;                 /* WBQ_REF_SELECT_* */
    int joint_weight;                /* WBQ_REF_WEIGHT_* */
    const double *Kc;                /* [ntasks][6] diagonal Cartesian stiffness */
    const double *Dc;                /* [ntasks][6] diagonal Cartesian damping */
    const double *Kq;                /* [n] joint stiffness */
    const double *Dq;                /* [n] joint damping */
    const double *tau_max;           /* [n] */
    const double *tau_min;           /* [n] */
    /* JointLimits toggle (QPPVMPlugin.cpp:169-171; include/wbq.h): the box on tau also holds
     * Kjl (q_min - q) - Djl qd <= tau <= Kjl (q_max - q) - Djl qd */
    int joint_limits;
    const double *q_min, *q_max, *Kjl, *Djl; /* [n] */
    /* priority level of each Cartesian task (include/wbq.h task_level): 0 the first level (the
     * tasks there summed), 1 a second Cartesian level -- the elbow tasks of QPPVMPlugin.cpp:154-166.
     * All zero: the reference stack. */
    int task_level[WBQ_REF_MAX_TASKS];
    /* 1: no joint task (include/wbq.h no_joint_task): the stack ends at the last Cartesian level, the
     * reference's commented elbow stack ((ee_r + ee_l) / (elbow_l + elbow_r)) << limits
     * (QPPVMPlugin.cpp:177-178 in place of :179); the last level's x is the minimum-norm point among
     * its optima (H1 = I, g1 = 0: the eps -> 0 limit of QPOases_sot's regularisation, :188). */
    int no_joint_task;
} wbq_ref_desc;

/* One instance (all row-major fp64):
 *   M [n][n] SPD inertia, J [ntasks][6][n] geometric Jacobians (linear rows 0-2,
 *   angular 3-5), pose / pose_ref [ntasks][12] = [R | p] as 3x4 row-major,
 *   q, qd, qref, h [n]. */
typedef struct {
    const double *M, *J, *pose, *pose_ref, *q, *qd, *qref, *h;
} wbq_ref_instance;

/* Cartesian error e = [p_ref - p ; vec(quat(R_ref R^T)) with w >= 0]. */
void wbq_ref_cart_error(const double pose[12], const double pose_ref[12], double e[6]);

/* Builds the two levels exactly as the OpenSoT tasks would (x = tau - h):
 *   A0 [m0][n], b0 [m0]   level 0: stacked Cartesian tasks  A = S J M^-1, b = S J M^-1 J^T F
 *   H1 [n][n], g1 [n]     level 1: joint task A1 = M^-1, b1 = M^-1 tau_imp, H1 = A1^T W A1, g1 = -A1^T W b1
 *   lb, ub [n]            torque limits shifted by -h
 * Returns m0 (>0) or -WBQ_REF_NUMERICAL when M is not SPD. */
int wbq_ref_assemble(const wbq_ref_desc *d, const wbq_ref_instance *in, double *A0, double *b0,
                     double *H1, double *g1, double *lb, double *ub);

/* Level 0: bounded least squares min 0.5||A x - b||^2, lb <= x <= ub (Stark-Parker BVLS with
 * minimum-norm free-set solves). state[n] in/out: 0 free, -1 at lb, +1 at ub (warm start).
 * Returns a WBQ_REF_* status. */
int wbq_ref_level0(int m, int n, const double *A, const double *b, const double *lb,
                   const double *ub, double *x, int *state, int *iters);

/* Rows of the stacked Cartesian tasks per level: returns the total m (level-0 rows first, then the
 * middle level's, as wbq_ref_assemble orders them) and sets *m_l0 to the level-0 count. */
int wbq_ref_task_rows(const wbq_ref_desc *d, int *m_l0);

/* Middle level: min 0.5||A x - b||^2 s.t. E x = e (level-0 optimality, me rows), lb <= x <= ub,
 * from a feasible x with bound state[n] (the level-0 solution): Stark-Parker BVLS whose free-set
 * solves stay in the null space of E's free columns (minimum-norm, SVD); multipliers of the bound
 * variables w = A^T (b - A x) - E^T nu. Returns a WBQ_REF_* status; w_out [n] (optional) the
 * final w (pins). */
int wbq_ref_level_mid(int me, const double *E, int m, int n, const double *A, const double *b, const double *lb,
                      const double *ub, double *x, int *state, double *w_out, int *iters);

/* Level 1: strictly convex QP min 0.5 x^T H x + g^T x s.t. Aeq x = beq, lb <= x <= ub,
 * primal active set (qpOASES family) started from a feasible x with bound state[n]. */
int wbq_ref_level1(int n, const double *H, const double *g, int me, const double *Aeq,
                   const double *beq, const double *lb, const double *ub, double *x, int *state,
                   int *iters);

/* Whole per-tick chain for one instance: tau = x* + h (x* = 0 on failure, QPPVMPlugin.cpp:246-256).
 * y0 (optional, [m0]) receives A0 x0*. Returns a WBQ_REF_* status. */
int wbq_ref_qppvm_one(const wbq_ref_desc *d, const wbq_ref_instance *in, double *tau, double *y0,
                      int *iters);

/* Batched driver over contiguous instance arrays (strides implied by n, ntasks). */
void wbq_ref_qppvm_batch(const wbq_ref_desc *d, int B, const double *M, const double *J,
                         const double *pose, const double *pose_ref, const double *q,
                         const double *qd, const double *qref, const double *h, double *tau,
                         int32_t *status, int32_t *iters);

/* ---------------------------------------------------------------- contact form (ForceAcc)
 * SURVEY.md 8a rows a10-a12; spec in wbq_oracle_contact.c. x = [qdd (n); f (3 per contact)]. */
#define WBQ_REF_MAX_CONTACTS 4
typedef struct {
    int n;              /* DoF including the n_fb floating-base coordinates (first) */
    int n_fb;           /* 6 */
    int nc;             /* contacts, <= WBQ_REF_MAX_CONTACTS */
    double Kp_w, Kd_w;  /* waist acceleration task gains */
    double Kp_f, Kd_f;  /* feet acceleration task gains */
    double Kp_p, Kd_p;  /* postural task gains */
    double f_lb[3], f_ub[3]; /* force box of an active contact (ForceAcc.cpp:74-76) */
    double eps_f;       /* min-norm tie-break weight on the forces */
    int torque_rows;    /* a12 extension: actuated torque-limit rows */
    const double *tau_max, *tau_min; /* [n] (rows n_fb.. used when torque_rows) */
    /* SURVEY 8f-2 extensions (zero-initialised = the reference's point forces, no cone) */
    int wrench_dim;     /* 3 (0 = 3): w_c = [f_c; 0]; 6: full wrench [f_c; m_c] ("put 6 for full
                         * wrench", ForceAcc.cpp:67), box [f_lb, m_lb] <= w_c <= [f_ub, m_ub] (:74-76) */
    double m_lb[3], m_ub[3]; /* moment box of a 6-D wrench (reference -1 / 1) */
    double mu;          /* > 0: linearised friction pyramid |f_x| <= mu f_z, |f_y| <= mu f_z (world
                         * frame, 4 rows per active contact); 0: none (the reference) */
} wbq_ref_contact_desc;

/* One instance: M [n][n], h, q, qd, qref [n]; waist Jw [6][n], jdqd_w [6] (Jdot qd),
 * pose_w / pose_w_ref [12]; contacts Jc [nc][6][n], jdqd_c [nc][6], pose_c / pose_c_ref
 * [nc][12]; contact_mask bit c = contact c active (inactive: f_c = 0). */
typedef struct {
    const double *M, *h, *q, *qd, *qref;
    const double *Jw, *jdqd_w, *pose_w, *pose_w_ref;
    const double *Jc, *jdqd_c, *pose_c, *pose_c_ref;
    int contact_mask;
} wbq_ref_contact_instance;

/* wrench components per contact (3 or 6) */
int wbq_ref_contact_wd(const wbq_ref_contact_desc *d);

/* Dense Goldfarb-Idnani dual active set, KKT re-solved by LU each step:
 *   min 0.5 x^T H x + g^T x  s.t.  E x = e (me rows),  clo <= C x <= chi (mi rows),  H SPD. */
int wbq_ref_dual_qp(int n, const double *H, const double *g, int me, const double *E, const double *e,
                    int mi, const double *C, const double *clo, const double *chi, double *x, int *iters);

/* Level-1 data of the contact form (nx = n + wd nc, wd = wrench_dim): H1, g1, E [12][nx] (waist
 * rows with rhs b_w, then dynamic feasibility), C [mi][nx] with clo/chi (mi = wd nc box rows, then
 * 4 nc friction rows when mu > 0, then n - n_fb torque rows); bw [6] the waist target. Returns mi. */
int wbq_ref_contact_assemble(const wbq_ref_contact_desc *d, const wbq_ref_contact_instance *in, double *H1,
                             double *g1, double *E, double *e, double *C, double *clo, double *chi, double *bw);

/* Whole chain for one instance: tau = M qdd + h - sum_c J_c^T [f_c; 0] (tau = h on failure),
 * x = [qdd; f]. l0_repaired = 1 when level 0 is not attainable at b_w (y0* != b_w). */
int wbq_ref_contact_one(const wbq_ref_contact_desc *d, const wbq_ref_contact_instance *in, double *tau,
                        double *x, int *iters, int *l0_repaired);

void wbq_ref_contact_batch(const wbq_ref_contact_desc *d, int B, const double *M, const double *h, const double *q,
                           const double *qd, const double *qref, const double *Jw, const double *jdqd_w,
                           const double *pose_w, const double *pose_w_ref, const double *Jc, const double *jdqd_c,
                           const double *pose_c, const double *pose_c_ref, const int32_t *cmask, double *tau,
                           double *x, int32_t *status, int32_t *iters, int32_t *l0_repaired);

/* ---- rigid-body dynamics (oracle/wbq_oracle_rbd.c): kinematic tree of revolute or prismatic
 * joints, one per link, parent[i] < i (-1 = fixed base); link frame = joint frame,
 * T_i = X_fixed[i] Rot(axis[i], q_i) (revolute) or X_fixed[i] Trans(axis[i] q_i) (prismatic) in the
 * parent link frame; a floating base is six such joints (3 prismatic + 3 revolute, massless
 * intermediate links). Task frame t = link task_link[t] times task_offset[t]. Same fields as
 * wbq_rbd_desc (include/wbq.h). */
#define WBQ_REF_RBD_MAX 64
typedef struct {
    int n;
    const int *parent;      /* [n] */
    const double *X_fixed;  /* [n][12] [R | p] row-major */
    const double *axis;     /* [n][3] unit, joint frame */
    const double *mass;     /* [n] */
    const double *com;      /* [n][3] link frame */
    const double *inertia;  /* [n][6] Ixx Iyy Izz Ixy Ixz Iyz about the COM, link frame */
    double gravity[3];
    int ntasks;
    const int *task_link;   /* [ntasks] */
    const int *jtype;       /* [n] 0 revolute, 1 prismatic; NULL = all revolute */
    const double *task_offset; /* [ntasks][12] [R | p] in the task link's frame; NULL = identity */
} wbq_ref_rbd_model;

void wbq_ref_rnea(const wbq_ref_rbd_model *m, const double *q, const double *qd, const double *qdd, double *tau);
void wbq_ref_crba(const wbq_ref_rbd_model *m, const double *q, double *M);
void wbq_ref_link_kinematics(const wbq_ref_rbd_model *m, const double *q, int e, double *pose, double *J);
/* Jdot qd of task frame t (the classical acceleration of its origin and the angular acceleration
 * at qdd = 0, no gravity; rows [linear; angular], world frame): XBotInterface computeJdotQdot. */
void wbq_ref_task_jdqd(const wbq_ref_rbd_model *m, const double *q, const double *qd, int t, double *jdqd);
void wbq_ref_rbd_one(const wbq_ref_rbd_model *m, const double *q, const double *qd, double *M, double *h,
                     double *J, double *pose);

#ifdef __cplusplus
}
#endif
#endif
