/*
 * wbq.h -- C ABI of the MI355X batched whole-body-QP engine (libwbq.so).
 *
 * Drop-in boundary for the per-tick torque solve of ADVRHumanoids/qppvm's XBot RT
 * plugins. The plugins keep their XBot surface; what they delegated to OpenSoT
 * (task assembly, AutoStack, QPOases_sot) and qpOASES is replaced by these calls,
 * batched over B robot instances / MPC rollouts. Entry points and the reference
 * interface each one replaces:
 *
 *   wbq_create        <- QPPVMPlugin::init_control_plugin's task/stack/solver wiring
 *                        (src/QPPVMPlugin.cpp:99-189: TorqueLimits :112,
 *                        JointImpedanceCtrl :114-118, CartesianImpedanceCtrl :129-152,
 *                        AutoStack :177-179, QPOases_sot(.., 1.0) :188).
 *                        All device memory is allocated here (the reference sizes its
 *                        Eigen buffers at init, :56-62), so wbq_solve never allocates.
 *   wbq_set_inputs    <- the per-tick model pulls inside autostack->update(q)
 *                        (:226; J, M, poses, qdot) plus h (:312), q_ref (:279) and the
 *                        torque-limit shift (:203-205).
 *   wbq_solve         <- solver->solve(tau_d) (:246) + tau_d = tau_qp + h (:256), for
 *                        the whole batch, asynchronously on the context's HIP stream.
 *   wbq_get_outputs   <- the tau_d handed to model->setJointEffort (:318) and the
 *                        bool of solve() (:246) as a per-instance status.
 *   wbq_reset_warmstart <- qpOASES hot-start state reset (QPOases_sot re-init) [upstream].
 *   wbq_destroy       <- plugin close()/destructor (:339-342).
 *   wbq_rollout       <- no reference counterpart: the MPC config, N
 *                        solves with the state integrated on the device between them.
 *
 * Contact form (ForceAcc plugin, src/ForceAcc.cpp):
 *   wbq_create_contact      <- ForceAccExample::init_control_plugin's wiring (:31-141: OptvarHelper
 *                              x = [qddot; f_c] :58-72, wrench bounds :74-95, feet tasks :83-89,
 *                              postural :105-107, DynamicFeasibility :109-114, waist :118-122,
 *                              AutoStack :131-133, QPOases_sot(.., 1e4) :135-137).
 *   wbq_set_contact_inputs  <- sync_model + autostack->update (:172-184; M, h, Jacobians, poses).
 *   wbq_solve               <- solver->solve(x) (:188-189) + the ID post-step
 *                              tau = M qdd + h - sum_c J_c^T [f_c; 0] (:196-219).
 *   wbq_get_contact_outputs <- the unpacked x = [qdd; f_c] (:196-201).
 *   wbq_get_outputs         <- tau handed to setJointEffort (:219) + per-instance status; on
 *                              status != 0 the reference skips the send (:189-193), here tau = h.
 *
 * Conventions: fp64, row-major, instance-major contiguous arrays:
 *   M [B][n][n] SPD joint-space inertia        J [B][ntasks][6][n] (rows 0-2 linear, 3-5 angular)
 *   pose, pose_ref [B][ntasks][12] = [R | p] 3x4 row-major (Eigen::Affine3d::matrix() top rows)
 *   q, qd, qref, h [B][n]                       tau [B][n] out, status/iters [B] out
 * Per-instance status: 0 ok, 1 iteration cap, 2 infeasible, 3 numerical. On status != 0
 * tau = h (the reference's "SOLVER ERROR!" fallback tau_qp = 0, QPPVMPlugin.cpp:246-249).
 * A context is not thread-safe: one context per caller thread, one HIP stream per context.
 */
#ifndef WBQ_H
#define WBQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* API return codes */
#define WBQ_SUCCESS 0
#define WBQ_E_INVALID (-1)
#define WBQ_E_DEVICE (-2)
#define WBQ_E_UNSUPPORTED (-3)
#define WBQ_E_CAPACITY (-4)

/* per-instance statuses */
#define WBQ_STATUS_OK 0
#define WBQ_STATUS_MAXITER 1
#define WBQ_STATUS_INFEASIBLE 2
#define WBQ_STATUS_NUMERICAL 3

/* problem forms */
#define WBQ_FORM_QPPVM 0   /* QPPVMPlugin: 2-level torque-space impedance QP */
#define WBQ_FORM_CONTACT 1 /* ForceAccExample: 2-level acceleration + contact-force QP */

/* Cartesian row selection semantics of OpenSoT::Indices::range(0,2) (QPPVMPlugin.cpp:134) */
#define WBQ_SELECT_SUBTASK 0 /* full 6-D task built, rows selected afterwards */
#define WBQ_SELECT_TASK 1    /* task-space force masked before J^T F */

/* joint-task weight W1 on level 1 (JointImpedanceCtrl, QPPVMPlugin.cpp:114-118):
 * IDENTITY  min ||M^-1 (x - tau_imp)||^2      (KAT-1)
 * INERTIA   min (x - tau_imp)^T M^-1 (x - tau_imp), the dynamically consistent form (KAT-2);
 *           needs m0 + n <= 64 (one lane per level-0 row and torque limit), else
 *           wbq_create returns WBQ_E_UNSUPPORTED */
#define WBQ_WEIGHT_IDENTITY 0
#define WBQ_WEIGHT_INERTIA 1

/* memory kinds for wbq_inputs.memory */
#define WBQ_MEM_HOST 0   /* copied (async H2D) into context-owned device buffers */
#define WBQ_MEM_DEVICE 1 /* device pointers adopted as-is (caller keeps them alive) */

typedef struct wbq_ctx wbq_ctx;

typedef struct {
    int form;          /* WBQ_FORM_* */
    int n;             /* joint DoF, 1..64 */
    int ntasks;        /* Cartesian tasks summed on level 0, 1..4 (reference: 2) */
    int row_mask[4];   /* per task, bit r keeps task row r (reference: 0x7) */
    int select_mode;   /* WBQ_SELECT_* */
    int joint_weight;  /* WBQ_WEIGHT_* */
    int max_batch;     /* capacity; every buffer is sized for it in wbq_create */
    int max_iter;      /* active-set step cap per instance, 0 = default (4 n + 32) */
    const double *Kc;  /* [ntasks][6] Cartesian stiffness diagonal (reference 700) */
    const double *Dc;  /* [ntasks][6] Cartesian damping diagonal (reference 70) */
    const double *Kq;  /* [n] joint stiffness (reference 5) */
    const double *Dq;  /* [n] joint damping (reference 2) */
    const double *tau_max; /* [n] effort limits */
    const double *tau_min; /* [n] (reference: -tau_max, QPPVMPlugin.cpp:58) */
    /* JointLimits toggle (OpenSoT torque::JointLimits, built at QPPVMPlugin.cpp:169-171 with gains
     * k0*10, d0*20; commented out of the reference stack). 1: every instance's box also holds the
     * joint-limit barrier  Kjl (q_min - q) - Djl qd <= tau <= Kjl (q_max - q) - Djl qd  (the
     * build's written spec of the [upstream] task; an instance whose box empties is infeasible,
     * status 2). 0: torque limits only (the reference stack). */
    int joint_limits;
    const double *q_min, *q_max; /* [n] joint position limits (ModelInterface::getJointLimits) */
    const double *Kjl, *Djl;     /* [n] barrier stiffness / damping */
    /* Priority level of each Cartesian task: 0 the first level (its tasks summed), 1 a second
     * Cartesian level -- the elbow tasks the reference builds on arm1_4 / arm2_4 (QPPVMPlugin.cpp:154-166
     * _elbow_task_left/right). Level 1 is lexicographic: min ||A1 x - b1||^2 keeping level 0 at its
     * optimum y0*. At most 6 rows per level (else wbq_create returns WBQ_E_UNSUPPORTED). All zero (a
     * zero-initialised tail): the reference stack. With no_joint_task = 1 and task_level {0, 0, 1, 1}
     * this is the reference's commented elbow stack (below); with no_joint_task = 0 the joint task
     * follows as a third level, ((ee_r + ee_l) / (elbow_l + elbow_r)) / joint << limits: an extension
     * the reference never spells. Every Cartesian task takes the hands' form A = J M^-1, b = A J^T F
     * (useInertiaMatrix(true), :139,:151); the reference does not call useInertiaMatrix on the elbow
     * tasks, and OpenSoT's default form for them is [upstream]: parity unpinned on that point. */
    int task_level[4];
    /* 1: no joint task -- the stack ends at the last Cartesian level, as in the reference's commented
     * elbow line, which closes the stack at :178 in place of :179:
     *   ((ee_r + ee_l) / (elbow_l + elbow_r)) << torque_limits          (QPPVMPlugin.cpp:177-178)
     * The last level leaves x non-unique (6 rows over n torques); QPOases_sot(.., 1.0) (:188) decides it
     * by qpOASES' Hessian regularisation eps I, whose eps -> 0 limit is taken here: x = the minimum-norm
     * point among the lexicographic optima, min ||x||^2 s.t. A0 x = y0*, A1 x = y1*, the box. Solved in
     * constraint space like W1 = M (joint_weight is ignored); needs m0 + n <= 64. wbq_rollout is
     * refused (WBQ_E_UNSUPPORTED): its qdd = M^-1 x step is not carried by this path. 0: the joint
     * task is the last level (the reference's live stack, :179). */
    int no_joint_task;
} wbq_desc;

typedef struct {
    int batch;  /* B <= max_batch */
    int memory; /* WBQ_MEM_* */
    const double *M, *J, *pose, *pose_ref, *q, *qd, *qref, *h;
} wbq_inputs;

/* Contact form: x = [qdd (n); w_c (wrench_dim per contact)] (ForceAcc.cpp:58-72); level 0 = waist
 * acceleration task, level 1 = postural + feet acceleration tasks + eps_f ||f||^2 (the explicit
 * minimum-norm tie-break of the internal forces); both levels: dynamic feasibility on the 6
 * floating-base rows, force box for active contacts (f = 0 for inactive ones), optional
 * actuated torque rows tau_min <= M_a qdd + h_a - J_c,a^T f <= tau_max. */
typedef struct {
    int n;            /* DoF incl. the floating base (first n_fb coordinates); n + wd nc <= 64 and the
                       * constraint rows (6 or n) + 6 + wd nc (+ 4 nc with mu) <= 64 */
    int n_fb;         /* must be 6 */
    int nc;           /* contacts, 1..4 */
    int torque_rows;  /* 0/1 */
    int max_batch;
    int max_iter;     /* 0 = default 10 (nx + m) + 50 */
    double Kp_w, Kd_w, Kp_f, Kd_f, Kp_p, Kd_p; /* waist / feet / postural task gains */
    double f_lb[3], f_ub[3];                   /* force box (reference: -1000,-1000,10 / 1000) */
    double eps_f;                              /* > 0 */
    const double *tau_max, *tau_min;           /* [n] (used with torque_rows) */
    /* SURVEY.md 8f-2 options; a zero-initialised tail is the reference's stack */
    int wrench_dim;            /* 3 (0 = 3): w_c = [f_c; 0]; 6: x carries the full wrench w_c = [f_c; m_c]
                                * ("put 6 for full wrench", ForceAcc.cpp:67), boxed by [f_lb, m_lb] ..
                                * [f_ub, m_ub] (:74-76), J_c^T w_c over all six Jacobian rows */
    double m_lb[3], m_ub[3];   /* moment box of a 6-D wrench (reference -1 / 1) */
    double mu;                 /* > 0: linearised friction pyramid |f_x| <= mu f_z, |f_y| <= mu f_z per
                                * active contact (world frame, 4 rows); 0: none (the reference) */
} wbq_contact_desc;

/* Contact-form batch, fp64 row-major, instance-major:
 *   M [B][n][n], h, q, qd, qref [B][n], Jw [B][6][n], jdqd_w [B][6], pose_w, pose_w_ref [B][12],
 *   Jc [B][nc][6][n], jdqd_c [B][nc][6], pose_c, pose_c_ref [B][nc][12], cmask [B] (bit c = active). */
typedef struct {
    int batch;
    int memory;
    const double *M, *h, *q, *qd, *qref, *Jw, *jdqd_w, *pose_w, *pose_w_ref;
    const double *Jc, *jdqd_c, *pose_c, *pose_c_ref;
    const int32_t *cmask;
} wbq_contact_inputs;

int wbq_create(const wbq_desc *desc, int device, wbq_ctx **out);
int wbq_create_contact(const wbq_contact_desc *desc, int device, wbq_ctx **out);
/* Launch on a caller-provided hipStream_t (NULL = the context's own stream, created non-blocking;
 * WBQ_NULL_STREAM = the device's legacy default stream, hipStream_t 0 -- e.g. torch's default stream,
 * whose handle is 0 and so cannot be passed as itself). Solves of one context must stay stream-ordered:
 * switch streams only between a completed solve and the next (a pending host-input copy made on the old
 * stream is waited for). */
#define WBQ_NULL_STREAM ((void *)1)
int wbq_set_stream(wbq_ctx *ctx, void *hip_stream);
/* WBQ_MEM_HOST inputs are copied into the context (pinned staging, one H2D copy on the stream);
 * WBQ_MEM_DEVICE inputs are adopted in place: the caller keeps them alive and unchanged until the
 * solves that read them have completed in stream order (with WBQ_MEM_DEVICE inputs every solve
 * enqueues all of its kernels, so a refill enqueued on the stream after wbq_solve is safe). */
int wbq_set_inputs(wbq_ctx *ctx, const wbq_inputs *in);
int wbq_set_contact_inputs(wbq_ctx *ctx, const wbq_contact_inputs *in);
int wbq_solve(wbq_ctx *ctx);
/* MPC-style rollout: `steps` sequential solves of the current batch,
 * each followed on the device by qdd = M^-1 (tau - h) (the contact form: x[0:n]) and
 * semi-implicit Euler qd += dt qdd, q += dt qd on the batch's q and qd in place (J, M, h and
 * poses frozen; mirrors the integration ForceAcc.cpp:225-226 leaves commented out). The
 * per-instance warm-start state carries from step to step. Host-staged inputs advance in the
 * context's copy, WBQ_MEM_DEVICE inputs in the caller's buffers. Outputs afterwards are the
 * last step's. */
int wbq_rollout(wbq_ctx *ctx, int steps, double dt);
/* Synchronous copy of the batch's current q, qd ([batch][n], either may be NULL). */
int wbq_get_state(wbq_ctx *ctx, double *q, double *qd);
/* Overwrite the batch's q, qd ([batch][n], either may be NULL; WBQ_MEM_*), stream-ordered: the
 * start state of the next rollout (an MPC re-plans each horizon from the measured state). */
int wbq_set_state(wbq_ctx *ctx, const double *q, const double *qd, int memory);
int wbq_sync(wbq_ctx *ctx);
/* Synchronous copy of the last solve's outputs to host memory (any pointer may be NULL). */
int wbq_get_outputs(wbq_ctx *ctx, double *tau, int32_t *status, int32_t *iters);
/* Contact form: synchronous copy of the last solve's x = [qdd; w] ([batch][n + wrench_dim nc]). */
int wbq_get_contact_outputs(wbq_ctx *ctx, double *x);
/* Write outputs into caller-owned device buffers ([batch][n] / [batch]) instead of the
 * context's (any NULL pointer reverts that output to the context buffer). */
int wbq_set_outputs(wbq_ctx *ctx, double *tau, int32_t *status, int32_t *iters);
/* Device-resident outputs of the last solve: final when this call returns (a solve left pending by the
 * on-demand follow-up, WBQ_OPT_FOLLOWUP, is completed first) and valid until the next wbq_solve /
 * wbq_rollout / wbq_destroy. */
int wbq_get_device_outputs(wbq_ctx *ctx, const double **tau, const int32_t **status,
                           const int32_t **iters);
/* Drop the warm-start working set of instances with mask[b] != 0, b < the current batch (the
 * mask has one entry per instance of the last wbq_set_inputs batch); NULL = every instance up
 * to max_batch. Stream-ordered with the solves. */
int wbq_reset_warmstart(wbq_ctx *ctx, const uint8_t *mask);
/* Read the per-instance warm-start hints of the current batch (1 = the last solve of that
 * instance went through the level-0 repair with level 0 infeasible at b0; all 0 in a form
 * without hints): diagnostics, e.g. the repair share of MPC rollout steps. Synchronous. */
int wbq_get_warmstart_hints(wbq_ctx *ctx, uint8_t *hints);
/* Kernel timing with HIP events on the launch stream: enable = N > 0 times every N-th solve
 * (events are stream packets: sampling keeps them from pacing the stream), 0 disables; then
 * read the summed device time (ms) and the number of timed solves since the last read. */
int wbq_set_timing(wbq_ctx *ctx, int enable);
int wbq_get_timing(wbq_ctx *ctx, double *total_ms, int *launches);
/* Same, split: summed device time of whole solves and of their dominant (first) kernel. */
int wbq_get_timing_detail(wbq_ctx *ctx, double *solve_ms, double *kernel_ms, int *launches);
/* Per-context execution options (path choices that never change a result; the tests run both ways):
 *   WBQ_OPT_INLINE_REPAIR   QPPVM W1 = I, n <= 32: -1 (default) the level-0 repair runs inside the
 *                           fast kernel for 64 solves after a solve that needed it, else in its own
 *                           follow-up kernel; 0 always the follow-up kernel; 1 always inline
 *   WBQ_OPT_FUSED_ROLLOUT   1 (default) wbq_rollout of a QPPVM W1 = I context with n <= 32 runs all
 *                           steps in one launch; 0 one launch per step
 * The environment variables WBQ_INLREP / WBQ_FUSED_ROLLOUT, when set, give the initial values of a
 * new context. */
#define WBQ_OPT_INLINE_REPAIR 1
#define WBQ_OPT_FUSED_ROLLOUT 2
/*   WBQ_OPT_FOLLOWUP        QPPVM W1 = I, n <= 32: 1 (default) while the last solves needed no level-0 repair, a
 *                           solve enqueues its fast kernel alone; if that solve does list a repair, it is
 *                           completed (its repair kernel run, then synchronised) by the next call that reads
 *                           outputs: wbq_sync, wbq_get_outputs, wbq_get_device_outputs, wbq_get_state,
 *                           wbq_get_warmstart_hints (a later wbq_solve supersedes it). Not applied with
 *                           caller-owned device outputs (wbq_set_outputs: a stream consumer reads them
 *                           without a call), WBQ_MEM_DEVICE inputs (the deferred repair would read the
 *                           caller's buffers when the outputs are read, after the caller may have refilled
 *                           them), rollouts or the constraint-space stacks. 0: every solve enqueues its
 *                           follow-up kernel, so its outputs are final in stream order. (env WBQ_FOLLOWUP)
 *   WBQ_OPT_HANDBACK        QPPVM W1 = I, n > 32: 1 (default) a repaired instance's pinned level-1 dual loop runs
 *                           in a third launch (the active-set kernel over work list 2); 0 inside the repair
 *                           kernel. (env WBQ_HANDBACK)
 *   WBQ_OPT_GI_HANDOFF      QPPVM W1 = I, n > 32: a dual loop of the active-set kernel still running after this
 *                           many steps (>= 0; default 24, 0 = never) is handed to the level-0 repair, which
 *                           settles level 0 first (same result). Takes effect with WBQ_OPT_HANDBACK = 1.
 *                           (env WBQ_GI_HANDOFF) */
#define WBQ_OPT_FOLLOWUP 3
#define WBQ_OPT_HANDBACK 4
#define WBQ_OPT_GI_HANDOFF 5
int wbq_set_option(wbq_ctx *ctx, int option, int value);
void wbq_destroy(wbq_ctx *ctx);
const char *wbq_last_error(const wbq_ctx *ctx);
const char *wbq_version(void);

/* ---------------------------------------------------------------- rigid-body dynamics
 * Batched model quantities the hot path consumes, from (q, qd) on the device. They replace the
 * XBotInterface ModelInterface calls of the reference (RBDL backend [upstream]):
 *   getInertiaMatrix      -> M       (used by every task, QPPVMPlugin.cpp:114-118,139,151)
 *   computeNonlinearTerm  -> h       (QPPVMPlugin.cpp:65,312; ForceAcc.cpp:208-217 via ID)
 *   getPose / getJacobian -> pose, J (QPPVMPlugin.cpp:272-284 and the Cartesian tasks :129-152)
 * Model: a kinematic tree of n <= 64 revolute or prismatic joints, one per link, parent[i] < i
 * (-1 = fixed base); link i's frame is its joint frame, T_i = X_fixed[i] * Rot(axis[i], q_i)
 * (revolute) or X_fixed[i] * Trans(axis[i] q_i) (prismatic) in the parent link frame. A floating
 * base is six virtual joints (3 prismatic + 3 revolute, massless links between; the ForceAcc
 * contact form's n_fb = 6 first coordinates). Task frame t is link task_link[t] times the fixed
 * task_offset[t] (a frame behind a fixed URDF joint, e.g. a foot sole). Outputs use the wbq_inputs
 * layouts (M [B][n][n], h [B][n], J [B][T][6][n] with rows [linear; angular] of the task frame's
 * origin in the world frame, pose [B][T][12] = [R | p], Jdot qd [B][T][6]), so they feed
 * wbq_set_inputs directly (WBQ_MEM_DEVICE) or wbq_rollout_rbd. */
typedef struct wbq_rbd_desc {
    int n;
    const int32_t *parent;  /* [n] */
    const double *X_fixed;  /* [n][12] [R | p] row-major, joint frame in the parent link frame at q = 0 */
    const double *axis;     /* [n][3] unit joint axis, joint frame */
    const double *mass;     /* [n] */
    const double *com;      /* [n][3] link frame */
    const double *inertia;  /* [n][6] Ixx, Iyy, Izz, Ixy, Ixz, Iyz about the COM, link frame */
    double gravity[3];      /* world, e.g. {0, 0, -9.81} */
    int ntasks;             /* <= 5: the Cartesian task frames (QPPVM: the two arms; contact form:
                             * the waist, then the contact frames) */
    const int32_t *task_link;
    int max_batch;
    const int32_t *jtype;       /* [n] 0 revolute, 1 prismatic; NULL = all revolute */
    const double *task_offset;  /* [ntasks][12] [R | p] in the task link's frame; NULL = identity */
} wbq_rbd_desc;

typedef struct wbq_rbd_ctx wbq_rbd_ctx;

int wbq_rbd_create(const wbq_rbd_desc *desc, int device, wbq_rbd_ctx **out);
/* One launch over `batch` instances on the context's stream (asynchronous; all pointers of the
 * same memory kind: WBQ_MEM_DEVICE pointers are used in place, WBQ_MEM_HOST ones are staged and
 * the call waits for the outputs). Any output may be NULL. */
int wbq_rbd_compute(wbq_rbd_ctx *ctx, int batch, const double *q, const double *qd, double *M, double *h,
                    double *J, double *pose, int memory);
/* Same plus Jdot qd [B][T][6] of every task frame (the classical acceleration of its origin and the
 * angular acceleration at qdd = 0, no gravity: XBotInterface computeJdotQdot, ForceAcc.cpp:184 via
 * the acceleration tasks). */
int wbq_rbd_compute_ex(wbq_rbd_ctx *ctx, int batch, const double *q, const double *qd, double *M, double *h,
                       double *J, double *pose, double *jdqd, int memory);
/* (NULL = the model context's own stream, WBQ_NULL_STREAM = the null stream, as wbq_set_stream) */
int wbq_rbd_set_stream(wbq_rbd_ctx *ctx, void *hip_stream);
void wbq_rbd_destroy(wbq_rbd_ctx *ctx);
/* MPC rollouts with the model re-evaluated every step: per step, M, h, J and
 * poses of the context's inputs are recomputed from its integrated q, qd, then one solve
 * integrates them (wbq_rollout). The context must hold device-resident inputs of its own
 * (set with WBQ_MEM_HOST, or WBQ_MEM_DEVICE buffers the caller lets it overwrite); both contexts on
 * one device. QPPVM form: the model's n and ntasks equal the context's. Contact form: the model's
 * tasks are the waist (task 0) and the nc contact frames (tasks 1..nc), which fill Jw, jdqd_w,
 * pose_w and Jc, jdqd_c, pose_c; n equal (the first 6 joints the floating base). */
int wbq_rollout_rbd(wbq_ctx *ctx, wbq_rbd_ctx *rbd, int steps, double dt);

#ifdef __cplusplus
}
#endif
#endif
