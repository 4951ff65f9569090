// Internal kernel interface of libwbq (not part of the public C ABI, see include/wbq.h).
#pragma once
#include <hip/hip_runtime.h>

namespace wbq {

constexpr int kWave = 64;
constexpr int kTMax = 4;    // Cartesian tasks on level 0
constexpr int kM0Max = 12;  // level-0 rows handled by the kernel

// Follow-up kernels (active set for n > 32, level-0 repair) run grid-stride over device work
// lists whose length the host never waits for. Their grid is sized from the counts the last
// follow-up kernel that ran on the context saw (written to mapped host memory, read by the host
// when it enqueues the next solve; stale by the solves in flight), with headroom and a decay, so
// a solve with nothing to repair launches a few blocks instead of up to 2,048: the repair kernel's
// scratch made that empty 2,048-block launch cost 5.2 us of a 38 us config-1 step (rocprofv3,
// profiles/r02_v15_kernel_stats.csv). The grid size never changes a result: every block loops
// over the list until it is drained.
struct FollowGrid {
    int *seen;    // [3] mapped host memory: counts of the two lists at the last follow-up launch; [2] set
                  // when an instance joins the repair list (the on-demand follow-up's completion check)
    int est[2];   // host estimate of this solve's counts (work items, not blocks)
};
constexpr unsigned kFollowMin = 16; // blocks: a count that grows from an estimate of 0 still has 16 waves
// Blocks for a list of about `est` instances, ipw instances per block, capped by `cap` and the batch.
inline unsigned follow_blocks(int est, int ipw, unsigned cap, int B)
{
    const long want = ((long)est * 5 / 4 + ipw - 1) / ipw + 1;
    long g = want < (long)kFollowMin ? (long)kFollowMin : want;
    if (g > (long)cap) g = cap;
    const long bmax = ((long)B + ipw - 1) / ipw;
    if (g > bmax) g = bmax;
    return (unsigned)(g < 1 ? 1 : g);
}
// Block 0 of the last follow-up kernel of a solve publishes the counts it saw.
__device__ __forceinline__ void follow_publish(const FollowGrid &fg, int c0, int c1)
{
    if (fg.seen && blockIdx.x == 0 && threadIdx.x == 0) {
        __hip_atomic_store(fg.seen, c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(fg.seen + 1, c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Everything one launch needs; passed by value as the kernel argument.
struct QppvmArgs {
    int B;           // instances
    int n;           // joints (<= NP of the instantiation)
    int ntasks;      // Cartesian tasks
    int m0;          // Cartesian rows (selected task rows of every task)
    int m_l0;        // of them level 0's (the first m_l0); the rest a middle level (wbq_desc task_level)
    int select_mode; // WBQ_SELECT_*
    int joint_weight; // WBQ_WEIGHT_*: W1 = I (qppvm_kernel.hip) or W1 = M (qppvm_w1m_kernel.hip)
    int minnorm;     // no joint task (wbq_desc no_joint_task): the last level's min-norm x, in the
                     // constraint-space kernel (qppvm_w1m_kernel.hip) with H = I
    int max_iter;    // active-set step cap
    int limits_crossed; // some tau_min > tau_max (batch-shared limits): every instance infeasible
    int row_mask[kTMax];
    const int *row_sel;      // [m0] task-row index t*6+r of level-0 row a (device)
    // the same by value: kernel-argument words are scalar loads (lgkmcnt), where a read through row_sel after
    // the stage's M loads is a vector load, and waiting for it waits for all of M (vmcnt retires in order)
    int row_selv[kM0Max];
    const double *Kc, *Dc;   // [ntasks*6] (device)
    const double *Kq, *Dq;   // [n]
    const double *tau_max, *tau_min; // [n]
    const double *M, *J, *pose, *pose_ref, *q, *qd, *qref, *h;  // batch inputs
    double *tau;     // [B][n]
    int *status;     // [B]
    int *iters;      // [B]
    unsigned long long *stamps; // diagnostic builds (-DWBQ_STAMPS): [grid][kStamps] s_memtime
    // fast kernel -> active-set kernel hand-off (device scratch sized for max_batch); the
    // fast kernel marks an instance that needs active-set steps with status -1, one whose
    // level-0 rows are inconsistent (level 0 needs the BVLS repair) with status -2
    double *u_scr;   // [B][NP]   u at the equality-constrained optimum
    double *q1_scr;  // [B][kM0Max][NP]  Q1 = G^T L^-T
    double *ui_scr;  // [B][NP]   u_imp = M^-1 tau_imp
    double *b0_scr;  // [B][kM0Max]  b0 = G w_t (level-0 targets)
    // per-solve work lists, double-buffered by solve parity: work[epoch*2 + 0] counts the
    // instances parked for the active-set kernel (listed in wl[0, B)), [+1] those for the
    // repair kernel (wl[B, 2B)). The follow-up kernels run small grid-stride grids over the
    // lists; the repair kernel (the last launch) clears the other parity's counters.
    int *work;       // [2][2] counters: instances appended to the two work lists this solve; [4 + epoch]: list 2
    int *wl;         // [3][B] work lists: [0, B) active-set kernel, [B, 2B) repair kernel, [2B, 3B) hand-back
    // NP = 64: the repair kernel hands an instance whose pinned level 1 needs the dual active set back to
    // an active-set pass over work list 2 (its pinned limits in lo_scr / hi_scr, u and Q1 in u_scr /
    // q1_scr, the BVLS bound set in ws_rows) instead of running the loop inside its own large frame
    double *lo_scr, *hi_scr; // [B][NP]
    int handback;
    // > 0 (NP = 64 active-set pass): a dual loop still running after that many steps is handed to the
    // level-0 repair (a loop that long mostly ends "level 0 infeasible" after all)
    int gi_handoff;
    int epoch;       // 0 / 1
    FollowGrid fg;   // follow-up grid sizing (see FollowGrid)
    // per-instance warm start across solves (the qpOASES hot-start analogue; it changes the
    // path, never the solution): hint bit 0 = the last solve needed the level-0 repair, so go there
    // directly; bit 1 (W1 = I) = ws_rows holds the last solve's final bound active set; state = BVLS
    // bound state (-1/0/+1 per joint) of that repair
    unsigned char *ws_hint; // [B]
    signed char *ws_state;  // [B][NP]
    // the side (+1 lower / -1 upper, 0 inactive) of every constraint row (W1 = M: dual_gi.h
    // warm_extend) or torque bound (W1 = I: gi_solve) in the last solve's final active set ([B][64])
    signed char *ws_rows;
    // JointLimits toggle (include/wbq.h): the box also holds Kjl (q_min - q) - Djl qd <= tau <=
    // Kjl (q_max - q) - Djl qd ([n] each, device)
    int joint_limits;
    const double *q_min, *q_max, *Kjl, *Djl;
    // MPC rollout step (wbq_rollout): after the final tau of an instance, qdd = M^-1 (tau - h)
    // and semi-implicit Euler on q, qd in place
    int integrate;
    double dt;
    // 1: the launcher raises the dynamic-LDS limit of every kernel variant this configuration can
    // launch (any batch size) and launches nothing. wbq_create does this once, so a solve takes no
    // lock and never allocates (include/wbq.h: wbq_solve is RT-safe)
    int prepare;
    // NP = 32: the level-0 repair runs at the end of the fast kernel (one launch per solve) instead
    // of in qppvm_repair_kernel
    int inline_repair;
    // > 0: the whole rollout of `steps` integrating solves in one launch (qppvm_rollout_kernel, NP =
    // 32, M0 <= 6): every wave carries its instances through all steps, so an instance that needs a
    // long level-0 repair in some step holds only its own wave, not every instance's next step
    int steps;
    // on-demand follow-up (WBQ_OPT_FOLLOWUP, NP = 32 merged path): skip_followup = the launcher does not
    // enqueue qppvm_repair_kernel after the fast kernel (the host completes a solve that listed repairs
    // when its outputs are read); self_book = the fast kernel then does the follow-up kernel's
    // bookkeeping itself (publishes the previous solve's counts, clears the next solve's counters)
    int skip_followup;
    int self_book;
};

// The box on x = tau - h of joint j (QPPVMPlugin.cpp:203-205: tau limits shifted by -h; with the
// JointLimits toggle also the joint-limit barrier at the joint's q, qd). lo > hi: the instance is
// infeasible (status 2).
__device__ __forceinline__ void torque_box(const QppvmArgs &a, int j, double q, double qd, double h, double &lo,
                                           double &hi)
{
    double l = a.tau_min[j], u = a.tau_max[j];
    if (a.joint_limits) {
        l = fmax(l, a.Kjl[j] * (a.q_min[j] - q) - a.Djl[j] * qd);
        u = fmin(u, a.Kjl[j] * (a.q_max[j] - q) - a.Djl[j] * qd);
    }
    lo = l - h;
    hi = u - h;
}

// fast 0-3,5,15 (+16,17 realtime); active-set 4,6,7 (+30,31); repair 8-12 (+28,29); BVLS split 20-27;
// dual-loop lap counters (gi_solve): inline 20-27 / 13-14, active kernel 32-39 / 40-41, repair 48-55 / 56-57
constexpr int kStamps = 64;

// Raise a kernel's dynamic-LDS limit on the current device to at least `bytes` (once per
// device and kernel; thread-safe: contexts on several devices or threads share it). Called only
// by the launchers' prepare pass (wbq_create*), never on the solve path.
hipError_t ensure_dynamic_lds(const void *kernel, size_t bytes);
// LDS bytes one workgroup may use on the current device (hipDeviceAttributeMaxSharedMemoryPerBlock or the
// opt-in limit, the larger; cached per device; 64 KB if the query fails)
size_t max_workgroup_lds();

// Launch the fused QPPVM solve (assemble -> 2-level hierarchical QP -> tau) for a batch.
// mid (optional): recorded on the stream right after the first (dominant) kernel.
hipError_t launch_qppvm(const QppvmArgs &a, hipStream_t stream, hipEvent_t mid = nullptr);
// The follow-up repair kernel alone for a solve launched with skip_followup (its epoch's list).
hipError_t launch_qppvm_followup(const QppvmArgs &a, hipStream_t stream);
// W1 = M (joint_weight 1): main kernel + level-0 repair kernel; needs m0 + n <= 64
hipError_t launch_qppvm_w1m(const QppvmArgs &a, hipStream_t stream, hipEvent_t mid = nullptr);

// ------------------------------------------------------------------ contact form (ForceAcc)
constexpr int kCMax = 4; // contacts

// One launch of the contact-form solve (reference
// src/ForceAcc.cpp:58-137,181-219). x = [qdd (n); w (wd per contact)].
struct ContactArgs {
    int B;           // instances
    int n;           // DoF incl. the 6 floating-base coordinates (first)
    int nc;          // contacts
    int torque_rows; // a12 extension: actuated torque-limit rows
    int max_iter;    // active-set step cap
    int limits_crossed;
    double Kp_w, Kd_w, Kp_f, Kd_f, Kp_p, Kd_p; // waist / feet / postural acceleration-task gains
    double eps_f;                              // min-norm tie-break on the contact variables
    int wd;                                    // wrench components per contact: 3 (forces) or 6
    int nfr;                                   // friction-pyramid rows (4 nc with mu > 0, else 0)
    double mu;                                 // friction coefficient of the pyramid rows
    double w_lb[6], w_ub[6];                   // box of an active contact's wd variables
    const double *tau_max, *tau_min;           // [n] (device)
    const double *M, *h, *q, *qd, *qref;       // [B][n][n], [B][n] x4
    const double *Jw, *jdqd_w, *pose_w, *pose_w_ref; // [B][6][n], [B][6], [B][12] x2
    const double *Jc, *jdqd_c, *pose_c, *pose_c_ref; // [B][nc][6][n], [B][nc][6], [B][nc][12] x2
    const int *cmask;                          // [B] bit c = contact c active
    double *tau;     // [B][n]
    double *x;       // [B][n + wd nc]
    int *status;     // [B]
    int *iters;      // [B]
    unsigned long long *stamps; // diagnostic builds (-DWBQ_STAMPS): [B][kStamps] s_memtime
    int integrate;   // MPC rollout step: qdd = x[0:n], semi-implicit Euler on q, qd in place
    double dt;
    // level-0 repair hand-off (as QppvmArgs): instances the main kernel finds level-0 infeasible at
    // b_w are listed in wl (count work[epoch*2 + 1]) for the repair kernel, which clears the other
    // parity's counters
    int *work;       // [2][2]
    int *wl;         // [B]
    int epoch;
    FollowGrid fg;   // repair grid sizing (est[1]; see FollowGrid)
    int prepare;     // as QppvmArgs::prepare
    // warm start: the side (+1 lower / -1 upper, 0 inactive) of every constraint row in the last
    // solve's final active set, per instance ([B][64]; dual_gi.h warm_extend)
    signed char *ws_rows;
    // set by the launcher for the repair kernel: its LDS holds the QR-form fallback (qr_gi.h)
    int qr_fallback;
};

// Semi-implicit Euler of one joint of instance b in place (lane i owns joint i of its
// instance): qd += dt qdd, q += dt qd. Failed solves (tau = h) have qdd = M^-1 (tau - h) = 0.
template <typename Args>
__device__ __forceinline__ void rollout_step(const Args &a, long b, int i, bool row, double qdd, bool ok)
{
    if (!a.integrate || !row) return;
    double *q = const_cast<double *>(a.q), *qd = const_cast<double *>(a.qd);
    const long k = b * a.n + i;
    const double v = qd[k] + a.dt * (ok ? qdd : 0.0);
    qd[k] = v;
    q[k] = q[k] + a.dt * v;
}

// mid (optional): recorded right after the main kernel, before the level-0 repair kernel
hipError_t launch_contact(const ContactArgs &a, hipStream_t stream, hipEvent_t mid = nullptr);

}  // namespace wbq

struct wbq_rbd_ctx; // rbd.hip

namespace wbq {

// Batched rigid-body quantities (rbd.hip): one launch over B instances, outputs in the wbq input
// layouts (any may be null).
hipError_t rbd_launch(const wbq_rbd_ctx *c, int B, const double *q, const double *qd, double *M, double *h, double *J,
                      double *pose, hipStream_t stream);
// tasks [0, split) into (J, pose, jdqd), tasks [split, ntasks) into (J2, pose2, jdqd2) (the contact
// form's waist and contact arrays)
hipError_t rbd_launch_split(const wbq_rbd_ctx *c, int B, const double *q, const double *qd, double *M, double *h,
                            int split, double *J, double *pose, double *jdqd, double *J2, double *pose2, double *jdqd2,
                            hipStream_t stream);
int rbd_n(const wbq_rbd_ctx *c);
int rbd_ntasks(const wbq_rbd_ctx *c);
int rbd_device(const wbq_rbd_ctx *c);

// Lanes per instance used for a given n (32 for n <= 32, else 64).
inline int lanes_per_instance(int n) { return n <= 32 ? 32 : 64; }

}  // namespace wbq
