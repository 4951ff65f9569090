// wbq_api.hip -- C ABI of libwbq (declared in include/wbq.h).
//
// The context owns every device buffer (allocated once in wbq_create, the analogue of
// QPPVMPlugin::init_control_plugin sizing its Eigen buffers, src/QPPVMPlugin.cpp:56-62),
// so wbq_solve is allocation-free and can be captured in a hipGraph.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/wbq.h"
#include "wbq_kernels.h"

static int env_option(const char *name, int dflt)
{
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

struct wbq_ctx {
    int device = 0;
    int form = WBQ_FORM_QPPVM;
    wbq_desc d{};              // QPPVM form (d.n, d.max_batch, d.max_iter are set for both forms)
    wbq_contact_desc cd{};     // contact form
    int nfield = 0;            // fp64 input fields and their elements per instance
    size_t fe[16] = {};
    int m0 = 0;
    int m_l0 = 0; // level-0 rows (m0 but with a middle level, task_level)
    int limits_crossed = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // batch-shared parameters (device)
    double *Kc = nullptr, *Dc = nullptr, *Kq = nullptr, *Dq = nullptr, *tmax = nullptr, *tmin = nullptr;
    int *row_sel = nullptr;
    int row_sel_host[wbq::kM0Max] = {}; // the same, passed by value in the kernel argument
    // owned inputs: one device block + one pinned host staging block, fields packed back to
    // back for the current batch, so a host-side set_inputs is a single H2D copy
    double *dev_in = nullptr, *host_in = nullptr;
    hipEvent_t in_copied = nullptr;
    hipStream_t in_stream = nullptr; // stream the last host-input copy was issued on
    bool in_pending = false;
    const double *in[16] = {};
    const int *cmask = nullptr; // contact form: [B] (packed after the fp64 fields when staged)
    double *dev_x = nullptr;     // contact form: x [max_batch][nx]
    int nx = 0;
    int batch = 0;
    bool have_inputs = false;
    bool inputs_device = false; // the current inputs are the caller's WBQ_MEM_DEVICE buffers
    // outputs: one device block [tau | status | iters] packed for the current batch (single
    // D2H copy into the pinned host block), and optional caller-owned device buffers
    double *dev_out = nullptr, *host_out = nullptr;
    double *tau = nullptr;
    int *status = nullptr;
    int *iters = nullptr;
    double *out_tau = nullptr;
    int *out_status = nullptr;
    int *out_iters = nullptr;
    // event timing
    bool timing = false;
    int timing_every = 1;       // time every timing_every-th solve
    unsigned long long solves = 0;
    std::vector<hipEvent_t> ev;  // triples (start, end of the dominant kernel, end)
    std::vector<int> ev_mid;     // per triple: index of the event ending the dominant kernel
    int ev_used = 0;
    double t_acc_ms = 0.0;
    double t_kern_ms = 0.0;
    int t_launches = 0;
    std::string err;
    unsigned long long *stamps = nullptr; // diagnostic builds only
    double *u_scr = nullptr, *q1_scr = nullptr; // fast -> active-set hand-off
    double *ui_scr = nullptr, *b0_scr = nullptr; // u_imp and b0 for the level-0 repair
    double *lo_scr = nullptr, *hi_scr = nullptr; // n > 32: repair -> active-set hand-back (pinned limits)
    int *work = nullptr; // [2][2] per-solve work counters (see wbq_kernels.h)
    int *wl = nullptr;   // [2][max_batch] work lists
    unsigned char *ws_hint = nullptr; // [B] warm start (see wbq_kernels.h)
    signed char *ws_state = nullptr;  // [B][NP]
    signed char *ws_rows = nullptr;   // [B][64] final active set per instance (contact, W1 = M)
    double *jl = nullptr;             // [4][n] joint-limit box: q_min, q_max, Kjl, Djl (JointLimits toggle)
    size_t np = 0;
    int epoch = 0;
    int inl_hold = 0; // solves left in the inline-repair variant since a solve last needed a repair
    // per-context options (wbq_set_option); the environment gives a new context's initial values
    int opt_inline = env_option("WBQ_INLREP", -1); // WBQ_OPT_INLINE_REPAIR
    int opt_fused = env_option("WBQ_FUSED_ROLLOUT", 1); // WBQ_OPT_FUSED_ROLLOUT
    int opt_followup = env_option("WBQ_FOLLOWUP", 1);  // WBQ_OPT_FOLLOWUP
    int opt_handback = env_option("WBQ_HANDBACK", 1);  // n > 32: repaired instances' dual loop in the active pass
    // n > 32: active-set steps before the repair takes over (stress plant p99 1.17 -> 1.06 ms at 16-32 steps,
    // profiles/r05_v6_dummy_stress_handoff.log; 0: never)
    int opt_handoff = env_option("WBQ_GI_HANDOFF", 24);
    // on-demand follow-up: the last solve skipped its repair kernel; completed when outputs are read
    bool pending = false;
    wbq::QppvmArgs pend_args{};
    // follow-up grid sizing (wbq_kernels.h FollowGrid): counts the last follow-up kernel saw, in
    // mapped pinned host memory (device view work_seen_dev), and the host's running estimate
    int *work_seen = nullptr, *work_seen_dev = nullptr;
    int fest[2] = {0, 0};
};

namespace wbq {

hipError_t ensure_dynamic_lds(const void *kernel, size_t bytes)
{
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, size_t> done; // (device, kernel) -> limit set
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    size_t &cur = done[{dev, kernel}];
    if (bytes <= cur) return hipSuccess;
    e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) cur = bytes;
    return e;
}

size_t max_workgroup_lds()
{
    static std::mutex mu;
    static std::map<int, size_t> seen; // device -> bytes
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 64 * 1024;
    std::lock_guard<std::mutex> lock(mu);
    auto it = seen.find(dev);
    if (it != seen.end()) return it->second;
    // (the opt-in limit is what hipFuncSetAttribute can raise a kernel to; the larger of the two)
    int v = 0, o = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) v = 0;
    if (hipDeviceGetAttribute(&o, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess) o = 0;
    const int m = v > o ? v : o;
    const size_t bytes = m > 0 ? (size_t)m : 64 * 1024;
    seen[dev] = bytes;
    return bytes;
}

}  // namespace wbq

namespace {

const char *kVersion = "wbq 0.2.0 (gfx950, fp64, QPPVM + contact forms)";

size_t field_elems(const wbq_desc &d, int f)
{
    const size_t n = (size_t)d.n, T = (size_t)d.ntasks;
    switch (f) {
    case 0: return n * n;      // M
    case 1: return T * 6 * n;  // J
    case 2: return T * 12;     // pose
    case 3: return T * 12;     // pose_ref
    default: return n;         // q, qd, qref, h
    }
}

// contact form fields: M, h, q, qd, qref, Jw, jdqd_w, pose_w, pose_w_ref, Jc, jdqd_c, pose_c, pose_c_ref
constexpr int kContactFields = 13;
size_t contact_field_elems(const wbq_contact_desc &d, int f)
{
    const size_t n = (size_t)d.n, nc = (size_t)d.nc;
    switch (f) {
    case 0: return n * n;
    case 1: case 2: case 3: case 4: return n;
    case 5: return 6 * n;
    case 6: return 6;
    case 7: case 8: return 12;
    case 9: return nc * 6 * n;
    case 10: return nc * 6;
    default: return nc * 12; // 11, 12
    }
}

int fail(wbq_ctx *c, int code, const std::string &msg)
{
    if (c) c->err = msg;
    return code;
}

int hip_fail(wbq_ctx *c, hipError_t e, const char *what)
{
    return fail(c, WBQ_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// Create-time warm-up: one solve of a benign single instance (M = I, waist / task rows e_r,
// resting poses) so that the first wbq_solve of a real-time loop does not pay the lazy load of
// the code object and the first-launch setup (config 0 measured a 10-15 ms first tick without
// it). The reference's QPOases_sot also solves once at construction (initProblem). The
// warm-start state is reset afterwards; the context is left without inputs.
int prime_qppvm(wbq_ctx *c);
int prime_contact(wbq_ctx *c);

// Follow-up grid estimate for the next solve: the counts of the last follow-up launch that has
// run (relaxed reads of the mapped host block), and at least half the previous estimate.
wbq::FollowGrid follow_grid(wbq_ctx *c)
{
    wbq::FollowGrid fg{};
    fg.seen = c->work_seen_dev;
    for (int k = 0; k < 2; ++k) {
        const int s = c->work_seen ? __atomic_load_n(c->work_seen + k, __ATOMIC_RELAXED) : 0;
        const int d = c->fest[k] / 2;
        c->fest[k] = s > d ? s : d;
        fg.est[k] = c->fest[k];
    }
    return fg;
}

bool alloc_work_seen(wbq_ctx *c)
{
    if (hipHostMalloc((void **)&c->work_seen, 3 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return false;
    c->work_seen[0] = c->work_seen[1] = c->work_seen[2] = 0;
    return hipHostGetDevicePointer((void **)&c->work_seen_dev, c->work_seen, 0) == hipSuccess;
}

#define WBQ_HIP(call)                                   \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return hip_fail(c, e_, #call); \
    } while (0)

int solve_contact(wbq_ctx *c, int integrate, double dt, bool prepare, const wbq_rbd_ctx *rbd = nullptr)
{
    const wbq_contact_desc &d = c->cd;
    wbq::ContactArgs a{};
    a.B = c->batch;
    a.n = d.n;
    a.nc = d.nc;
    a.torque_rows = d.torque_rows;
    a.max_iter = d.max_iter;
    a.limits_crossed = c->limits_crossed;
    a.Kp_w = d.Kp_w;
    a.Kd_w = d.Kd_w;
    a.Kp_f = d.Kp_f;
    a.Kd_f = d.Kd_f;
    a.Kp_p = d.Kp_p;
    a.Kd_p = d.Kd_p;
    a.eps_f = d.eps_f;
    a.wd = d.wrench_dim == 6 ? 6 : 3;
    a.mu = d.mu;
    a.nfr = d.mu > 0.0 ? 4 * d.nc : 0;
    for (int k = 0; k < 3; ++k) {
        a.w_lb[k] = d.f_lb[k];
        a.w_ub[k] = d.f_ub[k];
        a.w_lb[3 + k] = d.m_lb[k];
        a.w_ub[3 + k] = d.m_ub[k];
    }
    a.tau_max = c->tmax;
    a.tau_min = c->tmin;
    a.M = c->in[0];
    a.h = c->in[1];
    a.q = c->in[2];
    a.qd = c->in[3];
    a.qref = c->in[4];
    a.Jw = c->in[5];
    a.jdqd_w = c->in[6];
    a.pose_w = c->in[7];
    a.pose_w_ref = c->in[8];
    a.Jc = c->in[9];
    a.jdqd_c = c->in[10];
    a.pose_c = c->in[11];
    a.pose_c_ref = c->in[12];
    a.cmask = c->cmask;
    a.tau = c->out_tau ? c->out_tau : c->tau;
    a.status = c->out_status ? c->out_status : c->status;
    a.iters = c->out_iters ? c->out_iters : c->iters;
    a.x = c->dev_x;
    a.stamps = c->stamps;
    a.integrate = integrate;
    a.dt = dt;
    a.work = c->work;
    a.wl = c->wl;
    a.epoch = c->epoch;
    a.prepare = prepare ? 1 : 0;
    a.ws_rows = c->ws_rows;
    a.fg = follow_grid(c);
    WBQ_HIP(hipSetDevice(c->device));
    if (prepare) {
        WBQ_HIP(wbq::launch_contact(a, c->stream, nullptr));
        return WBQ_SUCCESS;
    }
    const bool timed = c->timing && a.B > 0 && c->ev_used + 3 <= (int)c->ev.size() &&
                       (c->solves++ % (unsigned long long)c->timing_every) == 0;
    if (timed) WBQ_HIP(hipEventRecord(c->ev[c->ev_used], c->stream));
    if (rbd) // the model at the integrated state: M, h, the waist (task 0) and contact frames (tasks 1..nc)
        WBQ_HIP(wbq::rbd_launch_split(rbd, c->batch, c->in[2], c->in[3], const_cast<double *>(c->in[0]),
                                      const_cast<double *>(c->in[1]), 1, const_cast<double *>(c->in[5]),
                                      const_cast<double *>(c->in[7]), const_cast<double *>(c->in[6]),
                                      const_cast<double *>(c->in[9]), const_cast<double *>(c->in[11]),
                                      const_cast<double *>(c->in[10]), c->stream));
    WBQ_HIP(wbq::launch_contact(a, c->stream, timed ? c->ev[c->ev_used + 1] : nullptr));
    if (a.B > 0) c->epoch ^= 1; // solves on one context are stream-ordered
    if (timed) {
        WBQ_HIP(hipEventRecord(c->ev[c->ev_used + 2], c->stream));
        c->ev_mid[c->ev_used / 3] = 1;
        c->ev_used += 3;
    }
    return WBQ_SUCCESS;
}

}  // namespace

extern "C" {

const char *wbq_version(void) { return kVersion; }

static int complete_pending(wbq_ctx *c); // (an on-demand solve is finished before its state changes)

const char *wbq_last_error(const wbq_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int wbq_create(const wbq_desc *desc, int device, wbq_ctx **out)
{
    if (!out || !desc) return WBQ_E_INVALID;
    *out = nullptr;
    const wbq_desc &d = *desc;
    if (d.form != WBQ_FORM_QPPVM) return WBQ_E_UNSUPPORTED;
    if (d.n < 1 || d.n > 64 || d.ntasks < 1 || d.ntasks > wbq::kTMax || d.max_batch < 1)
        return WBQ_E_INVALID;
    if (d.select_mode != WBQ_SELECT_SUBTASK && d.select_mode != WBQ_SELECT_TASK) return WBQ_E_INVALID;
    if (d.joint_weight != WBQ_WEIGHT_IDENTITY && d.joint_weight != WBQ_WEIGHT_INERTIA) return WBQ_E_INVALID;
    if (!d.Kc || !d.Dc || !d.Kq || !d.Dq || !d.tau_max || !d.tau_min) return WBQ_E_INVALID;
    if (d.joint_limits && (!d.q_min || !d.q_max || !d.Kjl || !d.Djl)) return WBQ_E_INVALID;
    int m0 = 0, m_l0 = 0;
    int sel[wbq::kM0Max];
    bool mid = false;
    for (int t = 0; t < d.ntasks; ++t) {
        if (d.task_level[t] != 0 && d.task_level[t] != 1) return WBQ_E_INVALID;
        mid |= d.task_level[t] == 1;
    }
    // the task rows, level 0's first, then the middle level's (task_level)
    for (int tt = 0; tt < 2 * d.ntasks; ++tt) {
        const int t = tt % d.ntasks;
        if ((d.task_level[t] != 0) != (tt >= d.ntasks)) continue;
        if (d.row_mask[t] <= 0 || d.row_mask[t] >= 64) return WBQ_E_INVALID;
        for (int r = 0; r < 6; ++r)
            if ((d.row_mask[t] >> r) & 1) {
                if (m0 == wbq::kM0Max) return WBQ_E_UNSUPPORTED;
                if (tt < d.ntasks) ++m_l0;
                sel[m0++] = t * 6 + r;
            }
    }
    if (d.no_joint_task != 0 && d.no_joint_task != 1) return WBQ_E_INVALID;
    // W1 = M and the stack without a joint task run the active set in constraint space, one lane per
    // Cartesian row and torque limit
    const bool cspace = d.joint_weight == WBQ_WEIGHT_INERTIA || d.no_joint_task;
    if (cspace && m0 + d.n > 64) return WBQ_E_UNSUPPORTED;
    // a second Cartesian level: at least one task on level 0, at most 6 rows per level (the
    // repair's 6-row bvls_eq blocks)
    if (mid && (m_l0 == 0 || m_l0 > 6 || m0 - m_l0 > 6)) return WBQ_E_UNSUPPORTED;
    wbq_ctx *c = new wbq_ctx();
    c->d = d;
    c->d.Kc = c->d.Dc = c->d.Kq = c->d.Dq = c->d.tau_max = c->d.tau_min = nullptr;
    c->d.q_min = c->d.q_max = c->d.Kjl = c->d.Djl = nullptr;
    c->d.joint_limits = d.joint_limits ? 1 : 0;
    if (c->d.max_iter <= 0) c->d.max_iter = 4 * d.n + 32;
    c->m0 = m0;
    c->m_l0 = m_l0;
    c->device = device;
    for (int j = 0; j < d.n; ++j)
        if (d.tau_min[j] > d.tau_max[j]) c->limits_crossed = 1;
    auto cleanup = [&](int rc) {
        wbq_destroy(c);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) return cleanup(WBQ_E_DEVICE);
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) return cleanup(WBQ_E_DEVICE);
    c->stream = c->own_stream;
    const size_t n = (size_t)d.n, T6 = (size_t)d.ntasks * 6, B = (size_t)d.max_batch;
    bool ok = hipMalloc(&c->Kc, T6 * 8) == hipSuccess && hipMalloc(&c->Dc, T6 * 8) == hipSuccess &&
              hipMalloc(&c->Kq, n * 8) == hipSuccess && hipMalloc(&c->Dq, n * 8) == hipSuccess &&
              hipMalloc(&c->tmax, n * 8) == hipSuccess && hipMalloc(&c->tmin, n * 8) == hipSuccess &&
              hipMalloc(&c->row_sel, sizeof(int) * wbq::kM0Max) == hipSuccess;
    if (ok && d.joint_limits) // [q_min | q_max | Kjl | Djl]
        ok = hipMalloc(&c->jl, 4 * n * 8) == hipSuccess && hipMemcpy(c->jl, d.q_min, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(c->jl + n, d.q_max, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(c->jl + 2 * n, d.Kjl, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(c->jl + 3 * n, d.Djl, n * 8, hipMemcpyHostToDevice) == hipSuccess;
    c->nfield = 8;
    for (int f = 0; f < 8; ++f) c->fe[f] = field_elems(d, f);
    size_t in_elems = 0;
    for (int f = 0; f < 8; ++f) in_elems += c->fe[f] * B;
    const size_t out_bytes = n * B * 8 + 2 * B * 4 + 16;
    ok = ok && hipMalloc(&c->dev_in, in_elems * 8) == hipSuccess &&
         hipHostMalloc((void **)&c->host_in, in_elems * 8, hipHostMallocDefault) == hipSuccess &&
         hipMalloc(&c->dev_out, out_bytes) == hipSuccess &&
         hipHostMalloc((void **)&c->host_out, out_bytes, hipHostMallocDefault) == hipSuccess &&
         hipEventCreateWithFlags(&c->in_copied, hipEventDisableTiming) == hipSuccess;
    if (!ok) return cleanup(WBQ_E_DEVICE);
    ok = hipMemcpy(c->Kc, d.Kc, T6 * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->Dc, d.Dc, T6 * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->Kq, d.Kq, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->Dq, d.Dq, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->tmax, d.tau_max, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->tmin, d.tau_min, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->row_sel, sel, sizeof(int) * m0, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) return cleanup(WBQ_E_DEVICE);
    for (int r = 0; r < m0; ++r) c->row_sel_host[r] = sel[r];
    {
        // scratch lanes per instance (the W1 = M repair runs one instance per wave)
        const size_t np = cspace ? 64 : (size_t)wbq::lanes_per_instance(d.n);
        ok = hipMalloc(&c->u_scr, B * np * 8) == hipSuccess &&
             hipMalloc(&c->q1_scr, B * wbq::kM0Max * np * 8) == hipSuccess &&
             hipMalloc(&c->ui_scr, B * np * 8) == hipSuccess &&
             hipMalloc(&c->b0_scr, B * wbq::kM0Max * 8) == hipSuccess &&
             hipMalloc(&c->work, 6 * sizeof(int)) == hipSuccess && hipMemset(c->work, 0, 6 * sizeof(int)) == hipSuccess &&
             alloc_work_seen(c) && hipMalloc(&c->wl, 3 * B * sizeof(int)) == hipSuccess &&
             hipMalloc(&c->ws_hint, B) == hipSuccess && hipMemset(c->ws_hint, 0, B) == hipSuccess &&
             hipMalloc(&c->ws_state, B * np) == hipSuccess && hipMemset(c->ws_state, 0, B * np) == hipSuccess;
        if (ok && np == 64 && !cspace) // (the hand-back of repaired instances, one per wave)
            ok = hipMalloc(&c->lo_scr, B * np * 8) == hipSuccess && hipMalloc(&c->hi_scr, B * np * 8) == hipSuccess;
        if (ok) // the active sets' warm start (W1 = M: dual_gi.h; W1 = I: qppvm_kernel.hip gi_solve)
            ok = hipMalloc(&c->ws_rows, B * 64) == hipSuccess && hipMemset(c->ws_rows, 0, B * 64) == hipSuccess;
        c->np = np;
        if (!ok) return cleanup(WBQ_E_DEVICE);
    }
#ifdef WBQ_STAMPS
    if (hipMalloc(&c->stamps, sizeof(unsigned long long) * wbq::kStamps * B) != hipSuccess)
        return cleanup(WBQ_E_DEVICE);
#endif
    if (prime_qppvm(c) != WBQ_SUCCESS) return cleanup(WBQ_E_DEVICE);
    *out = c;
    return WBQ_SUCCESS;
}

int wbq_create_contact(const wbq_contact_desc *desc, int device, wbq_ctx **out)
{
    if (!out || !desc) return WBQ_E_INVALID;
    *out = nullptr;
    const wbq_contact_desc &d = *desc;
    if (d.n_fb != 6 || d.n <= 6 || d.nc < 1 || d.nc > wbq::kCMax || d.max_batch < 1) return WBQ_E_INVALID;
    if (d.wrench_dim != 0 && d.wrench_dim != 3 && d.wrench_dim != 6) return WBQ_E_INVALID;
    if (!(d.mu >= 0.0)) return WBQ_E_INVALID;
    const int wd = d.wrench_dim == 6 ? 6 : 3, nfr = d.mu > 0.0 ? 4 * d.nc : 0;
    // one lane per primal variable and per constraint row
    if (d.n + wd * d.nc > 64 || (d.torque_rows ? d.n : 6) + 6 + wd * d.nc + nfr > 64) return WBQ_E_UNSUPPORTED;
    if (!(d.eps_f > 0.0)) return WBQ_E_INVALID;
    if (d.torque_rows && (!d.tau_max || !d.tau_min)) return WBQ_E_INVALID;
    for (int k = 0; k < 3; ++k)
        if (!(d.f_lb[k] <= d.f_ub[k]) || (wd == 6 && !(d.m_lb[k] <= d.m_ub[k]))) return WBQ_E_INVALID;
    wbq_ctx *c = new wbq_ctx();
    c->form = WBQ_FORM_CONTACT;
    c->cd = d;
    c->cd.tau_max = c->cd.tau_min = nullptr;
    c->nx = d.n + wd * d.nc;
    const int me = (d.torque_rows ? d.n : 6) + 6 + wd * d.nc + nfr;
    if (c->cd.max_iter <= 0) c->cd.max_iter = 10 * (c->nx + me) + 50;
    c->d.n = d.n;
    c->d.max_batch = d.max_batch;
    c->d.max_iter = c->cd.max_iter;
    c->device = device;
    if (d.torque_rows)
        for (int j = d.n_fb; j < d.n; ++j)
            if (d.tau_min[j] > d.tau_max[j]) c->limits_crossed = 1;
    auto cleanup = [&](int rc) {
        wbq_destroy(c);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) return cleanup(WBQ_E_DEVICE);
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) return cleanup(WBQ_E_DEVICE);
    c->stream = c->own_stream;
    const size_t n = (size_t)d.n, B = (size_t)d.max_batch;
    c->nfield = kContactFields;
    size_t in_elems = 0;
    for (int f = 0; f < kContactFields; ++f) {
        c->fe[f] = contact_field_elems(d, f);
        in_elems += c->fe[f] * B;
    }
    const size_t cm_elems = (B + 1) / 2; // the int32 contact masks, packed after the fp64 fields
    const size_t out_bytes = n * B * 8 + 2 * B * 4 + 16;
    std::vector<double> tmx(n, 0.0), tmn(n, 0.0);
    if (d.torque_rows) {
        std::memcpy(tmx.data(), d.tau_max, n * 8);
        std::memcpy(tmn.data(), d.tau_min, n * 8);
    }
    bool ok = hipMalloc(&c->tmax, n * 8) == hipSuccess && hipMalloc(&c->tmin, n * 8) == hipSuccess &&
              hipMalloc(&c->dev_in, (in_elems + cm_elems) * 8) == hipSuccess &&
              hipHostMalloc((void **)&c->host_in, (in_elems + cm_elems) * 8, hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&c->dev_out, out_bytes) == hipSuccess &&
              hipHostMalloc((void **)&c->host_out, out_bytes, hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&c->dev_x, B * c->nx * 8) == hipSuccess &&
              hipMalloc(&c->work, 4 * sizeof(int)) == hipSuccess && hipMemset(c->work, 0, 4 * sizeof(int)) == hipSuccess &&
              alloc_work_seen(c) && hipMalloc(&c->wl, B * sizeof(int)) == hipSuccess &&
              hipMalloc(&c->ws_rows, B * 64) == hipSuccess && hipMemset(c->ws_rows, 0, B * 64) == hipSuccess &&
              hipEventCreateWithFlags(&c->in_copied, hipEventDisableTiming) == hipSuccess;
    if (!ok) return cleanup(WBQ_E_DEVICE);
    ok = hipMemcpy(c->tmax, tmx.data(), n * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->tmin, tmn.data(), n * 8, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) return cleanup(WBQ_E_DEVICE);
#ifdef WBQ_STAMPS
    if (hipMalloc(&c->stamps, sizeof(unsigned long long) * wbq::kStamps * B) != hipSuccess)
        return cleanup(WBQ_E_DEVICE);
#endif
    if (prime_contact(c) != WBQ_SUCCESS) return cleanup(WBQ_E_DEVICE);
    *out = c;
    return WBQ_SUCCESS;
}

int wbq_set_contact_inputs(wbq_ctx *c, const wbq_contact_inputs *in)
{
    if (!c || !in) return WBQ_E_INVALID;
    if (c->form != WBQ_FORM_CONTACT) return fail(c, WBQ_E_INVALID, "wbq_set_contact_inputs on a QPPVM-form context");
    if (in->batch < 0 || in->batch > c->d.max_batch) return fail(c, WBQ_E_CAPACITY, "batch exceeds max_batch");
    const double *src[kContactFields] = {in->M, in->h, in->q, in->qd, in->qref, in->Jw, in->jdqd_w, in->pose_w,
                                         in->pose_w_ref, in->Jc, in->jdqd_c, in->pose_c, in->pose_c_ref};
    if (in->batch > 0) {
        for (int f = 0; f < kContactFields; ++f)
            if (!src[f]) return fail(c, WBQ_E_INVALID, "null input pointer");
        if (!in->cmask) return fail(c, WBQ_E_INVALID, "null contact mask");
    }
    if (in->memory != WBQ_MEM_DEVICE && in->memory != WBQ_MEM_HOST)
        return fail(c, WBQ_E_INVALID, "unknown memory kind");
    WBQ_HIP(hipSetDevice(c->device));
    if (in->memory == WBQ_MEM_DEVICE) {
        for (int f = 0; f < kContactFields; ++f) c->in[f] = src[f];
        c->cmask = in->cmask;
    } else {
        if (c->in_pending) WBQ_HIP(hipEventSynchronize(c->in_copied));
        size_t off = 0;
        for (int f = 0; f < kContactFields; ++f) {
            const size_t e = c->fe[f] * (size_t)in->batch;
            if (e) std::memcpy(c->host_in + off, src[f], e * 8);
            c->in[f] = c->dev_in + off;
            off += e;
        }
        if (in->batch > 0) std::memcpy(c->host_in + off, in->cmask, (size_t)in->batch * 4);
        c->cmask = (const int *)(c->dev_in + off);
        off += ((size_t)in->batch + 1) / 2;
        if (in->batch > 0) {
            WBQ_HIP(hipMemcpyAsync(c->dev_in, c->host_in, off * 8, hipMemcpyHostToDevice, c->stream));
            WBQ_HIP(hipEventRecord(c->in_copied, c->stream));
            c->in_pending = true;
            c->in_stream = c->stream;
        }
    }
    c->batch = in->batch;
    c->tau = c->dev_out;
    c->status = (int *)(c->dev_out + (size_t)c->batch * c->d.n);
    c->iters = c->status + c->batch;
    c->have_inputs = true;
    return WBQ_SUCCESS;
}

int wbq_get_contact_outputs(wbq_ctx *c, double *x)
{
    if (!c) return WBQ_E_INVALID;
    if (c->form != WBQ_FORM_CONTACT) return fail(c, WBQ_E_INVALID, "not a contact-form context");
    if (!x || c->batch == 0) return WBQ_SUCCESS;
    WBQ_HIP(hipSetDevice(c->device));
    WBQ_HIP(hipMemcpyAsync(x, c->dev_x, (size_t)c->batch * c->nx * 8, hipMemcpyDeviceToHost, c->stream));
    WBQ_HIP(hipStreamSynchronize(c->stream));
    return WBQ_SUCCESS;
}

int wbq_set_stream(wbq_ctx *c, void *hip_stream)
{
    if (!c) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    c->stream = hip_stream == WBQ_NULL_STREAM ? (hipStream_t)0 : hip_stream ? (hipStream_t)hip_stream : c->own_stream;
    return WBQ_SUCCESS;
}

int wbq_set_inputs(wbq_ctx *c, const wbq_inputs *in)
{
    if (!c || !in) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE; // (its repair reads the current inputs)
    if (c->form != WBQ_FORM_QPPVM) return fail(c, WBQ_E_INVALID, "wbq_set_inputs on a contact-form context");
    if (in->batch < 0 || in->batch > c->d.max_batch)
        return fail(c, WBQ_E_CAPACITY, "batch exceeds max_batch");
    const double *src[8] = {in->M, in->J, in->pose, in->pose_ref, in->q, in->qd, in->qref, in->h};
    for (int f = 0; f < 8; ++f)
        if (!src[f] && in->batch > 0) return fail(c, WBQ_E_INVALID, "null input pointer");
    if (in->memory != WBQ_MEM_DEVICE && in->memory != WBQ_MEM_HOST)
        return fail(c, WBQ_E_INVALID, "unknown memory kind");
    WBQ_HIP(hipSetDevice(c->device));
    c->inputs_device = in->memory == WBQ_MEM_DEVICE;
    if (in->memory == WBQ_MEM_DEVICE) {
        for (int f = 0; f < 8; ++f) c->in[f] = src[f];
    } else {
        // the staging block may still feed the previous copy: wait for it first
        if (c->in_pending) WBQ_HIP(hipEventSynchronize(c->in_copied));
        size_t off = 0;
        for (int f = 0; f < 8; ++f) {
            const size_t e = c->fe[f] * (size_t)in->batch;
            if (e) std::memcpy(c->host_in + off, src[f], e * 8);
            c->in[f] = c->dev_in + off;
            off += e;
        }
        if (off) {
            WBQ_HIP(hipMemcpyAsync(c->dev_in, c->host_in, off * 8, hipMemcpyHostToDevice, c->stream));
            WBQ_HIP(hipEventRecord(c->in_copied, c->stream));
            c->in_pending = true;
            c->in_stream = c->stream;
        }
    }
    c->batch = in->batch;
    // output block for this batch: [tau | status | iters]
    c->tau = c->dev_out;
    c->status = (int *)(c->dev_out + (size_t)c->batch * c->d.n);
    c->iters = c->status + c->batch;
    c->have_inputs = true;
    return WBQ_SUCCESS;
}

// prepare: raise the LDS limits of every kernel variant this context can launch, launch nothing
// (wbq_create*: the solve path then takes no lock and does not allocate). rbd: re-evaluate the model
// in place first (wbq_rollout_rbd), inside the timed window of a timed solve.
static int solve_impl(wbq_ctx *c, int integrate, double dt, bool prepare = false, const wbq_rbd_ctx *rbd = nullptr,
                      int steps = 0)
{
    if (!c) return WBQ_E_INVALID;
    if (!c->have_inputs) return fail(c, WBQ_E_INVALID, "wbq_set_inputs not called");
    if (c->in_pending && c->in_stream != c->stream) {
        // the stream was switched after the host inputs were copied: order the solve behind
        // that copy (the epoch-parity work counters also need the solves stream-ordered, so a
        // context should otherwise stay on one stream between solves)
        WBQ_HIP(hipSetDevice(c->device));
        WBQ_HIP(hipStreamWaitEvent(c->stream, c->in_copied, 0));
        c->in_stream = c->stream;
    }
    if (c->form == WBQ_FORM_CONTACT) return solve_contact(c, integrate, dt, prepare, rbd);
    wbq::QppvmArgs a{};
    a.B = c->batch;
    a.n = c->d.n;
    a.ntasks = c->d.ntasks;
    a.m0 = c->m0;
    a.m_l0 = c->m_l0;
    a.select_mode = c->d.select_mode;
    a.joint_weight = c->d.joint_weight;
    a.minnorm = c->d.no_joint_task;
    a.max_iter = c->d.max_iter;
    a.limits_crossed = c->limits_crossed;
    for (int t = 0; t < wbq::kTMax; ++t) a.row_mask[t] = t < c->d.ntasks ? c->d.row_mask[t] : 0;
    a.row_sel = c->row_sel;
    for (int r = 0; r < wbq::kM0Max; ++r) a.row_selv[r] = c->row_sel_host[r];
    a.Kc = c->Kc;
    a.Dc = c->Dc;
    a.Kq = c->Kq;
    a.Dq = c->Dq;
    a.tau_max = c->tmax;
    a.tau_min = c->tmin;
    a.M = c->in[0];
    a.J = c->in[1];
    a.pose = c->in[2];
    a.pose_ref = c->in[3];
    a.q = c->in[4];
    a.qd = c->in[5];
    a.qref = c->in[6];
    a.h = c->in[7];
    a.tau = c->out_tau ? c->out_tau : c->tau;
    a.status = c->out_status ? c->out_status : c->status;
    a.iters = c->out_iters ? c->out_iters : c->iters;
    a.stamps = c->stamps;
    a.u_scr = c->u_scr;
    a.q1_scr = c->q1_scr;
    a.ui_scr = c->ui_scr;
    a.lo_scr = c->lo_scr;
    a.hi_scr = c->hi_scr;
    a.handback = (c->lo_scr && c->opt_handback) ? 1 : 0;
    a.gi_handoff = a.handback ? c->opt_handoff : 0;
    a.b0_scr = c->b0_scr;
    a.work = c->work;
    a.wl = c->wl;
    a.epoch = c->epoch;
    a.fg = follow_grid(c);
    a.ws_hint = c->ws_hint;
    a.ws_state = c->ws_state;
    a.ws_rows = c->ws_rows;
    a.joint_limits = c->d.joint_limits;
    if (c->jl) {
        a.q_min = c->jl;
        a.q_max = c->jl + c->d.n;
        a.Kjl = c->jl + 2 * c->d.n;
        a.Djl = c->jl + 3 * c->d.n;
    }
    a.integrate = integrate;
    a.dt = dt;
    a.prepare = prepare ? 1 : 0;
    a.steps = steps;
    {
        // n <= 32: the level-0 repair runs inside the fast kernel when the last solves needed it
        // (one launch per solve instead of a follow-up launch that waits for the whole fast kernel:
        // config 4 7.8 -> 9.8 M QP/s), in qppvm_repair_kernel otherwise (the inline variant's fast
        // path is ~5 us slower than the ~3 us that launch costs: config 1). WBQ_INLREP=0/1 forces it.
        // (held for 64 solves after the last repair seen: rollouts repair a few instances now and then)
        const int seen1 = c->work_seen ? __atomic_load_n(c->work_seen + 1, __ATOMIC_RELAXED) : 0;
        if (seen1 > 0) c->inl_hold = 64;
        else if (c->inl_hold > 0) --c->inl_hold;
        a.inline_repair = c->opt_inline >= 0 ? c->opt_inline : (c->inl_hold > 0 ? 1 : 0);
        // On-demand follow-up (WBQ_OPT_FOLLOWUP): while the last solves listed no repair, the n <= 32
        // merged path enqueues the fast kernel alone (an empty follow-up launch costs ~1.5-3 us of a
        // ~35 us config-1 step); a solve that did list one is completed when its outputs are read
        // (complete_pending). Not with caller-owned device outputs (a stream consumer would read them
        // before that), caller-owned device inputs (the deferred repair would read them when the outputs
        // are read, after the caller may have refilled them on the stream), rollouts, rbd re-evaluation,
        // or the constraint-space and inline variants.
        a.skip_followup = (c->opt_followup == 1 && !prepare && !integrate && steps == 0 && !rbd && a.B > 0 &&
                           !c->inputs_device &&
                           c->d.n <= 32 && c->d.joint_weight == WBQ_WEIGHT_IDENTITY && !c->d.no_joint_task &&
                           !a.inline_repair && !c->out_tau && !c->out_status && !c->out_iters && seen1 == 0 &&
                           c->fest[1] == 0) ? 1 : 0;
        a.self_book = a.skip_followup;
    }

    WBQ_HIP(hipSetDevice(c->device));
    if (prepare) {
        WBQ_HIP(wbq::launch_qppvm(a, c->stream, nullptr));
        return WBQ_SUCCESS;
    }
    // timed solves record (start, after the dominant first kernel, end) on the launch stream
    const bool timed = c->timing && a.B > 0 && c->ev_used + 3 <= (int)c->ev.size() &&
                       (c->solves++ % (unsigned long long)c->timing_every) == 0;
    if (timed) WBQ_HIP(hipEventRecord(c->ev[c->ev_used], c->stream));
    if (rbd)
        WBQ_HIP(wbq::rbd_launch(rbd, c->batch, c->in[4], c->in[5], const_cast<double *>(c->in[0]),
                                const_cast<double *>(c->in[7]), const_cast<double *>(c->in[1]),
                                const_cast<double *>(c->in[2]), c->stream));
    WBQ_HIP(wbq::launch_qppvm(a, c->stream, timed ? c->ev[c->ev_used + 1] : nullptr));
    // (a skipped solve's predecessor, if it was pending, is superseded: its outputs are overwritten)
    c->pending = a.skip_followup != 0;
    if (c->pending) c->pend_args = a;
    if (a.B > 0) c->epoch ^= 1; // solves on one context are stream-ordered
    if (timed) {
        WBQ_HIP(hipEventRecord(c->ev[c->ev_used + 2], c->stream));
        c->ev_mid[c->ev_used / 3] = 1;
        c->ev_used += 3;
    }
    return WBQ_SUCCESS;
}

int wbq_solve(wbq_ctx *c) { return solve_impl(c, 0, 0.0); }

int wbq_set_option(wbq_ctx *c, int option, int value)
{
    if (!c) return WBQ_E_INVALID;
    switch (option) {
    case WBQ_OPT_INLINE_REPAIR:
        if (value < -1 || value > 1) return fail(c, WBQ_E_INVALID, "WBQ_OPT_INLINE_REPAIR: -1, 0 or 1");
        c->opt_inline = value;
        return WBQ_SUCCESS;
    case WBQ_OPT_FUSED_ROLLOUT:
        if (value < 0 || value > 1) return fail(c, WBQ_E_INVALID, "WBQ_OPT_FUSED_ROLLOUT: 0 or 1");
        c->opt_fused = value;
        return WBQ_SUCCESS;
    case WBQ_OPT_FOLLOWUP:
        if (value < 0 || value > 1) return fail(c, WBQ_E_INVALID, "WBQ_OPT_FOLLOWUP: 0 or 1");
        if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
        c->opt_followup = value;
        return WBQ_SUCCESS;
    case WBQ_OPT_HANDBACK:
        if (value < 0 || value > 1) return fail(c, WBQ_E_INVALID, "WBQ_OPT_HANDBACK: 0 or 1");
        if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
        c->opt_handback = value;
        return WBQ_SUCCESS;
    case WBQ_OPT_GI_HANDOFF:
        if (value < 0) return fail(c, WBQ_E_INVALID, "WBQ_OPT_GI_HANDOFF: >= 0");
        if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
        c->opt_handoff = value;
        return WBQ_SUCCESS;
    default:
        return fail(c, WBQ_E_INVALID, "wbq_set_option: unknown option");
    }
}

int wbq_rollout(wbq_ctx *c, int steps, double dt)
{
    if (!c) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    if (steps < 0 || !(dt >= 0.0)) return fail(c, WBQ_E_INVALID, "wbq_rollout: steps >= 0, dt >= 0");
    if (c->form == WBQ_FORM_QPPVM && c->d.no_joint_task)
        return fail(c, WBQ_E_UNSUPPORTED, "wbq_rollout: not with no_joint_task (qdd = M^-1 x is not carried)");
    // QPPVM W1 = I with n <= 32 and m0 <= 6: the whole rollout in one launch (qppvm_rollout_kernel);
    // WBQ_OPT_FUSED_ROLLOUT = 0 keeps one launch per step (the A/B of the two)
    if (c->opt_fused && steps > 0 && c->form == WBQ_FORM_QPPVM && c->d.joint_weight == WBQ_WEIGHT_IDENTITY &&
        c->d.n <= 32 && c->m0 <= 6 && c->m_l0 == c->m0)
        return solve_impl(c, 1, dt, false, nullptr, steps);
    for (int k = 0; k < steps; ++k) {
        const int rc = solve_impl(c, 1, dt);
        if (rc != WBQ_SUCCESS) return rc;
    }
    return WBQ_SUCCESS;
}

int wbq_rollout_rbd(wbq_ctx *c, wbq_rbd_ctx *rbd, int steps, double dt)
{
    if (!c || !rbd) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    if (!c->have_inputs) return fail(c, WBQ_E_INVALID, "no inputs set");
    const int want_t = c->form == WBQ_FORM_CONTACT ? 1 + c->cd.nc : c->d.ntasks;
    if (wbq::rbd_n(rbd) != c->d.n || wbq::rbd_ntasks(rbd) != want_t || wbq::rbd_device(rbd) != c->device)
        return fail(c, WBQ_E_INVALID, "wbq_rollout_rbd: model n / tasks / device differ from the context's "
                                      "(contact form: the waist and the nc contact frames)");
    if (steps < 0 || !(dt >= 0.0)) return fail(c, WBQ_E_INVALID, "wbq_rollout_rbd: steps >= 0, dt >= 0");
    if (c->form == WBQ_FORM_QPPVM && c->d.no_joint_task)
        return fail(c, WBQ_E_UNSUPPORTED, "wbq_rollout_rbd: not with no_joint_task (qdd = M^-1 x is not carried)");
    WBQ_HIP(hipSetDevice(c->device));
    if (c->in_pending && c->in_stream != c->stream) {
        WBQ_HIP(hipStreamWaitEvent(c->stream, c->in_copied, 0));
        c->in_stream = c->stream;
    }
    // the model is re-evaluated in place at the integrated state, then one integrating solve (a
    // timed step times both: its dominant-kernel window holds the model kernel and the fast kernel)
    for (int k = 0; k < steps; ++k) {
        const int rc = solve_impl(c, 1, dt, false, rbd);
        if (rc != WBQ_SUCCESS) return rc;
    }
    return WBQ_SUCCESS;
}

int wbq_get_state(wbq_ctx *c, double *q, double *qd)
{
    if (!c) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    if (!c->have_inputs) return fail(c, WBQ_E_INVALID, "no inputs set");
    if (c->batch == 0) return WBQ_SUCCESS;
    WBQ_HIP(hipSetDevice(c->device));
    const size_t bytes = (size_t)c->batch * c->d.n * 8;
    const double *dq = c->form == WBQ_FORM_CONTACT ? c->in[2] : c->in[4];
    const double *dqd = c->form == WBQ_FORM_CONTACT ? c->in[3] : c->in[5];
    if (q) WBQ_HIP(hipMemcpyAsync(q, dq, bytes, hipMemcpyDeviceToHost, c->stream));
    if (qd) WBQ_HIP(hipMemcpyAsync(qd, dqd, bytes, hipMemcpyDeviceToHost, c->stream));
    WBQ_HIP(hipStreamSynchronize(c->stream));
    return WBQ_SUCCESS;
}

int wbq_set_state(wbq_ctx *c, const double *q, const double *qd, int memory)
{
    if (!c) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    if (!c->have_inputs) return fail(c, WBQ_E_INVALID, "no inputs set");
    if (memory != WBQ_MEM_DEVICE && memory != WBQ_MEM_HOST) return fail(c, WBQ_E_INVALID, "unknown memory kind");
    if (c->batch == 0) return WBQ_SUCCESS;
    WBQ_HIP(hipSetDevice(c->device));
    const size_t bytes = (size_t)c->batch * c->d.n * 8;
    double *dq = const_cast<double *>(c->form == WBQ_FORM_CONTACT ? c->in[2] : c->in[4]);
    double *dqd = const_cast<double *>(c->form == WBQ_FORM_CONTACT ? c->in[3] : c->in[5]);
    const hipMemcpyKind kind = memory == WBQ_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (q) WBQ_HIP(hipMemcpyAsync(dq, q, bytes, kind, c->stream));
    if (qd) WBQ_HIP(hipMemcpyAsync(dqd, qd, bytes, kind, c->stream));
    if (memory == WBQ_MEM_HOST) WBQ_HIP(hipStreamSynchronize(c->stream)); // caller may reuse its buffers
    return WBQ_SUCCESS;
}

// An on-demand solve (WBQ_OPT_FOLLOWUP) whose fast kernel listed instances for the level-0 repair is
// finished here, before any of its outputs are read: the flag the listing set in mapped host memory,
// then the repair kernel over that solve's list. A solve that listed none costs one host read.
static int complete_pending(wbq_ctx *c)
{
    if (!c->pending) return WBQ_SUCCESS;
    c->pending = false;
    WBQ_HIP(hipSetDevice(c->device));
    WBQ_HIP(hipStreamSynchronize(c->stream));
    if (c->work_seen && __atomic_load_n(c->work_seen + 2, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(c->work_seen + 2, 0, __ATOMIC_RELEASE);
        wbq::QppvmArgs a = c->pend_args;
        a.skip_followup = 0;
        a.self_book = 0;
        a.fg = follow_grid(c);
        WBQ_HIP(wbq::launch_qppvm_followup(a, c->stream));
        WBQ_HIP(hipStreamSynchronize(c->stream));
    }
    return WBQ_SUCCESS;
}

int wbq_sync(wbq_ctx *c)
{
    if (!c) return WBQ_E_INVALID;
    if (c->pending) return complete_pending(c);
    WBQ_HIP(hipStreamSynchronize(c->stream));
    return WBQ_SUCCESS;
}

int wbq_get_outputs(wbq_ctx *c, double *tau, int32_t *status, int32_t *iters)
{
    if (!c) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    WBQ_HIP(hipSetDevice(c->device));
    const size_t B = (size_t)c->batch, n = (size_t)c->d.n;
    if (B == 0) return WBQ_SUCCESS;
    double *ht = c->host_out;
    int *hs = (int *)(c->host_out + B * n), *hi = hs + B;
    if (!c->out_tau && !c->out_status && !c->out_iters) {
        // one pinned D2H copy of the packed block
        WBQ_HIP(hipMemcpyAsync(c->host_out, c->dev_out, B * n * 8 + 2 * B * 4, hipMemcpyDeviceToHost, c->stream));
    } else {
        WBQ_HIP(hipMemcpyAsync(ht, c->out_tau ? c->out_tau : c->tau, B * n * 8, hipMemcpyDeviceToHost, c->stream));
        WBQ_HIP(hipMemcpyAsync(hs, c->out_status ? c->out_status : c->status, B * 4, hipMemcpyDeviceToHost, c->stream));
        WBQ_HIP(hipMemcpyAsync(hi, c->out_iters ? c->out_iters : c->iters, B * 4, hipMemcpyDeviceToHost, c->stream));
    }
    WBQ_HIP(hipStreamSynchronize(c->stream));
    if (tau) std::memcpy(tau, ht, B * n * 8);
    if (status) std::memcpy(status, hs, B * 4);
    if (iters) std::memcpy(iters, hi, B * 4);
    return WBQ_SUCCESS;
}

int wbq_set_outputs(wbq_ctx *c, double *tau, int32_t *status, int32_t *iters)
{
    if (!c) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE; // (the last solve wrote the old buffers)
    c->out_tau = tau;
    c->out_status = status;
    c->out_iters = iters;
    return WBQ_SUCCESS;
}

int wbq_get_device_outputs(wbq_ctx *c, const double **tau, const int32_t **status, const int32_t **iters)
{
    if (!c) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE; // (then valid on the stream as well)
    if (tau) *tau = c->out_tau ? c->out_tau : c->tau;
    if (status) *status = c->out_status ? c->out_status : c->status;
    if (iters) *iters = c->out_iters ? c->out_iters : c->iters;
    return WBQ_SUCCESS;
}

int wbq_reset_warmstart(wbq_ctx *c, const uint8_t *mask)
{
    // Drops the per-instance warm start (repair hint, BVLS bound state, the dual loop's last
    // active set), stream-ordered with the solves; a cold instance takes the default path next time.
    if (!c) return WBQ_E_INVALID;
    // a solve left pending (on-demand follow-up) first: its deferred repair writes the warm-start state
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    if (!c->ws_hint && !c->ws_rows) return WBQ_SUCCESS; // no warm-start state in this form
    WBQ_HIP(hipSetDevice(c->device));
    const int B = mask ? c->batch : c->d.max_batch; // a mask has one entry per instance of the batch
    int b = 0;
    while (b < B) {
        if (mask && !mask[b]) {
            ++b;
            continue;
        }
        int e = b + 1;
        while (e < B && (!mask || mask[e])) ++e;
        if (c->ws_hint) {
            WBQ_HIP(hipMemsetAsync(c->ws_hint + b, 0, (size_t)(e - b), c->stream));
            WBQ_HIP(hipMemsetAsync(c->ws_state + (size_t)b * c->np, 0, (size_t)(e - b) * c->np, c->stream));
        }
        if (c->ws_rows) WBQ_HIP(hipMemsetAsync(c->ws_rows + (size_t)b * 64, 0, (size_t)(e - b) * 64, c->stream));
        b = e;
    }
    return WBQ_SUCCESS;
}

int wbq_get_warmstart_hints(wbq_ctx *c, uint8_t *hints)
{
    if (!c || !hints) return WBQ_E_INVALID;
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    if (c->batch == 0) return WBQ_SUCCESS;
    if (!c->ws_hint) {
        std::memset(hints, 0, (size_t)c->batch);
        return WBQ_SUCCESS;
    }
    WBQ_HIP(hipSetDevice(c->device));
    WBQ_HIP(hipMemcpyAsync(hints, c->ws_hint, (size_t)c->batch, hipMemcpyDeviceToHost, c->stream));
    WBQ_HIP(hipStreamSynchronize(c->stream));
    for (int b = 0; b < c->batch; ++b) hints[b] &= 1; // bit 1 (W1 = I: ws_rows valid) is internal
    return WBQ_SUCCESS;
}

int wbq_set_timing(wbq_ctx *c, int enable)
{
    if (!c) return WBQ_E_INVALID;
    // (a pending solve's deferred repair belongs to the solves before this window, not to the timed ones)
    if (complete_pending(c) != WBQ_SUCCESS) return WBQ_E_DEVICE;
    WBQ_HIP(hipSetDevice(c->device));
    if (enable && c->ev.empty()) {
        c->ev.resize(3 * 4096);
        c->ev_mid.assign(4096, 2);
        for (auto &e : c->ev) WBQ_HIP(hipEventCreate(&e));
    }
    c->timing = enable > 0;
    c->timing_every = enable > 0 ? enable : 1;
    c->solves = 0;
    c->ev_used = 0;
    c->t_acc_ms = 0.0;
    c->t_kern_ms = 0.0;
    c->t_launches = 0;
    return WBQ_SUCCESS;
}

int wbq_get_timing_detail(wbq_ctx *c, double *solve_ms, double *kernel_ms, int *launches)
{
    if (!c) return WBQ_E_INVALID;
    WBQ_HIP(hipSetDevice(c->device));
    for (int k = 0; k + 2 < c->ev_used; k += 3) {
        WBQ_HIP(hipEventSynchronize(c->ev[k + 2]));
        float ms = 0.f, km = 0.f;
        WBQ_HIP(hipEventElapsedTime(&ms, c->ev[k], c->ev[k + 2]));
        WBQ_HIP(hipEventElapsedTime(&km, c->ev[k], c->ev[k + c->ev_mid[k / 3]]));
        c->t_acc_ms += ms;
        c->t_kern_ms += km;
        c->t_launches += 1;
    }
    c->ev_used = 0;
    if (solve_ms) *solve_ms = c->t_acc_ms;
    if (kernel_ms) *kernel_ms = c->t_kern_ms;
    if (launches) *launches = c->t_launches;
    c->t_acc_ms = 0.0;
    c->t_kern_ms = 0.0;
    c->t_launches = 0;
    return WBQ_SUCCESS;
}

int wbq_get_timing(wbq_ctx *c, double *total_ms, int *launches)
{
    return wbq_get_timing_detail(c, total_ms, nullptr, launches);
}

#ifdef WBQ_STAMPS
// Diagnostic-only symbol (not in include/wbq.h): per-block phase stamps of the last solve.
int wbq_diag_stamps(wbq_ctx *c, unsigned long long *host, int nblocks)
{
    if (!c || !c->stamps) return WBQ_E_INVALID;
    WBQ_HIP(hipStreamSynchronize(c->stream));
    WBQ_HIP(hipMemcpy(host, c->stamps, sizeof(unsigned long long) * wbq::kStamps * nblocks,
                      hipMemcpyDeviceToHost));
    return WBQ_SUCCESS;
}
int wbq_diag_stamps_clear(wbq_ctx *c, int nblocks)
{
    if (!c || !c->stamps) return WBQ_E_INVALID;
    WBQ_HIP(hipStreamSynchronize(c->stream));
    WBQ_HIP(hipMemset(c->stamps, 0, sizeof(unsigned long long) * wbq::kStamps * nblocks));
    return WBQ_SUCCESS;
}
#endif

void wbq_destroy(wbq_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    for (auto &e : c->ev) (void)hipEventDestroy(e);
    double *bufs[] = {c->Kc, c->Dc, c->Kq, c->Dq, c->tmax, c->tmin, c->dev_in, c->dev_out};
    for (double *p : bufs)
        if (p) (void)hipFree(p);
    if (c->host_in) (void)hipHostFree(c->host_in);
    if (c->host_out) (void)hipHostFree(c->host_out);
    if (c->in_copied) (void)hipEventDestroy(c->in_copied);
    if (c->row_sel) (void)hipFree(c->row_sel);
    if (c->stamps) (void)hipFree(c->stamps);
    if (c->u_scr) (void)hipFree(c->u_scr);
    if (c->q1_scr) (void)hipFree(c->q1_scr);
    if (c->ui_scr) (void)hipFree(c->ui_scr);
    if (c->lo_scr) (void)hipFree(c->lo_scr);
    if (c->hi_scr) (void)hipFree(c->hi_scr);
    if (c->b0_scr) (void)hipFree(c->b0_scr);
    if (c->work) (void)hipFree(c->work);
    if (c->work_seen) (void)hipHostFree(c->work_seen);
    if (c->wl) (void)hipFree(c->wl);
    if (c->ws_hint) (void)hipFree(c->ws_hint);
    if (c->ws_state) (void)hipFree(c->ws_state);
    if (c->ws_rows) (void)hipFree(c->ws_rows);
    if (c->jl) (void)hipFree(c->jl);
    if (c->dev_x) (void)hipFree(c->dev_x);

    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

}  // extern "C"

namespace {

// identity rotation, zero translation (row-major 3 x 4)
void rest_pose(double *p)
{
    for (int k = 0; k < 12; ++k) p[k] = (k == 0 || k == 5 || k == 10) ? 1.0 : 0.0;
}

void prime_reset(wbq_ctx *c)
{
    c->have_inputs = false;
    c->batch = 0;
    c->in_pending = false;
    for (auto &p : c->in) p = nullptr;
    c->cmask = nullptr;
}

int prime_qppvm(wbq_ctx *c)
{
    const int n = c->d.n, T = c->d.ntasks;
    std::vector<double> M((size_t)n * n, 0.0), J((size_t)T * 6 * n, 0.0), pose((size_t)T * 12), v(n, 0.0);
    for (int j = 0; j < n; ++j) M[(size_t)j * n + j] = 1.0;
    for (int t = 0; t < T; ++t) {
        for (int r = 0; r < 6; ++r) J[((size_t)t * 6 + r) * n + (t * 6 + r) % n] = 1.0;
        rest_pose(pose.data() + 12 * t);
    }
    wbq_inputs in{};
    in.batch = 1;
    in.memory = WBQ_MEM_HOST;
    in.M = M.data();
    in.J = J.data();
    in.pose = in.pose_ref = pose.data();
    in.q = in.qd = in.qref = in.h = v.data();
    int rc = wbq_set_inputs(c, &in);
    if (rc == WBQ_SUCCESS) rc = solve_impl(c, 0, 0.0, true);
    if (rc == WBQ_SUCCESS) rc = wbq_solve(c);
    if (rc == WBQ_SUCCESS) rc = wbq_sync(c);
    if (rc == WBQ_SUCCESS) rc = wbq_reset_warmstart(c, nullptr);
    if (rc == WBQ_SUCCESS) rc = wbq_sync(c);
    prime_reset(c);
    return rc;
}

int prime_contact(wbq_ctx *c)
{
    const int n = c->cd.n, nc = c->cd.nc;
    std::vector<double> M((size_t)n * n, 0.0), v(n, 0.0), Jw((size_t)6 * n, 0.0), z6(6 * nc, 0.0),
        Jc((size_t)nc * 6 * n, 0.0), pw(12), pc((size_t)nc * 12);
    for (int j = 0; j < n; ++j) M[(size_t)j * n + j] = 1.0;
    for (int r = 0; r < 6; ++r) Jw[(size_t)r * n + r] = 1.0;
    for (int k = 0; k < nc; ++k)
        for (int r = 0; r < 6; ++r) Jc[((size_t)k * 6 + r) * n + r] = 1.0;
    rest_pose(pw.data());
    for (int k = 0; k < nc; ++k) rest_pose(pc.data() + 12 * k);
    const int32_t cm = 0; // no contact: forces fixed at zero
    wbq_contact_inputs in{};
    in.batch = 1;
    in.memory = WBQ_MEM_HOST;
    in.M = M.data();
    in.h = in.q = in.qd = in.qref = v.data();
    in.Jw = Jw.data();
    in.jdqd_w = z6.data();
    in.pose_w = in.pose_w_ref = pw.data();
    in.Jc = Jc.data();
    in.jdqd_c = z6.data();
    in.pose_c = in.pose_c_ref = pc.data();
    in.cmask = &cm;
    int rc = wbq_set_contact_inputs(c, &in);
    if (rc == WBQ_SUCCESS) rc = solve_impl(c, 0, 0.0, true);
    if (rc == WBQ_SUCCESS) rc = wbq_solve(c);
    if (rc == WBQ_SUCCESS) rc = wbq_sync(c);
    if (rc == WBQ_SUCCESS) rc = wbq_reset_warmstart(c, nullptr);
    if (rc == WBQ_SUCCESS) rc = wbq_sync(c);
    prime_reset(c);
    return rc;
}

}  // namespace
