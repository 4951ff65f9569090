// rbd.hip -- batched rigid-body dynamics on gfx950 (fp64): M(q) (CRBA), h(q, qd) (RNEA with
// qdd = 0), task poses and geometric Jacobians, from (q, qd), in the wbq_inputs layouts. The
// XBotInterface ModelInterface calls of the reference (RBDL backend [upstream]) these replace:
// getInertiaMatrix, computeNonlinearTerm (QPPVMPlugin.cpp:65,312), getPose / getJacobian
// (QPPVMPlugin.cpp:272-284, the Cartesian tasks :129-152), the ID of ForceAcc.cpp:208-217.
//
// One instance per wave64, lane k <-> link k (n <= 64); everything in the WORLD frame with
// Plucker coordinates at the world origin, so the recursions become sums over ancestor /
// descendant sets (precomputed bit masks) that every lane evaluates for its own link:
//   FK        W_k = W_parent T_k(q_k)                       depth-ordered levels (one compose each)
//   S_k       [a_k; o_k x a_k] (revolute), [0; a_k] (prismatic)  world joint axis a_k through o_k
//   v_k, a_k  v_parent + S_k qd_k,  a_parent + v_k x S_k qd_k (a_base = [0; -g]; depth levels)
//   f_k       I_k a_k + v_k x* (I_k v_k)
//   h_k       S_k . sum_{j in subtree(k)} f_j              (RNEA backward pass as a subtree sum)
//   Ic_k      sum_{j in subtree(k)} I_j,  u_k = Ic_k S_k     (CRBA composite inertias)
//   M_ij      S_i . u_j  if i is an ancestor of j (u_i . S_j the other way round, 0 otherwise)
//   J_e[:, j] [a_j x (p_e - o_j); a_j] (prismatic [a_j; 0]) for the joints j on the path of task
//             frame e (its link's frame times a fixed offset)
//   Jdot qd   [a_l + a_w x p_e + w x (v_l + w x p_e); a_w] from the link's spatial acceleration
//             (a_w, a_l) with qdd = 0 and gravity removed, and its velocity (w, v_l)
// The checker (oracle/wbq_oracle_rbd.c) uses the link-frame recursions instead.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/wbq.h"
#include "wbq_kernels.h"

namespace wbq {

namespace {

constexpr int kRbdTMax = 5; // the contact form's waist + 4 contact frames

struct RbdArgs {
    int B, n, ntasks, maxdepth;
    const int *parent, *depth, *jtype; // jtype [n]: 0 revolute, 1 prismatic
    const unsigned long long *anc; // [n] bit j: link j is an ancestor of link k or k itself
    const double *Xf, *axis, *mass, *com, *inertia;
    const double *toff; // [ntasks][12] task frame in its link's frame
    double g[3];
    int task_link[kRbdTMax];
    const double *q, *qd;
    double *M, *h;
    // task outputs in two groups: tasks [0, split) into J, pose, jdqd ([B][split][..]), tasks
    // [split, ntasks) into J2, pose2, jdqd2 ([B][ntasks - split][..]); the contact form's waist and
    // contact frames live in separate input arrays (any pointer may be null)
    int split;
    double *J, *pose, *jdqd, *J2, *pose2, *jdqd2;
};

// LDS per instance, doubles per link
struct RbdLds {
    static constexpr int W = 0, S = 12, V = 18, A = 24, F = 30, U = 36, IC = 42, STRIDE = 53; // odd stride
};

__device__ __forceinline__ void cross(const double *a, const double *b, double *c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

__global__ __launch_bounds__(64) void rbd_kernel(const RbdArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int k = threadIdx.x;
    const long b = blockIdx.x;
    const int n = a.n;
    const bool lk = k < n;
    const int kc = lk ? k : n - 1;
    double *L = smem + k * RbdLds::STRIDE;
    auto at = [&](int j) { return smem + j * RbdLds::STRIDE; };
    const double qk = lk ? a.q[b * n + k] : 0.0, qdk = lk ? a.qd[b * n + k] : 0.0;
    const int par = a.parent[kc], dep = a.depth[kc];
    const bool pri = a.jtype[kc] == 1;

    // ---- local transform T_k = X_fixed Rot(axis, q) (revolute) or X_fixed Trans(axis q) (prismatic)
    double T[12];
    {
        const double *ax = a.axis + 3 * kc, *X = a.Xf + 12 * kc;
        double s, c;
        sincos(pri ? 0.0 : qk, &s, &c);
        const double v = 1.0 - c, x = ax[0], y = ax[1], z = ax[2];
        const double Rq[9] = {c + x * x * v, x * y * v - z * s, x * z * v + y * s,
                              y * x * v + z * s, c + y * y * v, y * z * v - x * s,
                              z * x * v - y * s, z * y * v + x * s, c + z * z * v};
        const double tq = pri ? qk : 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
                T[4 * r + cc] = X[4 * r] * Rq[cc] + X[4 * r + 1] * Rq[3 + cc] + X[4 * r + 2] * Rq[6 + cc];
            T[4 * r + 3] = X[4 * r + 3] + tq * (X[4 * r] * x + X[4 * r + 1] * y + X[4 * r + 2] * z);
        }
    }
    // ---- forward kinematics by depth level: W_k = W_parent T_k
    double W[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) W[e] = T[e];
    for (int d = 0; d < a.maxdepth; ++d) {
        if (lk && dep == d) {
            if (par < 0) {
#pragma unroll
                for (int e = 0; e < 12; ++e) W[e] = T[e];
            } else {
                const double *P = at(par) + RbdLds::W;
#pragma unroll
                for (int r = 0; r < 3; ++r) {
#pragma unroll
                    for (int cc = 0; cc < 4; ++cc)
                        W[4 * r + cc] = P[4 * r] * T[cc] + P[4 * r + 1] * T[4 + cc] + P[4 * r + 2] * T[8 + cc] +
                                        (cc == 3 ? P[4 * r + 3] : 0.0);
                }
            }
#pragma unroll
            for (int e = 0; e < 12; ++e) L[RbdLds::W + e] = W[e];
        }
        __syncthreads();
    }
    // ---- world joint axis, motion subspace, inertia (about the COM, world frame)
    double ax[3], o[3], S[6], m = 0.0, c[3], Ic[6]; // Ic: xx yy zz xy xz yz
    {
        const double *al = a.axis + 3 * kc, *cl = a.com + 3 * kc, *il = a.inertia + 6 * kc;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            ax[r] = W[4 * r] * al[0] + W[4 * r + 1] * al[1] + W[4 * r + 2] * al[2];
            o[r] = W[4 * r + 3];
            c[r] = W[4 * r] * cl[0] + W[4 * r + 1] * cl[1] + W[4 * r + 2] * cl[2] + o[r];
        }
        const double I3[9] = {il[0], il[3], il[4], il[3], il[1], il[5], il[4], il[5], il[2]};
        double RI[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
                RI[3 * r + cc] = W[4 * r] * I3[cc] + W[4 * r + 1] * I3[3 + cc] + W[4 * r + 2] * I3[6 + cc];
        auto rir = [&](int r, int cc) {
            return RI[3 * r] * W[4 * cc] + RI[3 * r + 1] * W[4 * cc + 1] + RI[3 * r + 2] * W[4 * cc + 2];
        };
        Ic[0] = rir(0, 0); Ic[1] = rir(1, 1); Ic[2] = rir(2, 2);
        Ic[3] = rir(0, 1); Ic[4] = rir(0, 2); Ic[5] = rir(1, 2);
        m = lk ? a.mass[kc] : 0.0;
        if (pri) {
            S[0] = S[1] = S[2] = 0.0;
            S[3] = ax[0]; S[4] = ax[1]; S[5] = ax[2];
        } else {
            S[0] = ax[0]; S[1] = ax[1]; S[2] = ax[2];
            cross(o, ax, S + 3);
        }
    }
    // spatial inertia at the world origin: A = Ic + m [c]x [c]x^T (symmetric), mc = m c, m
    double IA[6], mc[3];
    {
        const double cc2 = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
        // [c]x [c]x^T = |c|^2 1 - c c^T
        IA[0] = Ic[0] + m * (cc2 - c[0] * c[0]);
        IA[1] = Ic[1] + m * (cc2 - c[1] * c[1]);
        IA[2] = Ic[2] + m * (cc2 - c[2] * c[2]);
        IA[3] = Ic[3] - m * c[0] * c[1];
        IA[4] = Ic[4] - m * c[0] * c[2];
        IA[5] = Ic[5] - m * c[1] * c[2];
        mc[0] = m * c[0]; mc[1] = m * c[1]; mc[2] = m * c[2];
    }
    if (lk) {
#pragma unroll
        for (int e = 0; e < 6; ++e) L[RbdLds::S + e] = S[e];
#pragma unroll
        for (int e = 0; e < 6; ++e) L[RbdLds::IC + e] = IA[e];
#pragma unroll
        for (int e = 0; e < 3; ++e) L[RbdLds::IC + 6 + e] = mc[e];
        L[RbdLds::IC + 9] = m;
    }
    // ---- velocities and bias accelerations by depth level
    double v[6] = {0, 0, 0, 0, 0, 0}, acc[6] = {0, 0, 0, 0, 0, 0};
    for (int d = 0; d < a.maxdepth; ++d) {
        if (lk && dep == d) {
            double vp[6], ap[6], sq[6], t[6];
            if (par < 0) {
#pragma unroll
                for (int e = 0; e < 6; ++e) vp[e] = 0.0;
                ap[0] = ap[1] = ap[2] = 0.0;
                ap[3] = -a.g[0]; ap[4] = -a.g[1]; ap[5] = -a.g[2];
            } else {
#pragma unroll
                for (int e = 0; e < 6; ++e) {
                    vp[e] = at(par)[RbdLds::V + e];
                    ap[e] = at(par)[RbdLds::A + e];
                }
            }
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                sq[e] = S[e] * qdk;
                v[e] = vp[e] + sq[e];
            }
            // v x sq (motion cross product): [w x sw; w x sl + vl x sw]
            cross(v, sq, t);
            double t2[3], t3[3];
            cross(v, sq + 3, t2);
            cross(v + 3, sq, t3);
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                acc[e] = ap[e] + t[e];
                acc[3 + e] = ap[3 + e] + t2[e] + t3[e];
            }
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                L[RbdLds::V + e] = v[e];
                L[RbdLds::A + e] = acc[e];
            }
        }
        __syncthreads();
    }
    // ---- link force f_k = I a + v x* (I v); I x = [IA w + mc x l; l m - mc x w] for x = [w; l]
    if (lk) {
        auto Imul = [&](const double *x, double *y) {
            double t[3], u[3];
            cross(mc, x + 3, t);
            cross(mc, x, u);
            y[0] = IA[0] * x[0] + IA[3] * x[1] + IA[4] * x[2] + t[0];
            y[1] = IA[3] * x[0] + IA[1] * x[1] + IA[5] * x[2] + t[1];
            y[2] = IA[4] * x[0] + IA[5] * x[1] + IA[2] * x[2] + t[2];
#pragma unroll
            for (int e = 0; e < 3; ++e) y[3 + e] = m * x[3 + e] - u[e];
        };
        double Ia[6], Iv[6], t1[3], t2[3], t3[3];
        Imul(acc, Ia);
        Imul(v, Iv);
        // v x* f = [w x fn + vl x ff; w x ff]
        cross(v, Iv, t1);
        cross(v + 3, Iv + 3, t2);
        cross(v, Iv + 3, t3);
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            L[RbdLds::F + e] = Ia[e] + t1[e] + t2[e];
            L[RbdLds::F + 3 + e] = Ia[3 + e] + t3[e];
        }
    }
    __syncthreads();
    // ---- subtree sums: force (h) and composite inertia (u = Ic S)
    double Fs[6] = {0, 0, 0, 0, 0, 0}, Cs[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (lk) {
        for (int j = k; j < n; ++j) { // descendants have larger indices
            if (!((a.anc[j] >> k) & 1ull)) continue;
            const double *Lj = at(j);
#pragma unroll
            for (int e = 0; e < 6; ++e) Fs[e] += Lj[RbdLds::F + e];
#pragma unroll
            for (int e = 0; e < 10; ++e) Cs[e] += Lj[RbdLds::IC + e];
        }
    }
    const double hk = S[0] * Fs[0] + S[1] * Fs[1] + S[2] * Fs[2] + S[3] * Fs[3] + S[4] * Fs[4] + S[5] * Fs[5];
    double u[6];
    {
        double t[3], w[3];
        cross(Cs + 6, S + 3, t); // mc x l
        cross(S, Cs + 6, w);     // w x mc
        u[0] = Cs[0] * S[0] + Cs[3] * S[1] + Cs[4] * S[2] + t[0];
        u[1] = Cs[3] * S[0] + Cs[1] * S[1] + Cs[5] * S[2] + t[1];
        u[2] = Cs[4] * S[0] + Cs[5] * S[1] + Cs[2] * S[2] + t[2];
#pragma unroll
        for (int e = 0; e < 3; ++e) u[3 + e] = Cs[9] * S[3 + e] + w[e];
    }
    if (lk) {
#pragma unroll
        for (int e = 0; e < 6; ++e) L[RbdLds::U + e] = u[e];
    }
    __syncthreads();
    if (lk && a.h) a.h[b * n + k] = hk;
    // ---- M: lane i computes row i (= column i), stored column-wise for coalescing
    if (lk && a.M) {
        const unsigned long long ai = a.anc[k];
        double *Mb = a.M + b * (long)n * n;
        for (int j = 0; j < n; ++j) {
            const double *Lj = at(j);
            double mij = 0.0;
            if ((a.anc[j] >> k) & 1ull) { // k is an ancestor of j (or j itself): Ic_j
#pragma unroll
                for (int e = 0; e < 6; ++e) mij = fma(S[e], Lj[RbdLds::U + e], mij);
            } else if ((ai >> j) & 1ull) { // j is an ancestor of k: Ic_k
#pragma unroll
                for (int e = 0; e < 6; ++e) mij = fma(u[e], Lj[RbdLds::S + e], mij);
            }
            Mb[(long)j * n + k] = mij;
        }
    }
    // ---- task frames: poses, Jacobians, Jdot qd
    for (int t = 0; t < a.ntasks; ++t) {
        const int e = a.task_link[t];
        const double *Le = at(e), *We = Le + RbdLds::W, *X = a.toff + 12 * t;
        double Pe[12]; // We * X (every lane, redundantly)
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
                Pe[4 * r + cc] = We[4 * r] * X[cc] + We[4 * r + 1] * X[4 + cc] + We[4 * r + 2] * X[8 + cc] +
                                 (cc == 3 ? We[4 * r + 3] : 0.0);
        }
        const bool g2 = t >= a.split;
        const int tl = g2 ? t - a.split : t, tn = g2 ? a.ntasks - a.split : a.split;
        double *Jo = g2 ? a.J2 : a.J, *Po = g2 ? a.pose2 : a.pose, *Do = g2 ? a.jdqd2 : a.jdqd;
        if (Jo && lk) {
            const bool on = (a.anc[e] >> k) & 1ull;
            const double d[3] = {Pe[3] - o[0], Pe[7] - o[1], Pe[11] - o[2]};
            double lin[3];
            cross(ax, d, lin);
            double *Jb = Jo + ((b * tn + tl) * 6) * (long)n;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                Jb[r * n + k] = on ? (pri ? ax[r] : lin[r]) : 0.0;
                Jb[(3 + r) * n + k] = (on && !pri) ? ax[r] : 0.0;
            }
        }
        if (Po && k < 12) Po[(b * tn + tl) * 12 + k] = Pe[k];
        if (Do && k < 6) {
            // the link's spatial velocity / acceleration at the world origin; gravity entered the
            // base acceleration as [0; -g] and propagates unchanged in world coordinates
            const double w[3] = {Le[RbdLds::V], Le[RbdLds::V + 1], Le[RbdLds::V + 2]};
            const double vl[3] = {Le[RbdLds::V + 3], Le[RbdLds::V + 4], Le[RbdLds::V + 5]};
            const double aw[3] = {Le[RbdLds::A], Le[RbdLds::A + 1], Le[RbdLds::A + 2]};
            const double al[3] = {Le[RbdLds::A + 3] + a.g[0], Le[RbdLds::A + 4] + a.g[1], Le[RbdLds::A + 5] + a.g[2]};
            const double pe[3] = {Pe[3], Pe[7], Pe[11]};
            double t1[3], t2[3], vp[3], t3[3];
            cross(aw, pe, t1);
            cross(w, pe, t2);
#pragma unroll
            for (int r = 0; r < 3; ++r) vp[r] = vl[r] + t2[r];
            cross(w, vp, t3);
            double out = 0.0;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                out = k == r ? al[r] + t1[r] + t3[r] : out;
                out = k == 3 + r ? aw[r] : out;
            }
            Do[(b * tn + tl) * 6 + k] = out;
        }
    }
}

}  // namespace

}  // namespace wbq

struct wbq_rbd_ctx {
    int device = 0;
    int n = 0, ntasks = 0, maxdepth = 0, max_batch = 0;
    double g[3] = {0, 0, 0};
    int task_link[wbq::kRbdTMax] = {};
    int *parent = nullptr, *depth = nullptr, *jtype = nullptr;
    unsigned long long *anc = nullptr;
    double *Xf = nullptr, *axis = nullptr, *mass = nullptr, *com = nullptr, *inertia = nullptr, *toff = nullptr;
    double *stage = nullptr;  // device: q, qd, M, h, J, pose, jdqd for host-memory calls
    hipStream_t own_stream = nullptr, stream = nullptr;
};

namespace wbq {

hipError_t rbd_launch_split(const wbq_rbd_ctx *c, int B, const double *q, const double *qd, double *M, double *h,
                            int split, double *J, double *pose, double *jdqd, double *J2, double *pose2, double *jdqd2,
                            hipStream_t stream)
{
    if (B <= 0) return hipSuccess;
    RbdArgs a{};
    a.B = B;
    a.n = c->n;
    a.ntasks = c->ntasks;
    a.maxdepth = c->maxdepth;
    a.parent = c->parent;
    a.depth = c->depth;
    a.jtype = c->jtype;
    a.toff = c->toff;
    a.anc = c->anc;
    a.Xf = c->Xf;
    a.axis = c->axis;
    a.mass = c->mass;
    a.com = c->com;
    a.inertia = c->inertia;
    for (int k = 0; k < 3; ++k) a.g[k] = c->g[k];
    for (int t = 0; t < kRbdTMax; ++t) a.task_link[t] = c->task_link[t];
    a.q = q;
    a.qd = qd;
    a.M = M;
    a.h = h;
    a.split = split;
    a.J = J;
    a.pose = pose;
    a.jdqd = jdqd;
    a.J2 = J2;
    a.pose2 = pose2;
    a.jdqd2 = jdqd2;
    const size_t lds = sizeof(double) * RbdLds::STRIDE * 64;
    hipLaunchKernelGGL(rbd_kernel, dim3((unsigned)B), dim3(64), lds, stream, a);
    return hipGetLastError();
}

hipError_t rbd_launch(const wbq_rbd_ctx *c, int B, const double *q, const double *qd, double *M, double *h, double *J,
                      double *pose, hipStream_t stream)
{
    return rbd_launch_split(c, B, q, qd, M, h, c->ntasks, J, pose, nullptr, nullptr, nullptr, nullptr, stream);
}

int rbd_n(const wbq_rbd_ctx *c) { return c->n; }
int rbd_ntasks(const wbq_rbd_ctx *c) { return c->ntasks; }
int rbd_device(const wbq_rbd_ctx *c) { return c->device; }

}  // namespace wbq

extern "C" {

int wbq_rbd_create(const wbq_rbd_desc *d, int device, wbq_rbd_ctx **out)
{
    if (!d || !out) return WBQ_E_INVALID;
    *out = nullptr;
    const int n = d->n;
    if (n < 1 || n > 64 || d->ntasks < 0 || d->ntasks > wbq::kRbdTMax || d->max_batch < 1) return WBQ_E_INVALID;
    if (!d->parent || !d->X_fixed || !d->axis || !d->mass || !d->com || !d->inertia) return WBQ_E_INVALID;
    if (d->ntasks > 0 && !d->task_link) return WBQ_E_INVALID;
    std::vector<int> depth(n);
    std::vector<unsigned long long> anc(n);
    int maxdepth = 0;
    for (int i = 0; i < n; ++i) {
        const int p = d->parent[i];
        if (p >= i || p < -1) return WBQ_E_INVALID; // parent[i] < i: a topological order
        if (d->jtype && d->jtype[i] != 0 && d->jtype[i] != 1) return WBQ_E_INVALID;
        depth[i] = p < 0 ? 0 : depth[p] + 1;
        anc[i] = (p < 0 ? 0ull : anc[p]) | (1ull << i);
        maxdepth = depth[i] + 1 > maxdepth ? depth[i] + 1 : maxdepth;
        const double *a = d->axis + 3 * i;
        if (std::fabs(a[0] * a[0] + a[1] * a[1] + a[2] * a[2] - 1.0) > 1e-9) return WBQ_E_INVALID;
    }
    for (int t = 0; t < d->ntasks; ++t)
        if (d->task_link[t] < 0 || d->task_link[t] >= n) return WBQ_E_INVALID;
    auto *c = new wbq_rbd_ctx();
    c->device = device;
    c->n = n;
    c->ntasks = d->ntasks;
    c->maxdepth = maxdepth;
    c->max_batch = d->max_batch;
    for (int k = 0; k < 3; ++k) c->g[k] = d->gravity[k];
    for (int t = 0; t < d->ntasks; ++t) c->task_link[t] = d->task_link[t];
    auto fail = [&](int rc) {
        wbq_rbd_destroy(c);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) return fail(WBQ_E_DEVICE);
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) return fail(WBQ_E_DEVICE);
    c->stream = c->own_stream;
    const size_t B = (size_t)d->max_batch, T = (size_t)d->ntasks;
    const size_t stage = B * ((size_t)2 * n + (size_t)n * n + n + T * 6 * n + T * 12 + T * 6);
    std::vector<int> jt(n, 0);
    if (d->jtype) std::memcpy(jt.data(), d->jtype, n * sizeof(int));
    std::vector<double> toff(12 * (T > 0 ? T : 1), 0.0);
    for (size_t t = 0; t < T; ++t)
        for (int e = 0; e < 12; ++e)
            toff[12 * t + e] = d->task_offset ? d->task_offset[12 * t + e] : ((e == 0 || e == 5 || e == 10) ? 1.0 : 0.0);
    bool ok = hipMalloc(&c->parent, n * sizeof(int)) == hipSuccess &&
              hipMalloc(&c->jtype, n * sizeof(int)) == hipSuccess &&
              hipMalloc(&c->toff, toff.size() * 8) == hipSuccess &&
              hipMalloc(&c->depth, n * sizeof(int)) == hipSuccess &&
              hipMalloc(&c->anc, n * sizeof(unsigned long long)) == hipSuccess &&
              hipMalloc(&c->Xf, n * 12 * 8) == hipSuccess && hipMalloc(&c->axis, n * 3 * 8) == hipSuccess &&
              hipMalloc(&c->mass, n * 8) == hipSuccess && hipMalloc(&c->com, n * 3 * 8) == hipSuccess &&
              hipMalloc(&c->inertia, n * 6 * 8) == hipSuccess && hipMalloc(&c->stage, stage * 8) == hipSuccess;
    if (!ok) return fail(WBQ_E_DEVICE);
    ok = hipMemcpy(c->parent, d->parent, n * sizeof(int), hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->jtype, jt.data(), n * sizeof(int), hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->toff, toff.data(), toff.size() * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->depth, depth.data(), n * sizeof(int), hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->anc, anc.data(), n * sizeof(unsigned long long), hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->Xf, d->X_fixed, n * 12 * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->axis, d->axis, n * 3 * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->mass, d->mass, n * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->com, d->com, n * 3 * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(c->inertia, d->inertia, n * 6 * 8, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) return fail(WBQ_E_DEVICE);
    *out = c;
    return WBQ_SUCCESS;
}

int wbq_rbd_set_stream(wbq_rbd_ctx *c, void *hip_stream)
{
    if (!c) return WBQ_E_INVALID;
    c->stream = hip_stream == WBQ_NULL_STREAM ? (hipStream_t)0 : hip_stream ? (hipStream_t)hip_stream : c->own_stream;
    return WBQ_SUCCESS;
}

int wbq_rbd_compute(wbq_rbd_ctx *c, int B, const double *q, const double *qd, double *M, double *h, double *J,
                    double *pose, int memory)
{
    return wbq_rbd_compute_ex(c, B, q, qd, M, h, J, pose, nullptr, memory);
}

int wbq_rbd_compute_ex(wbq_rbd_ctx *c, int B, const double *q, const double *qd, double *M, double *h, double *J,
                       double *pose, double *jdqd, int memory)
{
    if (!c) return WBQ_E_INVALID;
    if (B < 0 || B > c->max_batch) return WBQ_E_CAPACITY;
    if (B == 0) return WBQ_SUCCESS;
    if (!q || !qd) return WBQ_E_INVALID;
    if (memory != WBQ_MEM_DEVICE && memory != WBQ_MEM_HOST) return WBQ_E_INVALID;
    if (hipSetDevice(c->device) != hipSuccess) return WBQ_E_DEVICE;
    const size_t n = (size_t)c->n, T = (size_t)c->ntasks, Bs = (size_t)B;
    if (memory == WBQ_MEM_DEVICE)
        return wbq::rbd_launch_split(c, B, q, qd, M, h, c->ntasks, J, pose, jdqd, nullptr, nullptr, nullptr,
                                     c->stream) == hipSuccess ? WBQ_SUCCESS : WBQ_E_DEVICE;
    double *dq = c->stage, *dqd = dq + Bs * n, *dM = dqd + Bs * n, *dh = dM + Bs * n * n, *dJ = dh + Bs * n,
           *dp = dJ + Bs * T * 6 * n, *dd = dp + Bs * T * 12;
    bool ok = hipMemcpyAsync(dq, q, Bs * n * 8, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
              hipMemcpyAsync(dqd, qd, Bs * n * 8, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
              wbq::rbd_launch_split(c, B, dq, dqd, M ? dM : nullptr, h ? dh : nullptr, c->ntasks, J ? dJ : nullptr,
                                    pose ? dp : nullptr, jdqd ? dd : nullptr, nullptr, nullptr, nullptr,
                                    c->stream) == hipSuccess;
    if (ok && M) ok = hipMemcpyAsync(M, dM, Bs * n * n * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
    if (ok && h) ok = hipMemcpyAsync(h, dh, Bs * n * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
    if (ok && J) ok = hipMemcpyAsync(J, dJ, Bs * T * 6 * n * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
    if (ok && pose) ok = hipMemcpyAsync(pose, dp, Bs * T * 12 * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
    if (ok && jdqd) ok = hipMemcpyAsync(jdqd, dd, Bs * T * 6 * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
    if (ok) ok = hipStreamSynchronize(c->stream) == hipSuccess;
    return ok ? WBQ_SUCCESS : WBQ_E_DEVICE;
}

void wbq_rbd_destroy(wbq_rbd_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (void *p : {(void *)c->parent, (void *)c->depth, (void *)c->anc, (void *)c->Xf, (void *)c->axis,
                    (void *)c->mass, (void *)c->com, (void *)c->inertia, (void *)c->stage, (void *)c->jtype,
                    (void *)c->toff})
        if (p) (void)hipFree(p);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

}  // extern "C"
