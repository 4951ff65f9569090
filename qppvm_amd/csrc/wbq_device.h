// wbq_device.h -- device helpers shared by the QPPVM and contact-form kernels (gfx950, fp64).
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>

namespace wbq {

constexpr double kInf = 1.0e300;

// |v| of a finite bound, 0 for an unbounded side (+-kInf): tolerances scale with finite bounds only
__device__ __forceinline__ double fin_abs(double v) { return fabs(v) < 1.0e299 ? fabs(v) : 0.0; }

// Phase stamps for the diagnostic build only (never compiled into the product library).
#ifdef WBQ_STAMPS
#define WBQ_STAMP(k)                                                                    \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                     \
        __builtin_amdgcn_sched_barrier(0);                                              \
        if (threadIdx.x == 0 && a.stamps) a.stamps[blockIdx.x * kStamps + (k)] = t_;    \
    } while (0)
// the constant 100 MHz clock, synchronised across XCDs (s_memtime is per-XCD)
#define WBQ_RTSTAMP(k)                                                                  \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                 \
        __builtin_amdgcn_sched_barrier(0);                                              \
        if (threadIdx.x == 0 && a.stamps) a.stamps[blockIdx.x * kStamps + (k)] = t_;    \
    } while (0)
// lap counters: cycles of a loop's phases summed over its iterations (WBQ_LAP_INIT, WBQ_LAP(k) ends
// phase k, WBQ_LAP_ADD(k, v) adds a count), added to stamp slot k by WBQ_LAP_FLUSH (slots cleared by
// wbq_diag_stamps_clear)
#define WBQ_LAP_INIT                                                                    \
    unsigned long long lap_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, lap_cnt_[2] = {0, 0};     \
    unsigned long long lap_t_ = __builtin_amdgcn_s_memtime()
#define WBQ_LAP(k)                                                                      \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                     \
        __builtin_amdgcn_sched_barrier(0);                                              \
        lap_acc_[k] += t_ - lap_t_;                                                     \
        lap_t_ = t_;                                                                    \
    } while (0)
#define WBQ_LAP_ADD(k, v) (lap_cnt_[k] += (v))
#define WBQ_LAP_FLUSH(base, cbase)                                                      \
    do {                                                                                \
        if (threadIdx.x == 0 && a.stamps) {                                             \
            for (int k_ = 0; k_ < 8; ++k_) a.stamps[blockIdx.x * kStamps + (base) + k_] += lap_acc_[k_]; \
            for (int k_ = 0; k_ < 2; ++k_) a.stamps[blockIdx.x * kStamps + (cbase) + k_] += lap_cnt_[k_]; \
        }                                                                               \
    } while (0)
#else
#define WBQ_STAMP(k) do {} while (0)
#define WBQ_RTSTAMP(k) do {} while (0)
#define WBQ_LAP_INIT do {} while (0)
#define WBQ_LAP(k) do {} while (0)
#define WBQ_LAP_ADD(k, v) do {} while (0)
#define WBQ_LAP_FLUSH(base, cbase) do {} while (0)
#endif

// Workgroup barrier that orders LDS only. __syncthreads() is a workgroup fence on every
// address space, so it drains this wave's outstanding global loads (vmcnt(0)) before the
// barrier; with the fence narrowed to LDS ("local") the barrier waits for lgkmcnt only and
// loads issued before it stay in flight (the stage's M rows stream in behind the forces).
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Ordering of LDS accesses inside one-wave workgroups (round 6; every kernel of this library is one wave per
// workgroup): the LDS unit executes one wave's DS instructions in issue order, so a lane's write is seen by another
// lane's later read without a workgroup barrier, and only the compiler must keep the order. __syncthreads() also
// waits for every outstanding memory access (s_waitcnt vmcnt(0) lgkmcnt(0)). WBQ_WAVE_SYNC = 0: __syncthreads()
// (A/B). Used by block_gj and the contact-form / W1 = M kernels' LDS hand-offs.
#ifndef WBQ_WAVE_SYNC
#define WBQ_WAVE_SYNC 1
#endif
__device__ __forceinline__ void wave_sync()
{
#if WBQ_WAVE_SYNC
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
#else
    __syncthreads();
#endif
}

// fast reciprocal / reciprocal square root: hardware estimate + one Newton step (~0.5 ulp)
__device__ __forceinline__ double frcp(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double frsq(double x)
{
    double y = __builtin_amdgcn_rsq(x);
    return y * fma(-0.5 * x * y, y, 1.5);
}

// Raw buffer loads: one 32-bit per-lane byte offset + a uniform SGPR offset per load, so an
// unrolled run of loads costs no address VGPRs (a flat load would need a 64-bit address each).
// Out-of-range offsets read 0 (hardware bounds check on num_records).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const double *p, long elems)
{
    const long bytes = elems * 8;
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                             0x00020000);
}
// A value every lane holds alike, moved to SGPRs (v_readfirstlane) so that what is built
// from it (a buffer resource) is wave-uniform.
__device__ __forceinline__ long uniform_long(long v)
{
    const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xffffffffL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (long)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
}

// Resource over instances [b0, B) of a field with `per` elements per instance. b0 is the
// first instance of the wave (wave-uniform, so the descriptor stays in SGPRs): the 32-bit
// per-lane byte offsets then only span the instances of one wave, never the whole batch, so
// no batch size reaches the 2^31-byte offset limit.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_at(const double *p, long b0, long B, long per)
{
    return rsrc(p + b0 * per, (B - b0) * per);
}
__device__ __forceinline__ double bload(__amdgpu_buffer_rsrc_t r, int voff_bytes, int soff_bytes)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff_bytes, soff_bytes, 0));
}

// One row of an NP-column matrix per lane: in VGPRs (compile-time indices, runtime
// writes by select) or in LDS.
template <int NP, bool REG>
struct RowStore;

template <int NP>
struct RowStore<NP, true> {
    double v[NP];
    __device__ void bind(double *, bool = true) {}
    __device__ void zero()
    {
#pragma unroll
        for (int j = 0; j < NP; ++j) v[j] = 0.0;
    }
    __device__ void set(int c, double x)
    {
#pragma unroll
        for (int j = 0; j < NP; ++j) v[j] = (j == c) ? x : v[j];
    }
    __device__ double get(int c) const
    {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < NP; ++j) r = (j == c) ? v[j] : r;
        return r;
    }
    __device__ double at(int c) const { return v[c]; } // c static (after unrolling)
    __device__ double dot(const double *b, int cnt) const
    {
        double s[4] = {0.0, 0.0, 0.0, 0.0}; // four accumulators: a shorter dependent chain
#pragma unroll
        for (int j = 0; j < NP; ++j)
            if (j < cnt) s[j & 3] = fma(v[j], b[j], s[j & 3]);
        return (s[0] + s[1]) + (s[2] + s[3]);
    }
    // (the full row, LDS reads a chunk ahead: rdotp below)
    __device__ double dotp(const double *b) const;
};

template <int NP>
struct RowStore<NP, false> {
    double *row;
    bool live = true; // false: a lane past the layout's rows, bound to a zero row: reads 0, writes nothing
    __device__ void bind(double *p, bool lv = true)
    {
        row = p;
        live = lv;
    }
    __device__ void zero()
    {
        if (live)
            for (int j = 0; j < NP; ++j) row[j] = 0.0;
    }
    __device__ void set(int c, double x)
    {
        if (live) row[c] = x;
    }
    __device__ double get(int c) const { return row[c]; }
    __device__ double at(int c) const { return row[c]; }
    // chunks of 8 independent LDS reads into four accumulators instead of a chain of cnt dependent
    // LDS round trips. Entries past cnt (up to NP) are read and masked.
    __device__ double dot(const double *b, int cnt) const
    {
        double s[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j0 = 0; j0 < cnt; j0 += 8) {
            double rv[8], bv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                rv[u] = j0 + u < NP ? row[j0 + u] : 0.0;
                bv[u] = j0 + u < NP ? b[j0 + u] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) s[u & 3] = fma(j0 + u < cnt ? rv[u] : 0.0, j0 + u < cnt ? bv[u] : 0.0, s[u & 3]);
        }
        return (s[0] + s[1]) + (s[2] + s[3]);
    }
    __device__ double dotp(const double *b) const { return dot(b, NP); }
};

// Dot product of two N-vectors (LDS or registers) with four independent accumulators: the
// 32-long chains of dependent DP FMAs of the per-lane dots were latency on the critical path.
template <int N>
__device__ __forceinline__ double dot4(const double *a, const double *b)
{
    static_assert(N % 4 == 0, "dot4: N multiple of 4");
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
    for (int j = 0; j < N; j += 4) {
        s0 = fma(a[j], b[j], s0);
        s1 = fma(a[j + 1], b[j + 1], s1);
        s2 = fma(a[j + 2], b[j + 2], s2);
        s3 = fma(a[j + 3], b[j + 3], s3);
    }
    return (s0 + s1) + (s2 + s3);
}
// same with a stride on the first operand (a column of a row-major LDS matrix)
template <int N>
__device__ __forceinline__ double dot4s(const double *a, int stride, const double *b)
{
    static_assert(N % 4 == 0, "dot4s: N multiple of 4");
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
    for (int j = 0; j < N; j += 4) {
        s0 = fma(a[j * stride], b[j], s0);
        s1 = fma(a[(j + 1) * stride], b[j + 1], s1);
        s2 = fma(a[(j + 2) * stride], b[j + 2], s2);
        s3 = fma(a[(j + 3) * stride], b[j + 3], s3);
    }
    return (s0 + s1) + (s2 + s3);
}

// The same dot products with every LDS read issued a chunk (CH elements) ahead of the FMAs that use it (round
// 6): inside the dual active-set loop, at the 256-VGPR cap, the compiler's own schedule read two elements and
// waited (lgkmcnt(0)) before the next two -- ~16 dependent LDS round trips per dot, which set the step time of
// the waves that run the loop long after the others have finished. Two chunks are in
// registers at a time (4 CH doubles per operand pair; CH = 8 spilled the fast kernel that inlines the loop).
template <int N, int CH = 4>
__device__ __forceinline__ double dot4p(const double *a, const double *b)
{
    static_assert(N % CH == 0 && CH % 4 == 0, "dot4p: N, CH");
    constexpr int NCH = N / CH;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    double av[2][CH], bv[2][CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        av[0][u] = a[u];
        bv[0][u] = b[u];
    }
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        if (ch + 1 < NCH) {
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                av[(ch + 1) & 1][u] = a[(ch + 1) * CH + u];
                bv[(ch + 1) & 1][u] = b[(ch + 1) * CH + u];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) s[u & 3] = fma(av[ch & 1][u], bv[ch & 1][u], s[u & 3]);
        __builtin_amdgcn_sched_barrier(0);
    }
    return (s[0] + s[1]) + (s[2] + s[3]);
}
// a strided (a column of a row-major LDS matrix)
template <int N, int CH = 4>
__device__ __forceinline__ double dot4sp(const double *a, int stride, const double *b)
{
    static_assert(N % CH == 0 && CH % 4 == 0, "dot4sp: N, CH");
    constexpr int NCH = N / CH;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    double av[2][CH], bv[2][CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
        av[0][u] = a[u * stride];
        bv[0][u] = b[u];
    }
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        if (ch + 1 < NCH) {
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                av[(ch + 1) & 1][u] = a[((ch + 1) * CH + u) * stride];
                bv[(ch + 1) & 1][u] = b[(ch + 1) * CH + u];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) s[u & 3] = fma(av[ch & 1][u], bv[ch & 1][u], s[u & 3]);
        __builtin_amdgcn_sched_barrier(0);
    }
    return (s[0] + s[1]) + (s[2] + s[3]);
}
// a register vector (compile-time indices) times an LDS vector
template <int N, int CH = 4>
__device__ __forceinline__ double rdotp(const double (&v)[N], const double *b)
{
    static_assert(N % CH == 0 && CH % 4 == 0, "rdotp: N, CH");
    constexpr int NCH = N / CH;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    double bv[2][CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) bv[0][u] = b[u];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        if (ch + 1 < NCH) {
#pragma unroll
            for (int u = 0; u < CH; ++u) bv[(ch + 1) & 1][u] = b[(ch + 1) * CH + u];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < CH; ++u) s[u & 3] = fma(v[ch * CH + u], bv[ch & 1][u], s[u & 3]);
        __builtin_amdgcn_sched_barrier(0);
    }
    return (s[0] + s[1]) + (s[2] + s[3]);
}

template <int NP>
__device__ __forceinline__ double RowStore<NP, true>::dotp(const double *b) const
{
    return rdotp<NP>(v, b);
}

// ---------------------------------------------------------------- reductions inside an instance
// NP = 32: lanes [0, 32) and [32, 64) of the wave are two instances; NP = 64: one. The moves inside a
// 16-lane row are DPP (quad_perm xor 1, xor 2, row_half_mirror, row_mirror: a VALU operand modifier,
// ~no latency), the four row partials are then combined from v_readlane (SGPR) values. With
// __shfl_xor every stage was a pair of ds_bpermute round trips through the LDS unit waited for one by
// one: a level-0 BVLS step of the config-4 repair (27 sums of 6 x 6 Grams and right-hand sides, the
// argmin and the KKT max) measured ~20k cycles (scripts/diag_mpc_repair.py). Each stage pairs lanes
// by an involution and a pair computes a + b and b + a, so every lane of an instance ends with the
// same bits. Callers run them with every lane of the wave active (values masked, not branched on).
// (Measured and not kept: combining the rows with gfx950's v_permlane16/32_swap instead of v_readlane
// broke every contact-form variant whose dual loop reduces under a lane mask -- the swap moves active
// lanes only -- while v_readlane reads the row's partial whatever the mask.)
// The reductions read the four row partials with v_readlane whatever EXEC holds: a call under a lane
// mask would read stale partials of inactive lanes. Builds with -DWBQ_EXEC_CHECK check the
// precondition at every reduction and report a violation (printf from the first active lane; no
// trap: a fault can take the whole GPU down); the product build does not. (Not part of the stamp build:
// the printf at every reduction made a stamped qppvm unit take ~25 min to compile.)
// With NP = 32 a reduction reads only its own instance's half of the wave, so a mask that keeps each
// half whole (an instance-uniform branch) is fine; NP = 64 (and the contact kernel's 64-lane
// reductions) need every lane.
#ifdef WBQ_EXEC_CHECK
#define WBQ_FULL_EXEC_NP(NP_)                                                           \
    do {                                                                                \
        const unsigned long long ex_ = __builtin_amdgcn_read_exec();                    \
        const unsigned lo_ = (unsigned)ex_, hi_ = (unsigned)(ex_ >> 32);                 \
        const bool ok_ = (NP_) == 32 ? ((lo_ == 0u || lo_ == ~0u) && (hi_ == 0u || hi_ == ~0u)) \
                                     : ex_ == ~0ull;                                    \
        if (!ok_ && (int)(threadIdx.x & 63) == __builtin_ctzll(ex_))                     \
            printf("wbq: reduction under a lane mask (exec %llx) in block %d at %s:%d\n", \
                   ex_, (int)blockIdx.x, __FILE__, __LINE__);                            \
    } while (0)
#else
#define WBQ_FULL_EXEC_NP(NP_) do {} while (0)
#endif
#define WBQ_FULL_EXEC() WBQ_FULL_EXEC_NP(64)

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned long long)(unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ double lane_f64(double v, int lane)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | (unsigned long long)lo);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

template <int NP>
__device__ __forceinline__ double isum(double v)
{
    static_assert(NP == 32 || NP == 64, "isum: NP");
    WBQ_FULL_EXEC_NP(NP);
    v += dpp_f64<kDppXor1>(v);
    v += dpp_f64<kDppXor2>(v);
    v += dpp_f64<kDppHalfMirror>(v);
    v += dpp_f64<kDppMirror>(v);
    const double r0 = lane_f64(v, 0), r1 = lane_f64(v, 16), r2 = lane_f64(v, 32), r3 = lane_f64(v, 48);
    if constexpr (NP == 32) return (threadIdx.x & 32) ? r2 + r3 : r0 + r1;
    else return (r0 + r1) + (r2 + r3);
}

template <int NP>
__device__ __forceinline__ double imax(double v)
{
    static_assert(NP == 32 || NP == 64, "imax: NP");
    WBQ_FULL_EXEC_NP(NP);
    v = fmax(v, dpp_f64<kDppXor1>(v));
    v = fmax(v, dpp_f64<kDppXor2>(v));
    v = fmax(v, dpp_f64<kDppHalfMirror>(v));
    v = fmax(v, dpp_f64<kDppMirror>(v));
    const double r0 = lane_f64(v, 0), r1 = lane_f64(v, 16), r2 = lane_f64(v, 32), r3 = lane_f64(v, 48);
    if constexpr (NP == 32) return (threadIdx.x & 32) ? fmax(r2, r3) : fmax(r0, r1);
    else return fmax(fmax(r0, r1), fmax(r2, r3));
}

// (value, index) reductions inside an instance; ties -> lowest index (a total order, so the tree shape
// does not change the winner)
template <bool MAX>
__device__ __forceinline__ void arg_take(double &v, int &idx, double ov, int oi)
{
    if ((MAX ? ov > v : ov < v) || (ov == v && oi < idx)) {
        v = ov;
        idx = oi;
    }
}
template <int CTRL, bool MAX>
__device__ __forceinline__ void arg_stage(double &v, int &idx)
{
    const double ov = dpp_f64<CTRL>(v);
    const int oi = dpp_i32<CTRL>(idx);
    arg_take<MAX>(v, idx, ov, oi);
}
template <int NP, bool MAX>
__device__ __forceinline__ void iarg(double &v, int &idx)
{
    static_assert(NP == 32 || NP == 64, "iarg: NP");
    WBQ_FULL_EXEC_NP(NP);
    arg_stage<kDppXor1, MAX>(v, idx);
    arg_stage<kDppXor2, MAX>(v, idx);
    arg_stage<kDppHalfMirror, MAX>(v, idx);
    arg_stage<kDppMirror, MAX>(v, idx);
    double r[4];
    int k[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r[q] = lane_f64(v, 16 * q);
        k[q] = __builtin_amdgcn_readlane(idx, 16 * q);
    }
    arg_take<MAX>(r[0], k[0], r[1], k[1]);
    arg_take<MAX>(r[2], k[2], r[3], k[3]);
    if constexpr (NP == 32) {
        const bool hi = threadIdx.x & 32;
        v = hi ? r[2] : r[0];
        idx = hi ? k[2] : k[0];
    } else {
        arg_take<MAX>(r[0], k[0], r[2], k[2]);
        v = r[0];
        idx = k[0];
    }
}
template <int NP>
__device__ __forceinline__ void iargmax(double &v, int &idx) { iarg<NP, true>(v, idx); }
template <int NP>
__device__ __forceinline__ void iargmin(double &v, int &idx) { iarg<NP, false>(v, idx); }

// K sums at once (the stages of all K interleave)
template <int NP, int K>
__device__ __forceinline__ void isum_vec(double (&v)[K])
{
    static_assert(NP == 32 || NP == 64, "isum_vec: NP");
    WBQ_FULL_EXEC_NP(NP);
#pragma unroll
    for (int c = 0; c < K; ++c) v[c] += dpp_f64<kDppXor1>(v[c]);
#pragma unroll
    for (int c = 0; c < K; ++c) v[c] += dpp_f64<kDppXor2>(v[c]);
#pragma unroll
    for (int c = 0; c < K; ++c) v[c] += dpp_f64<kDppHalfMirror>(v[c]);
#pragma unroll
    for (int c = 0; c < K; ++c) v[c] += dpp_f64<kDppMirror>(v[c]);
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const double r0 = lane_f64(v[c], 0), r1 = lane_f64(v[c], 16), r2 = lane_f64(v[c], 32), r3 = lane_f64(v[c], 48);
        if constexpr (NP == 32) v[c] = (threadIdx.x & 32) ? r2 + r3 : r0 + r1;
        else v[c] = (r0 + r1) + (r2 + r3);
    }
}

// Cartesian error component r of e = [p_ref - p ; vec(quat(R_ref R^T)), w >= 0]
// (same specification as oracle/wbq_oracle.c:wbq_ref_cart_error).
__device__ double cart_error_component(const double *P, const double *Pr, int r)
{
    if (r < 3) return Pr[4 * r + 3] - P[4 * r + 3];
    double Re[9];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            Re[3 * a + c] = Pr[4 * a] * P[4 * c] + Pr[4 * a + 1] * P[4 * c + 1] + Pr[4 * a + 2] * P[4 * c + 2];
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
    return sg * (r == 3 ? qx : (r == 4 ? qy : qz));
}

// In-place block Gauss-Jordan on an SPD matrix held one row per lane (A = row i), with NR
// right-hand sides per row; returns true if a pivot was not positive (M not SPD). On exit
// rhs = M^-1 rhs (row i). PN: LDS [2][NP][4] panel, RH: LDS [2][4][RHS] pivot-row rhs.
//
// Gauss-Jordan pivot block rows (panel: 2 x NP x kGjBS doubles). Measured: 2 and 4
// rows within 0.5 %, 8 rows 28 % slower (the 8 x 8 pivot Cholesky chain and its registers)
constexpr int kGjBS = 4;

// Trailing-update read schedule (round 5): the panel entries of CH columns are read a chunk ahead of
// their FMAs (two chunks in registers). The compiler's own schedule kept one ds_read_b128 in flight and
// waited for it before the next: the elimination ran at the LDS latency (a lone wave's 8 steps took 16k
// cycles). 0 = the compiler's schedule.
#ifndef WBQ_GJ_CH
#define WBQ_GJ_CH 0
#endif
// One update form for every row (round 5): row_i += hh . row_P with hh = D^-1 e_ri - e_ri for the
// pivot block's own rows (row_i - row_P[ri] + (D^-1 row_P)[ri], the normalised pivot row to roundoff)
// and hh = -D^-1 a_i elsewhere, instead of cc * row_i with cc = 0 / 1: one v_mul_f64 less per column
// and step. 0 = the cc form.
#ifndef WBQ_GJ_UNI
#define WBQ_GJ_UNI 0
#endif

// Pivot blocks of BS = 4 rows. M is SPD, so no pivoting is needed and the trailing Schur
// complement stays symmetric: pivot row k+r, column j, equals lane j's entry in column k+r.
// Every lane publishes its BS panel entries; every lane factors the BS x BS pivot block D
// redundantly and applies one rank-BS update:
//   rows outside the block: row -= (a_i D^-1) P,   rows inside: row = (D^-1)_ri P,
// so each row ends up normalised by its own pivot block (x_i = rhs_i, no division).
// The next panel is updated and published first (lookahead), then the rest of the row.
// NC (a multiple of BS, n <= NC <= NP): the columns held per lane. Lanes i >= NC and columns past
// NC are identity / zero and never pivoted, so an instantiation for n <= 40 in 64 lanes carries
// 40 columns instead of 64 (the n = 39 fast kernel: 48 fewer VGPRs, 40 % less update work).
template <int NP, int NR, int RHS, int NC = NP, int CH = WBQ_GJ_CH, bool UNI = (WBQ_GJ_UNI != 0)>
__device__ __forceinline__ bool block_gj(double (&A)[NC], double (&rhs)[NR], int n, int i, double *PN, double *RH)
{
    static_assert(NC % kGjBS == 0 && NC <= NP, "block_gj: NC");
    constexpr int BS = kGjBS;
    bool notspd = false;
    if (i < NP) {
#pragma unroll
        for (int c = 0; c < BS; ++c) PN[i * BS + c] = A[c];
    }
    if (i < BS) {
#pragma unroll
        for (int m = 0; m < NR; ++m) RH[i * RHS + m] = rhs[m];
    }
#pragma unroll
    for (int kb = 0; kb < NC / BS; ++kb) {
        const int k = kb * BS;
        if (k < n) {
            wave_sync();
            const double *pn = PN + (kb & 1) * NP * BS;
            const double *rh = RH + (kb & 1) * BS * RHS;
            double *pnn = PN + ((kb + 1) & 1) * NP * BS;
            double *rhn = RH + ((kb + 1) & 1) * BS * RHS;
            // Cholesky of the pivot block (redundant per lane)
            double d[BS][BS];
#pragma unroll
            for (int r = 0; r < BS; ++r)
#pragma unroll
                for (int c = 0; c <= r; ++c) d[r][c] = pn[(k + r) * BS + c];
            double la[BS][BS]; // (CH > 0) the lookahead panel, read with the pivot block
            if constexpr (CH > 0) {
#pragma unroll
                for (int u = 0; u < BS; ++u)
#pragma unroll
                    for (int c = 0; c < BS; ++c) la[u][c] = (k + BS + u < NC) ? pn[(k + BS + u) * BS + c] : 0.0;
            }
            double il[BS];
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                double dd = d[c][c];
#pragma unroll
                for (int q_ = 0; q_ < c; ++q_) dd = fma(-d[c][q_], d[c][q_], dd);
                notspd |= !(dd > 0.0);
                il[c] = frsq(dd);
#pragma unroll
                for (int r = c + 1; r < BS; ++r) {
                    double t = d[r][c];
#pragma unroll
                    for (int q_ = 0; q_ < c; ++q_) t = fma(-d[r][q_], d[c][q_], t);
                    d[r][c] = t * il[c];
                }
            }
            // solve D y = e, e = unit(i-k) for the block's own rows, else a_i = row i's panel
            const int ri = i - k;
            const bool inK = ri >= 0 && ri < BS;
            double y[BS];
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                double v = inK ? (ri == c ? 1.0 : 0.0) : A[k + c];
#pragma unroll
                for (int q_ = 0; q_ < c; ++q_) v = fma(-d[c][q_], y[q_], v);
                y[c] = v * il[c];
            }
#pragma unroll
            for (int c = BS - 1; c >= 0; --c) {
                double v = y[c];
#pragma unroll
                for (int q_ = c + 1; q_ < BS; ++q_) v = fma(-d[q_][c], y[q_], v);
                y[c] = v * il[c];
            }
            const double cc = inK ? 0.0 : 1.0;
            double hh[BS];
#pragma unroll
            for (int c = 0; c < BS; ++c) hh[c] = UNI ? (inK ? y[c] - (ri == c ? 1.0 : 0.0) : -y[c]) : (inK ? y[c] : -y[c]);
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                double v = UNI ? rhs[m] : cc * rhs[m];
#pragma unroll
                for (int c = 0; c < BS; ++c) v = fma(hh[c], rh[c * RHS + m], v);
                rhs[m] = v;
            }
            // lookahead: next panel first
#pragma unroll
            for (int j = k + BS; j < k + 2 * BS && j < NC; ++j) {
                double v = UNI ? A[j] : cc * A[j];
#pragma unroll
                for (int c = 0; c < BS; ++c) v = fma(hh[c], CH > 0 ? la[j - k - BS][c] : pn[j * BS + c], v);
                A[j] = v;
            }
            if (k + BS < n) {
                if (i < NP) {
#pragma unroll
                    for (int c = 0; c < BS; ++c)
                        if (k + BS + c < NC) pnn[i * BS + c] = A[(k + BS + c) < NC ? k + BS + c : NC - 1];
                }
                const int rn = i - (k + BS);
                if (rn >= 0 && rn < BS) {
#pragma unroll
                    for (int m = 0; m < NR; ++m) rhn[rn * RHS + m] = rhs[m];
                }
            }
            if constexpr (CH == 0) {
#pragma unroll
                for (int j = k + 2 * BS; j < NC; ++j) {
                    double v = UNI ? A[j] : cc * A[j];
#pragma unroll
                    for (int c = 0; c < BS; ++c) v = fma(hh[c], pn[j * BS + c], v);
                    A[j] = v;
                }
            } else {
                // trailing columns in chunks of CH: the next chunk's reads issue before this chunk's FMAs
                constexpr int NCH = (NC + CH - 1) / CH;
                double pv[2][CH][BS];
#pragma unroll
                for (int ch = 0; ch <= NCH; ++ch) {
                    const int j0 = k + 2 * BS + ch * CH;
                    if (ch < NCH && j0 < NC) {
#pragma unroll
                        for (int u = 0; u < CH; ++u)
#pragma unroll
                            for (int c = 0; c < BS; ++c) pv[ch & 1][u][c] = (j0 + u < NC) ? pn[(j0 + u) * BS + c] : 0.0;
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    const int jp = j0 - CH;
                    if (ch > 0 && jp < NC) {
#pragma unroll
                        for (int u = 0; u < CH; ++u) {
                            const int j = jp + u;
                            if (j < NC) {
                                double v = UNI ? A[j] : cc * A[j];
#pragma unroll
                                for (int c = 0; c < BS; ++c) v = fma(hh[c], pv[(ch - 1) & 1][u][c], v);
                                A[j] = v;
                            }
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    }
    return notspd;
}

}  // namespace wbq
