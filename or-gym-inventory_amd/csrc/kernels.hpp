// Kernel parameter blocks and launcher declarations (host <-> device contract).
//
// HBM layout: every per-env field is Structure-of-Arrays, row r of a field
// lives at  base + r * Npad + env  (Npad = N rounded up to 256), so a wave's
// 64 lanes touch 64 consecutive elements of one row: fully coalesced.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "group_rng.hpp"
#include "numpy_dists.hpp"

namespace invsim {

enum { AR_NEXT_STEP = 0, AR_SAME_STEP = 1, AR_DISABLED = 2 };

// Profiling-only per-wave phase timestamps (`make timing`; never in the shipped
// library): lane 0 of wave b writes s_memrealtime (100 MHz) for probe i to
// g_tbuf[b][i]; probe 7 holds (XCC_ID << 32) | HW_ID.
#ifdef INVSIM_TIMING
constexpr int TB_WAVES = 8192, TB_PROBES = 8;   // probe 7: hardware ids
#define TPROBE(i)                                                                              \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.x < TB_WAVES)                                         \
            g_tbuf[blockIdx.x * TB_PROBES + (i)] = __builtin_amdgcn_s_memrealtime();           \
    } while (0)
#define TPROBE_ID()                                                                            \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.x < TB_WAVES)                                         \
            g_tbuf[blockIdx.x * TB_PROBES + 7] =                                               \
                ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |                 \
                (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);                           \
    } while (0)
#define TPROBE_AT(i, tid)                                                                      \
    do {                                                                                       \
        if (threadIdx.x == (tid) && blockIdx.x < TB_WAVES)                                     \
            g_tbuf[blockIdx.x * TB_PROBES + (i)] = __builtin_amdgcn_s_memrealtime();           \
    } while (0)
// per wave of a multi-wave workgroup: row blockIdx.x * waves + wave, lane 0
#define TPROBE_W(i)                                                                            \
    do {                                                                                       \
        const unsigned tw_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                \
        if ((threadIdx.x & 63) == 0 && tw_ < (unsigned)TB_WAVES)                               \
            g_tbuf[tw_ * TB_PROBES + (i)] = __builtin_amdgcn_s_memrealtime();                  \
    } while (0)
#define TPROBE_W_ID()                                                                          \
    do {                                                                                       \
        const unsigned tw_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                \
        if ((threadIdx.x & 63) == 0 && tw_ < (unsigned)TB_WAVES) {                             \
            g_tbuf[tw_ * TB_PROBES + 7] =                                                      \
                ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |                 \
                (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);                           \
            g_tbar[tw_] = 0;                                                                   \
            g_ttrip[tw_] = 0;                                                                  \
        }                                                                                      \
    } while (0)
// accumulated barrier wait of each wave (the rollout kernels' workgroup
// syncs): g_tbar[wave row] (100 MHz ticks), zeroed by TPROBE_W_ID at entry
static __device__ uint64_t g_tbar[TB_WAVES];
#define TBAR_T0() const uint64_t tb0_ = __builtin_amdgcn_s_memrealtime()
#define TBAR_ADD()                                                                             \
    do {                                                                                       \
        const unsigned tw_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                \
        if ((threadIdx.x & 63) == 0 && tw_ < (unsigned)TB_WAVES)                               \
            g_tbar[tw_] += __builtin_amdgcn_s_memrealtime() - tb0_;                            \
    } while (0)
// loop trips of each wave (wave-uniform counts added by lane 0), zeroed with g_tbar
static __device__ uint32_t g_ttrip[TB_WAVES];
#define TTRIP_ADD(n)                                                                           \
    do {                                                                                       \
        const unsigned tw_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                \
        if ((threadIdx.x & 63) == 0 && tw_ < (unsigned)TB_WAVES) g_ttrip[tw_] += (uint32_t)(n); \
    } while (0)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = (uint32_t)__shfl_xor((int)v, o);
        v = v > w ? v : w;
    }
    return v;
}
#define TWAIT() __builtin_amdgcn_s_waitcnt(0)
#else
#define TTRIP_ADD(n) do {} while (0)
#define TBAR_T0() do {} while (0)
#define TBAR_ADD() do {} while (0)
#define TPROBE_W(i) do {} while (0)
#define TPROBE_W_ID() do {} while (0)
#define TPROBE_AT(i, tid) do {} while (0)
#define TPROBE(i) do {} while (0)
#define TPROBE_ID() do {} while (0)
#define TWAIT() do {} while (0)
#endif

// Launch-choice switches for A/B measurements and tests (INVSIM_* environment
// variables).  capi.hip reads the environment ONCE, when a handle is created
// (read_knobs), into Common::kn; the launchers read only these fields, so a
// variable set after creation changes nothing.  Kernels ignore them.
struct Knobs {
    bool im_split = true;            // INVSIM_IM_SPLIT=0: single steps on the one-wave kernel
    bool im_la_last = false;         // INVSIM_IM_LA_LAST=1: lookahead workgroups at the end of the grid
    bool im_roll = true;             // INVSIM_IM_ROLL=0: rollouts on the one-wave kernel
    bool im_pol_roll = true;         // INVSIM_IM_POL_ROLL=0: policy rollouts on im_run_kernel
    bool im_ahead = true;            // INVSIM_IM_AHEAD=0: no demand lookahead
    int8_t im_roll3o_g2 = -1;        // INVSIM_IM_ROLL3O_G2=1 / =0: two groups per workgroup on / off
                                     //   (-1: policy rollouts only)
    bool nv_xcd = true;              // INVSIM_NV_XCD=0: lookahead workgroups adjacent, not XCD-paired
    bool nv_roll = true;             // INVSIM_NV_ROLL=0: rollouts on nv_run_kernel
    bool nv_pol_roll = true;         // INVSIM_NV_POL_ROLL=0: policy rollouts on nv_run_kernel
    bool nv_ahead = true;            // INVSIM_NV_AHEAD=0: no demand lookahead
    bool net_roll = true;            // INVSIM_NET_ROLL=0: rollouts on net_spec_kernel
    bool net_roll3 = true;           // INVSIM_NET_ROLL3=0: net_roll_kernel instead of net_roll3o_kernel
    bool net_split = true;           // INVSIM_NET_SPLIT=0: the step on the one-wave net_step1_kernel
    bool net_pol_roll = true;        // INVSIM_NET_POL_ROLL=0: ConstantOrder rollouts on net_spec_kernel
    bool net_ahead = true;           // INVSIM_NET_AHEAD=0: no demand lookahead
    bool net_generic = false;        // INVSIM_NET_GENERIC=1: the generic kernel for the built-in graphs
    int64_t im_roll3o_max_n = 32768; // INVSIM_IM_ROLL3O_MAX_N: largest batch for the 3-role rollout
    int64_t im_roll_sub = 65536;     // INVSIM_IM_ROLL_SUB: 2-role rollouts as back-to-back launches of at most this many envs (0: one launch)
    int64_t net_roll4_max_n = 16384; // INVSIM_NET_ROLL4_MAX_N: largest batch for the 4-role Net rollout (0: never)
    int64_t net_rollq_max_n = 0;     // INVSIM_NET_ROLLQ_MAX_N: largest batch for the 16-lane-row Net rollout
                                     //   (net_rollq_kernel; 0 = never, the default: measured 6 % slower than
                                     //   net_roll3o_kernel at 4 096 envs and 1.9x slower at 8 192)
};

struct Common {
    int64_t N;       // envs in this handle
    int64_t Npad;    // SoA row stride (elements)
    int32_t autoreset;
    RngSoA rng;      // PCG64 state/inc rows
    int32_t *period; // [N] step counter within the episode
    int64_t *info_demand;  // optional [N][demand_dim]
    uint32_t *status;      // sticky error word (DISABLED-mode overrun)
    uint64_t *u32buf;      // [Npad] PCG64 32-bit output buffer (has << 32 | value), or null
    void *info_rec;        // optional per-step info record (invsim_set_info_record), last step of a launch
    int32_t philox;        // demand stream: 0 numpy PCG64 (parity), 1 fast Philox (PhiloxGen)
    uint64_t ph_step;      // fast stream: the handle's launch-step counter at this launch's first step
    Knobs kn;              // host-side launch choices (read at handle creation)
    // episode sink (invsim_set_episode_sink), or null: the running return of
    // every env [N] and the per-64-env-group partials [ceil(N / 64)][4] (EpSink)
    double *ep_ret;
    double *ep_part;
};

// ---------------------------------------------------------------- episode sink
// The evaluation harness's episodic returns (benchmark_InvManagementBacklogEnv.py:
// 371, 386, 434: `episode_reward += reward` per step, appended at done) kept on
// the device.  Per env, in step order over the rows of ONE launch:
//   ret += reward; all += reward; at terminated | truncated: s += ret,
//   s2 += ret * ret, c += 1, ret = 0
// (s, s2, c, all: per-lane accumulators that start at 0 each launch).  At the
// launch's end each 64-env group g (envs 64 g .. 64 g + 63, one wave) reduces
// its lanes' four accumulators (wave_sum_f64) and lane 0 adds them to
// part[g] = [sum of returns, sum of squares, episodes, sum of rewards] -- a
// read-modify-write by the group's only owner, so no atomics and a
// deterministic result.  The fused kernels and the fold kernel
// (episode_fold_groups_kernel) run this same code, so a launch's fused sink
// equals the fold of its output rows bit for bit.
// The wave's sum of v, the same value in every lane (all 64 lanes active):
// within each 16-lane row a DPP butterfly (quad_perm xor 1, xor 2, then
// row_half_mirror and row_mirror: each pairs lanes holding partial sums of
// disjoint lane sets, and x + y == y + x exactly, so every lane of the row ends
// with the same row sum), then the four row sums read from lanes 0, 16, 32 and
// 48 and added as (r0 + r1) + (r2 + r3).  Tens of cycles of dependent VALU
// work; the first version, a six-level ds_bpermute butterfly (__shfl_xor of
// each half), made the sink cost the InvMgmt step 0.55 us (measured, 65 536
// envs), most of it that chain's LDS round trips at the dynamics wave's tail.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double wave_sum_f64(double v) {
    v += dpp_f64<0xB1>(v);     // quad_perm [1, 0, 3, 2]: lane ^ 1
    v += dpp_f64<0x4E>(v);     // quad_perm [2, 3, 0, 1]: lane ^ 2
    v += dpp_f64<0x141>(v);    // row_half_mirror: lane i <-> 7 - i within 8
    v += dpp_f64<0x140>(v);    // row_mirror: lane i <-> 15 - i within 16
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

struct EpLane {
    double r = 0.0, s = 0.0, s2 = 0.0, c = 0.0, all = 0.0;
    __device__ __forceinline__ void add(double rew, bool done) {
        r += rew;
        all += rew;
        if (done) {
            s += r;
            s2 += r * r;
            c += 1.0;
            r = 0.0;
        }
    }
};

// EpLane for the rollout kernels: the running return and the reward sum in
// registers, the three sums that change only at an episode's end in LDS (the
// owning lane's column of a [3][WAVE] block), so the sink holds 4 VGPRs
// through the launch's loop (the 2-role policy kernel sits at 256).  The same
// operations in the same order as EpLane.
struct EpLaneLds {
    static constexpr int W = 64;   // lanes (the column stride)
    double r = 0.0, all = 0.0;
    double *sl;
    __device__ __forceinline__ void init(double *base, int lane, double r0) {
        sl = base + lane;
        sl[0] = 0.0;
        sl[W] = 0.0;
        sl[2 * W] = 0.0;
        r = r0;
    }
    __device__ __forceinline__ void add(double rew, bool done) {
        r += rew;
        all += rew;
        if (done) {
            sl[0] += r;
            sl[W] += r * r;
            sl[2 * W] += 1.0;
            r = 0.0;
        }
    }
    __device__ __forceinline__ EpLane get() const {
        EpLane a;
        a.r = r;
        a.all = all;
        a.s = sl[0];
        a.s2 = sl[W];
        a.c = sl[2 * W];
        return a;
    }
};

// The group's partials, loaded early (before the launch's other work ends) so
// the read-modify-write at the end waits for nothing
struct EpPart {
    double v[4];
    __device__ __forceinline__ void load(const double *part_g) {
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = part_g[j];
    }
    // any_done: some lane of the wave folded an episode in this launch (wave-uniform);
    // without one s, s2, c are 0 in every lane and adding them changes nothing
    __device__ __forceinline__ void flush(double *part_g, const EpLane &a, bool any_done, int lane) {
        const double all = wave_sum_f64(a.all);
        double x[3] = {0.0, 0.0, 0.0};
        if (any_done) {
            x[0] = wave_sum_f64(a.s);
            x[1] = wave_sum_f64(a.s2);
            x[2] = wave_sum_f64(a.c);
        }
        if (lane == 0) {
            if (any_done) {
#pragma unroll
                for (int j = 0; j < 3; j++) part_g[j] = v[j] + x[j];
            }
            part_g[3] = v[3] + all;
        }
    }
};

// ---------------------------------------------------------------- Newsvendor
struct NvParams {
    Common cm;
    int32_t L;           // lead time
    int32_t step_limit;
    double max_inventory, max_order;
    double p_max, h_max, k_max, mu_max;
    double *par;         // [5][Npad]  price, cost, h, k, mu  (Python floats)
    const double *lgtab; // [RHS_LDS_MAX] loggam(k + 1), host (numpy's formula)
    float *pipe;         // [L][Npad]  order ring, slot = step index mod L
    // demand lookahead cache (not part of the state blob): two slots of rows
    // [state hi, state lo, next demand] x Npad (nv_step1_kernel), and the
    // episode's Poisson constants of every env, written by the launch that
    // starts a lookahead chain (mu is fixed while a chain runs)
    uint64_t *ahead;
    double *pcon;        // [6][Npad]  a, b, vr, loglam, log_invalpha, enlam
};

// ---------------------------------------------------------------- InvMgmt
constexpr int IM_MAX_M1 = 8;  // up to 9 stages
struct ImParams {
    Common cm;
    int32_t periods;
    int32_t lt_max;              // D = max lead time (obs window rows)
    int32_t dist;                // 1 poisson, 2 binomial, 3 integers, 4 geometric, 5 user_D
    NpDist nd;                   // dist 2-4 constants (numpy_dists.hpp)
    int32_t L[IM_MAX_M1];
    int32_t ring_off[IM_MAX_M1]; // first R-ring row of stage i (depth L[i])
    int64_t c[IM_MAX_M1];
    int64_t I0[IM_MAX_M1];
    double up[IM_MAX_M1 + 1], uc[IM_MAX_M1 + 1], hc[IM_MAX_M1 + 1], kc[IM_MAX_M1 + 1];
    PtrsConst pc;                // Poisson(mu) constants, host libm
    const double *rhs;           // PTRS right-hand-side table (host libm), pc.k0 .. pc.k0+pc.nk
    const double *alpha_pow;     // [periods]  alpha ** t (Python float pow)
    const int64_t *user_D;       // [periods]
    int64_t *I;                  // [M1][Npad]   on-hand inventory I[t]
    int64_t *B;                  // [M1+1][Npad] backlog B[t] (backlog mode only)
    int64_t *Rring;              // [sum L][Npad] fulfilled orders R, ring per stage
    uint32_t *alog32;            // [D][Npad][M1] requested orders (action_log) ring, 32-bit;
                                 //   IM_WIDE = the value is >= 2^32 - 1 and lives in alog
    int64_t *alog;               // [D][Npad][M1] int64 ring, written only for IM_WIDE entries
    // demand lookahead cache (dist 1-4; not part of the state blob): two slots
    // of rows [state hi, state lo, next demand, 32-bit buffer] x Npad = the env's
    // PCG64 one draw past the committed state in cm.rng, and that draw.  Valid
    // only while the host says so (invsim_handle::im_ahead, im_slot); the
    // committed state stays exact.
    uint64_t *ahead;
};

// ---------------------------------------------------------------- NetInvMgmt
struct NetParams {
    Common cm;
    int32_t J, E, RL, T, backlog, sumL;
    // topology tables (device, read with wave-uniform indices)
    const double *I0, *h, *C, *o, *v;
    const int32_t *is_factory, *is_retail;
    const int32_t *sup, *pur, *sup_is_factory, *L, *ring_off;
    const int32_t *win_off;      // [E] obs offset of link e's order window (links with L > 0)
    const double *lp, *lg;
    const int32_t *rl_node, *rl_user;
    const double *rl_p, *rl_b;
    const PtrsConst *rl_pc;      // [RL]
    const int32_t *rl_dist;      // [RL] 1 poisson, 2 binomial, 3 integers, 4 geometric (non-Poisson: generic kernel)
    const NpDist *rl_nd;         // [RL] numpy_dists constants of the non-Poisson markets
    const double *rhs;           // PTRS right-hand-side tables of all retail links (rl_pc[r].toff)
    const double *user_D;        // [RL][T]
    const int32_t *succ_ptr, *succ_kind, *succ_idx, *pred_ptr, *pred_idx;
    const double *alpha_pow;     // [T]
    // state
    double *X;                   // [J][Npad]
    double *U;                   // [RL][Npad]
    double *Y;                   // [E][Npad]
    double *Rring;               // [sumL][Npad]
    // demand lookahead cache of the specialised kernels (not part of the state
    // blob): two slots of rows [state hi, state lo, demand per retail link] x Npad
    uint64_t *ahead;
};

// Step I/O of one launch: K consecutive steps (K = 1 for invsim_step); row k
// of every output is at  base + k * N * width.
template <typename A, typename O>
struct StepIO {
    int K;
    const A *act;      // [K][N][action_dim]
    O *obs;            // [K][N][obs_dim]
    double *rew;       // [K][N]
    uint8_t *term;     // [K][N]
    uint8_t *trunc;    // [K][N]
    O *fobs;           // [N][obs_dim] final obs (SAME_STEP, K == 1), may be null
};

// Closed-loop rollouts (invsim_rollout_policy): each step's action is computed
// in the kernel from the env state by a restated heuristic agent, every output
// is optional, and per-env evaluation metrics accumulate in registers.
enum { POL_NONE = 0, POL_CONSTANT = 1, POL_BASE_STOCK = 2, POL_ORDER_UP_TO = 3, POL_CLASSIC_NV = 4,
       POL_SS = 5 };
constexpr int POL_MAX_A = 32;
struct PolicyIO {
    int32_t kind;
    int32_t mdim;             // metrics per env (0: none)
    int32_t variant;          // CLASSIC_NV: 0 'k_vs_h', 1 'profit_margin'
    int32_t pad_;
    double sf, mu;            // safety factor (SS: S_buffer_factor); BASE_STOCK demand mean
    int64_t ci[POL_MAX_A];    // CONSTANT actions, int64 action spaces
    float cf[POL_MAX_A];      // CONSTANT actions, f32 action spaces
    void *act_out;            // [K][N][action_dim] actions taken, may be null
    double *metrics;          // [N][mdim], accumulated (+=), may be null
};

// Lock-step period: when every env of the handle is at the same period the host
// knows it (t_u >= 0) and the kernels neither read nor write the per-env
// period row; t_u = -1 means "read period[e]".  Next period after one step at t
// (t >= horizon means "done": NEXT_STEP resets it this step).
__host__ __device__ inline int next_period(int t, int horizon, int autoreset, bool wrap_disabled) {
    if (t >= horizon) return (autoreset == AR_NEXT_STEP) ? 0 : t + (wrap_disabled ? 1 : 0);
    int t1 = t + 1;
    if (t1 >= horizon && autoreset == AR_SAME_STEP) return 0;
    return t1;
}

constexpr int WAVE = 64;          // one-wave workgroups: LDS obs tile stored with 16-B coalesced rows
constexpr int RHS_LDS_MAX = 512;  // PTRS RHS table entries per Poisson rate (staged in LDS)

struct LgTab {    // loggam(k + 1) for k < RHS_LDS_MAX (Newsvendor's per-episode rate; see RhsTab)
    const double *lg;
    __device__ __forceinline__ double fast(int64_t k, const PtrsConst &c, bool &ok) const {
        ok = k >= 0 && k < RHS_LDS_MAX;
        return (-c.lam + (double)k * c.loglam) - lg[ok ? (int)k : 0];
    }
    // the same for a candidate's floor value kd (ptrs_decide): no int64 -> f64 conversion
    __device__ __forceinline__ double fastd(double kd, const PtrsConst &c, bool &ok) const {
        ok = (kd >= 0.0) & (kd < (double)RHS_LDS_MAX);
        return (-c.lam + kd * c.loglam) - lg[ok ? (int)kd : 0];
    }
    __device__ __forceinline__ double exact(int64_t k, const PtrsConst &c) const {
        return -c.lam + (double)k * c.loglam - np_loggam((double)(k + 1));
    }
};
// Lanes per env.  1 = one thread per env with the sequential sampler; GRP (4) =
// the lane-group sampler of group_rng.hpp.  tools/poisson_bench.hip measured the
// sequential sampler (host RHS table + f32 pre-test) 1.1-1.6x faster than the
// group one at 65 536 - 524 288 envs on MI355X, so 1 it is.
constexpr int LPE = 1;
constexpr int EPW = WAVE / LPE;   // envs per wave

template <class G>
__device__ __forceinline__ int64_t env_poisson(G &g, const PtrsConst &c, const double *rhs) {
    if constexpr (LPE == 1) return np_poisson(g, c, rhs);
    else return np_poisson_grp(g, c, rhs);
}
template <class G>
__device__ __forceinline__ int64_t env_poisson_dyn(G &g, double lam) {
    if constexpr (LPE == 1) return np_poisson_dyn(g, lam);
    else return np_poisson_dyn_grp(g, lam);
}
template <class G>
__device__ __forceinline__ int64_t env_poisson_dyn(G &g, double lam, const double *lgtab, int lgn) {
    return np_poisson_dyn(g, lam, lgtab, lgn);
}

// Workgroups are one wave, and a wave's LDS instructions execute in issue
// order, so ordering the tile writes before other lanes' reads needs only a
// compiler barrier.  (__syncthreads() would also drain every outstanding
// global load/store: s_waitcnt vmcnt(0) before the s_barrier.)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A RHS_LDS_MAX-entry read-only table (PTRS right-hand sides / loggam) copied to
// LDS: each lane loads its NT entries early, and the LDS write happens once the
// step's other global loads are in flight (a wait for these loads would
// otherwise hold back every load issued after them: vmcnt is in order).
struct TableStage {
    static constexpr int NT = RHS_LDS_MAX / WAVE;
    double *dst;
    double v[NT];
    __device__ __forceinline__ void load(const double *src, int n, int lane) {
        const int qm = n > 0 ? n - 1 : 0;
#pragma unroll
        for (int u = 0; u < NT; u++) v[u] = src[min(lane + u * WAVE, qm)];
    }
    __device__ __forceinline__ void flush(int lane) {
#pragma unroll
        for (int u = 0; u < NT; u++) dst[lane + u * WAVE] = v[u];
        __builtin_amdgcn_wave_barrier();
    }
};

// Output-stream stores (obs rows, reward, flags) are non-temporal: the caller
// reads them in a later kernel or on the host, and streaming them past L2 leaves
// less dirty data for the end-of-kernel write-back (measured on MI355X: +7 %
// step, +15 % rollout throughput for InvMgmt).  State stores (st_store) stay
// cached unless INVSIM_NT_STATE (profiling experiment).
template <typename V>
__device__ __forceinline__ void out_store(V *p, V v) {
    __builtin_nontemporal_store(v, p);
}
template <typename V>
__device__ __forceinline__ void st_store(V *p, V v) {
#ifdef INVSIM_NT_STATE
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// Copy `count` elements of an LDS tile to global memory, 16 B per lane.
// MAXIT > 0: tiles of at most MAXIT * 64 16-B chunks are copied by straight-line
// predicated code (no loop: the compiler drains every outstanding global store,
// s_waitcnt vmcnt(0), in front of a store loop); larger tiles use the loop.
template <int MAXIT = 0, typename T>
__device__ __forceinline__ void store_tile(const T *__restrict__ tile, T *__restrict__ dst,
                                           int64_t count, int lane) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const int64_t bytes = count * (int64_t)sizeof(T);
    int64_t done = 0;
    if ((((uintptr_t)dst) & 15) == 0) {
        const int n16 = (int)(bytes >> 4);
        const v4i *s4 = reinterpret_cast<const v4i *>(tile);
        v4i *d4 = reinterpret_cast<v4i *>(dst);
        if (MAXIT > 0 && n16 <= MAXIT * WAVE) {
            constexpr int MI = MAXIT > 0 ? MAXIT : 1;
            v4i r[MI];
#pragma unroll
            for (int u = 0; u < MI; u++) {
                const int i = lane + u * WAVE;
                r[u] = s4[i < n16 ? i : n16 - 1];
            }
#pragma unroll
            for (int u = 0; u < MI; u++)
                if (lane + u * WAVE < n16) out_store(d4 + lane + u * WAVE, r[u]);
        } else {
            int i = lane;
            for (; i + 7 * WAVE < n16; i += 8 * WAVE) {   // 8 LDS reads in flight, then 8 stores
                v4i r[8];
#pragma unroll
                for (int u = 0; u < 8; u++) r[u] = s4[i + u * WAVE];
#pragma unroll
                for (int u = 0; u < 8; u++) out_store(d4 + i + u * WAVE, r[u]);
            }
            for (; i < n16; i += WAVE) out_store(d4 + i, s4[i]);
        }
        done = ((int64_t)n16 << 4) / (int64_t)sizeof(T);
        if (done + lane < count) out_store(dst + done + lane, tile[done + lane]);   // < 16 B tail
        return;
    }
    for (int64_t i = lane; i < count; i += WAVE) out_store(dst + i, tile[i]);
}

// Cross-wave LDS handoff inside a workgroup: orders LDS traffic only (an
// __syncthreads() would also drain each wave's outstanding global loads and
// stores, s_waitcnt vmcnt(0), before the s_barrier)
__device__ __forceinline__ void roll_wg_sync() {
    TBAR_T0();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    TBAR_ADD();
}

// One numpy random_poisson attempt for a fixed-rate stream: a PTRS candidate
// (lam >= 10; false = rejected, the next attempt continues the stream), or the
// whole multiplication-method draw (0 < lam < 10), or 0 (lam == 0) -- the
// branches of np_poisson, so the attempts up to the first `true` consume the
// stream exactly as one np_poisson call.
template <class G>
__device__ __forceinline__ bool np_poisson_try(G &g, const PtrsConst &c, const double *rhs, int64_t &k) {
    if (c.lam >= 10) return ptrs_candidate(g, c, RhsTab{rhs}, k);   // rhs: an LDS table (never null here)
    k = (c.lam == 0) ? 0 : np_poisson_mult(g, c.enlam);
    return true;
}

// The stream wave of a lock-step rollout kernel as a flat loop: each lane
// works through its own demand draws (launch step j, draw r of the step's RL),
// one attempt per iteration, so a PTRS rejection delays only its own lane
// instead of every draw waiting for the wave's slowest lane.  Draws go to a
// ring of RD chunks of CH launch steps (slot j mod RD*CH).  The consumer reads
// chunk c between barriers c and c + 1; the wave passes barrier b (of nb) as
// soon as every lane has drawn chunk b, and a lane may draw step j only once
// the consumer is done with the slot's previous step j - RD*CH (barrier
// (j / CH - RD) + 1 passed).  A NEXT_STEP reset step (t >= T) draws nothing.
//   draw(j, r, k) -> bool: one attempt for draw r of launch step j; put(slot, r, k): store it
// A stream wave can also stage other per-step inputs of chunk b for the
// consumer waves (stage(b), e.g. LDS-DMA loads of the actions): issued when the
// wave starts chunk b (right after barrier b - 1), waited for (stage.wait())
// before barrier b.  The stream wave issues no global stores, so that wait
// waits for nothing else; the consumers then load nothing from global memory in
// their loops, where a load would wait for their own earlier stores (vmcnt
// counts stores, and completes in order).
struct NoStage {
    __device__ __forceinline__ void operator()(int) const {}
    __device__ __forceinline__ void wait() const {}
};

template <int CH, int RD, int RL, class Draw, class Put, class Stage = NoStage>
__device__ __forceinline__ void stream_flat_loop(int K, int nb, int t, int T, Draw draw, Put put,
                                                 Stage stage = Stage()) {
    static_assert(RD >= 2, "the ring needs two chunks");
    int j = 0, r = 0, b = 0;
    stage(0);
    for (;;) {
        while (b < nb && __all(j >= min((b + 1) * CH, K))) {
            stage.wait();
            roll_wg_sync();                        // barrier b: chunk b drawn
            b++;
            stage(b);
        }
        if (b == nb) break;
        if (j < K && j / CH - RD + 2 <= b) {
            if (t >= T) {
                t = 0;
                j++;
            } else {
                int64_t kd = 0;
                if (draw(j, r, kd)) {
                    put((j % (RD * CH)), r, kd);
                    if (++r == RL) {
                        r = 0;
                        j++;
                        t++;
                    }
                }
            }
        }
    }
}

// launchers (return hipGetLastError() of the launch)
hipError_t seed_range_launch(const Common &cm, uint64_t base_lo, uint64_t base_hi, int64_t first,
                             const uint8_t *mask, hipStream_t s);
hipError_t seed_words_launch(const Common &cm, const uint32_t *words, const int32_t *nwords,
                             const uint8_t *mask, hipStream_t s);
hipError_t period_fill_launch(const Common &cm, int32_t t, hipStream_t s);
hipError_t episode_fold_launch(const double *rew, const uint8_t *term, const uint8_t *trunc, int32_t K,
                               int64_t N, double *ret, double *acc, hipStream_t s);
// the EpSink fold of K output rows into per-group partials (no atomics)
hipError_t episode_fold_groups_launch(const double *rew, const uint8_t *term, const uint8_t *trunc, int32_t K,
                                      int64_t N, double *ret, double *part, hipStream_t s);

hipError_t nv_reset_launch(const NvParams &p, const uint8_t *mask, float *obs, hipStream_t s);
// ahead / slot: the demand lookahead cache state, as for im_run_launch
hipError_t nv_run_launch(const NvParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                         bool &ahead, int &slot, hipStream_t s);
hipError_t nv_commit_launch(const NvParams &p, int slot, hipStream_t s);
// the fast-stream (cm.philox) kernels, newsvendor_ph.hip (demand-only lookahead cache)
hipError_t nv_run_launch_ph(const NvParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                            bool &ahead, int &slot, hipStream_t s);

hipError_t im_reset_launch(const ImParams &p, int M1, bool backlog, const uint8_t *mask,
                           int64_t *obs, hipStream_t s);
// ahead: in = lookahead slot `slot` holds every env's next demand; out = the
// slot (updated) does now
// sunk: out = the launched kernel folded its rows into the episode sink
// (Common::ep_ret), or had nothing to fold; else the caller folds the outputs
hipError_t im_run_launch(const ImParams &p, int M1, bool backlog, int t_u, const PolicyIO *pol,
                         const StepIO<int64_t, int64_t> &io, bool &ahead, int &slot, bool &sunk, hipStream_t s);
// the fast-stream (cm.philox) kernels, invmgmt_ph.hip; ahead / slot: the
// fast stream's demand-only lookahead cache (never committed: it holds no state)
hipError_t im_run_launch_ph(const ImParams &p, int M1, bool backlog, int t_u, const PolicyIO *pol,
                            const StepIO<int64_t, int64_t> &io, bool &ahead, int &slot, bool &sunk, hipStream_t s);
// cm.rng <- the committed generator state held by the lookahead cache (whose
// current slot is `slot`); needed before anything reads cm.rng while it is valid
hipError_t im_commit_launch(const ImParams &p, int slot, hipStream_t s);

// Compile-time specialised NetInvMgmt kernels for the reference's own graphs
// (netspec.hip): which built-in topology a spec equals, and its launcher.
enum { NET_SPEC_NONE = 0, NET_SPEC_DEFAULT = 1, NET_SPEC_CUSTOM = 2 };
hipError_t net_spec_launch(int which, const NetParams &p, int t_u, const PolicyIO *pol,
                           const StepIO<float, float> &io, bool &ahead, int &slot, hipStream_t s);
hipError_t net_commit_launch(const NetParams &p, int slot, hipStream_t s);
hipError_t net_reset_launch(const NetParams &p, const uint8_t *mask, float *obs, hipStream_t s);
// generic (table-walking) kernel; pol: CONSTANT policy rollouts, or null
hipError_t net_run_launch(const NetParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                          hipStream_t s);
size_t net_lds_bytes(const NetParams &p);

}  // namespace invsim
