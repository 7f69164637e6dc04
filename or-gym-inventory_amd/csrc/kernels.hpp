// Kernel parameter blocks and launcher declarations (host <-> device contract).
//
// HBM layout: every per-env field is Structure-of-Arrays, row r of a field
// lives at  base + r * Npad + env  (Npad = N rounded up to 256), so a wave's
// 64 lanes touch 64 consecutive elements of one row: fully coalesced.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"

namespace invsim {

enum { AR_NEXT_STEP = 0, AR_SAME_STEP = 1, AR_DISABLED = 2 };

struct Common {
    int64_t N;       // envs in this handle
    int64_t Npad;    // SoA row stride (elements)
    int32_t autoreset;
    RngSoA rng;      // PCG64 state/inc rows
    int32_t *period; // [N] step counter within the episode
    int64_t *info_demand;  // optional [N][demand_dim]
    uint32_t *status;      // sticky error word (DISABLED-mode overrun)
};

// ---------------------------------------------------------------- Newsvendor
struct NvParams {
    Common cm;
    int32_t L;           // lead time
    int32_t step_limit;
    double max_inventory, max_order;
    double p_max, h_max, k_max, mu_max;
    double *par;         // [5][Npad]  price, cost, h, k, mu  (Python floats)
    float *pipe;         // [L][Npad]  order ring, slot = step index mod L
};

// ---------------------------------------------------------------- InvMgmt
constexpr int IM_MAX_M1 = 8;  // up to 9 stages
struct ImParams {
    Common cm;
    int32_t periods;
    int32_t lt_max;              // D = max lead time (obs window rows)
    int32_t dist;                // 1 poisson, 5 user_D
    int32_t L[IM_MAX_M1];
    int32_t ring_off[IM_MAX_M1]; // first R-ring row of stage i (depth L[i])
    int64_t c[IM_MAX_M1];
    int64_t I0[IM_MAX_M1];
    double up[IM_MAX_M1 + 1], uc[IM_MAX_M1 + 1], hc[IM_MAX_M1 + 1], kc[IM_MAX_M1 + 1];
    PtrsConst pc;                // Poisson(mu) constants, host libm
    const double *alpha_pow;     // [periods]  alpha ** t (Python float pow)
    const int64_t *user_D;       // [periods]
    int64_t *I;                  // [M1][Npad]   on-hand inventory I[t]
    int64_t *B;                  // [M1+1][Npad] backlog B[t] (backlog mode only)
    int64_t *Rring;              // [sum L][Npad] fulfilled orders R, ring per stage
    int64_t *alog;               // [D][M1][Npad] requested orders (action_log), ring
};

// ---------------------------------------------------------------- NetInvMgmt
struct NetParams {
    Common cm;
    int32_t J, E, RL, T, backlog, sumL;
    // topology tables (device, read with wave-uniform indices)
    const double *I0, *h, *C, *o, *v;
    const int32_t *is_factory, *is_retail;
    const int32_t *sup, *pur, *sup_is_factory, *L, *ring_off;
    const double *lp, *lg;
    const int32_t *rl_node, *rl_user;
    const double *rl_p, *rl_b;
    const PtrsConst *rl_pc;      // [RL]
    const double *user_D;        // [RL][T]
    const int32_t *succ_ptr, *succ_kind, *succ_idx, *pred_ptr, *pred_idx;
    const double *alpha_pow;     // [T]
    // state
    double *X;                   // [J][Npad]
    double *U;                   // [RL][Npad]
    double *Y;                   // [E][Npad]
    double *Rring;               // [sumL][Npad]
};

// launchers (return hipGetLastError() of the launch)
hipError_t seed_range_launch(const Common &cm, uint64_t base_lo, uint64_t base_hi, int64_t first,
                             const uint8_t *mask, hipStream_t s);
hipError_t seed_words_launch(const Common &cm, const uint32_t *words, const int32_t *nwords,
                             const uint8_t *mask, hipStream_t s);

hipError_t nv_reset_launch(const NvParams &p, const uint8_t *mask, float *obs, hipStream_t s);
hipError_t nv_step_launch(const NvParams &p, const float *act, float *obs, double *rew,
                          uint8_t *term, uint8_t *trunc, float *fobs, hipStream_t s);
hipError_t nv_rollout_launch(const NvParams &p, int K, const float *act, float *obs, double *rew,
                             uint8_t *term, uint8_t *trunc, hipStream_t s);

hipError_t im_reset_launch(const ImParams &p, int M1, bool backlog, const uint8_t *mask,
                           int64_t *obs, hipStream_t s);
hipError_t im_step_launch(const ImParams &p, int M1, bool backlog, const int64_t *act,
                          int64_t *obs, double *rew, uint8_t *term, uint8_t *trunc,
                          int64_t *fobs, hipStream_t s);
hipError_t im_rollout_launch(const ImParams &p, int M1, bool backlog, int K, const int64_t *act,
                             int64_t *obs, double *rew, uint8_t *term, uint8_t *trunc,
                             hipStream_t s);

hipError_t net_reset_launch(const NetParams &p, const uint8_t *mask, float *obs, hipStream_t s);
hipError_t net_step_launch(const NetParams &p, const float *act, float *obs, double *rew,
                           uint8_t *term, uint8_t *trunc, float *fobs, hipStream_t s);
hipError_t net_rollout_launch(const NetParams &p, int K, const float *act, float *obs,
                              double *rew, uint8_t *term, uint8_t *trunc, hipStream_t s);

}  // namespace invsim
