// InvManagementMasterEnv.step / reset (inventory_management.py:186-352) as
// one-thread-per-env HIP kernels for gfx950, templated on the number of
// inventory stages M1 = m-1 (register arrays) and on backlog vs lost sales.
//
// Per-env HBM state (SoA rows of Npad, all int64 like the reference):
//   I[M1]            on-hand inventory at the start of the period   (:203)
//   B[M1+1]          backlog carried into the period (backlog only)  (:208)
//   Rring[sum L_i]   fulfilled orders R, stage i keeps the last L_i in a ring;
//                    slot t mod L_i holds R[t-L_i] = this period's arrival (:275)
//   alog[D][M1]      requested orders (action_log), ring of D = lt_max rows:
//                    exactly the observation window (:380)
//   period, PCG64
// Nothing needs clearing at reset: ring entries older than the episode are
// masked by the period counter, as the reference's zero history would.
#include "kernels.hpp"

namespace invsim {
namespace {

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a + (uint64_t)b);  // numpy int64 wrap-around
}

// np.minimum(int64, float64).astype(int64) for the supplier-inventory cap (:265)
__device__ __forceinline__ int64_t min_i64_via_f64(int64_t a, int64_t sup, bool inf) {
    if (inf) return a;
    double x = (double)a, y = (double)sup;
    return (int64_t)((x <= y) ? x : y);
}

// reset (:197-220): I = I0, B = 0, period = 0; obs = [I0, 0...]
template <int M1, bool BACKLOG>
__device__ __forceinline__ void im_reset_one(const ImParams &P, int64_t e, int64_t *orow) {
    const int64_t S = P.cm.Npad;
#pragma unroll
    for (int i = 0; i < M1; i++) P.I[i * S + e] = P.I0[i];
    if (BACKLOG) {
#pragma unroll
        for (int j = 0; j <= M1; j++) P.B[j * S + e] = 0;
    }
    P.cm.period[e] = 0;
    if (orow) {
        const int O = M1 * (P.lt_max + 1);
#pragma unroll
        for (int i = 0; i < M1; i++) orow[i] = P.I0[i];
        for (int j = M1; j < O; j++) orow[j] = 0;
    }
}

// One step (:224-352) for env e at period t < periods.  Returns truncated.
template <int M1, bool BACKLOG>
__device__ __forceinline__ bool im_step_one(const ImParams &P, int64_t e, Pcg &g,
                                            const int64_t *__restrict__ arow, int64_t *orow,
                                            double &reward, int64_t *dem) {
    const int64_t S = P.cm.Npad;
    const int t = P.cm.period[e];
    const int D = P.lt_max;
    int64_t req[M1], ordreq[M1], R[M1], Icur[M1];
    int64_t Bv[M1 + 1];
#pragma unroll
    for (int i = 0; i < M1; i++) {
        const int64_t a = arow[i];
        req[i] = a > 0 ? a : 0;                                     // :250
        Icur[i] = P.I[i * S + e];
    }
#pragma unroll
    for (int j = 0; j <= M1; j++) Bv[j] = BACKLOG ? P.B[j * S + e] : 0;
#pragma unroll
    for (int i = 0; i < M1; i++) {
        ordreq[i] = sat_add(req[i], Bv[i + 1]);                     // :253-255
        const int64_t r = ordreq[i] < P.c[i] ? ordreq[i] : P.c[i];  // :263
        R[i] = min_i64_via_f64(r, (i + 1 < M1) ? Icur[i + 1] : 0, i + 1 >= M1); // :260-265
    }
    // arrivals (:271-277): R[t - L_i] from the stage ring, or this period's R when L_i == 0
#pragma unroll
    for (int i = 0; i < M1; i++) {
        const int L = P.L[i];
        if (L == 0) {
            Icur[i] += R[i];
        } else {
            const int64_t row = P.ring_off[i] + (int)((uint32_t)t % (uint32_t)L);
            if (t >= L) Icur[i] += P.Rring[row * S + e];
            P.Rring[row * S + e] = R[i];
        }
    }
    int64_t d;
    if (P.dist == 5)
        d = P.user_D[t];                                            // :182
    else
        d = np_poisson(g, P.pc);                                    // :172
    if (d < 0) d = 0;                                               // :280
    const int64_t dfill = d + Bv[0];                                // :284-286
    const int64_t s0 = Icur[0] < dfill ? Icur[0] : dfill;           // :288
    Icur[0] -= s0;
    int64_t Sv[M1 + 1], U[M1 + 1];
    Sv[0] = s0;
#pragma unroll
    for (int i = 0; i < M1; i++) Sv[i + 1] = R[i];                  // :295
#pragma unroll
    for (int i = 1; i < M1; i++) Icur[i] -= R[i];                   // :300 (reference quirk, kept)
    U[0] = dfill - s0;                                              // :303
#pragma unroll
    for (int i = 0; i < M1; i++) U[i + 1] = ordreq[i] - R[i];       // :304
    // reward (:315-322): f32 coefficients widened to f64, numpy sum order
    double term[M1 + 1];
#pragma unroll
    for (int j = 0; j <= M1; j++) {
        const double Sj = (double)Sv[j];
        const int64_t inv = (j < M1) ? Icur[j] : 0;
        const double hold = P.hc[j] * (double)(inv > 0 ? inv : 0);
        term[j] = ((P.up[j] * Sj - P.uc[j] * Sj) - hold) - P.kc[j] * (double)U[j];
    }
    const double profit = np_sum<double>(M1 + 1, [&](int j) { return term[j]; });
    reward = P.alpha_pow[t] * profit;
    // state update (:307-312, :326-330)
#pragma unroll
    for (int i = 0; i < M1; i++) P.I[i * S + e] = Icur[i];
    if (BACKLOG) {
#pragma unroll
        for (int j = 0; j <= M1; j++) P.B[j * S + e] = U[j];
    }
    const int t1 = t + 1;
    P.cm.period[e] = t1;
    if (dem) dem[e] = d;
    // observation (:354-391): I[t+1], then the last n = min(t+1, D) requested
    // orders oldest-first, zero padded at the end.  Row t is req (registers).
    if (D > 0) {
        const int n = t1 < D ? t1 : D;
        int slot = (int)((uint32_t)(t1 - n) % (uint32_t)D);
        if (orow) {
#pragma unroll
            for (int i = 0; i < M1; i++) orow[i] = Icur[i];
            int64_t *w = orow + M1;
            for (int r = 0; r + 1 < n; r++) {
#pragma unroll
                for (int i = 0; i < M1; i++) w[r * M1 + i] = P.alog[((int64_t)slot * M1 + i) * S + e];
                slot = (slot + 1 == D) ? 0 : slot + 1;
            }
#pragma unroll
            for (int i = 0; i < M1; i++) w[(n - 1) * M1 + i] = req[i];
            for (int j = n * M1; j < D * M1; j++) w[j] = 0;
        }
        const int wslot = (int)((uint32_t)t % (uint32_t)D);
#pragma unroll
        for (int i = 0; i < M1; i++) P.alog[((int64_t)wslot * M1 + i) * S + e] = req[i];   // :268
    } else if (orow) {
#pragma unroll
        for (int i = 0; i < M1; i++) orow[i] = Icur[i];
    }
    return t1 >= P.periods;                                         // :350
}

template <int M1, bool BACKLOG>
__global__ void __launch_bounds__(256)
im_step_kernel(ImParams P, const int64_t *__restrict__ act, int64_t *__restrict__ obs,
               double *__restrict__ rew, uint8_t *__restrict__ term, uint8_t *__restrict__ trunc,
               int64_t *__restrict__ fobs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int O = M1 * (P.lt_max + 1);
    int64_t *orow = obs + e * O;
    const int t = P.cm.period[e];
    if (t >= P.periods) {
        if (P.cm.autoreset == AR_NEXT_STEP) {
            im_reset_one<M1, BACKLOG>(P, e, orow);
            rew[e] = 0.0;
            term[e] = 0;
            trunc[e] = 0;
        } else {
            atomicOr(P.cm.status, 1u);  // stepping past the horizon (reference: IndexError)
        }
        return;
    }
    Pcg g = P.cm.rng.load(e);
    double r;
    const bool tr = im_step_one<M1, BACKLOG>(P, e, g, act + e * M1, orow, r, P.cm.info_demand);
    rew[e] = r;
    term[e] = 0;
    trunc[e] = tr ? 1 : 0;
    if (tr && P.cm.autoreset == AR_SAME_STEP) {
        if (fobs)
            for (int j = 0; j < O; j++) fobs[e * O + j] = orow[j];
        im_reset_one<M1, BACKLOG>(P, e, orow);
    }
    P.cm.rng.store_state(e, g);
}

template <int M1, bool BACKLOG>
__global__ void __launch_bounds__(256)
im_rollout_kernel(ImParams P, int K, const int64_t *__restrict__ act, int64_t *__restrict__ obs,
                  double *__restrict__ rew, uint8_t *__restrict__ term,
                  uint8_t *__restrict__ trunc) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int64_t N = P.cm.N;
    const int O = M1 * (P.lt_max + 1);
    Pcg g = P.cm.rng.load(e);
    for (int k = 0; k < K; k++) {
        const int64_t oi = (int64_t)k * N + e;
        int64_t *orow = obs + oi * O;
        const int t = P.cm.period[e];
        if (t >= P.periods) {
            if (P.cm.autoreset == AR_NEXT_STEP) {
                im_reset_one<M1, BACKLOG>(P, e, orow);
                rew[oi] = 0.0;
                term[oi] = 0;
                trunc[oi] = 0;
                continue;
            }
            atomicOr(P.cm.status, 1u);
            break;
        }
        double r;
        const bool tr = im_step_one<M1, BACKLOG>(P, e, g, act + oi * M1, orow, r,
                                                 k == K - 1 ? P.cm.info_demand : nullptr);
        rew[oi] = r;
        term[oi] = 0;
        trunc[oi] = tr ? 1 : 0;
        if (tr && P.cm.autoreset == AR_SAME_STEP) im_reset_one<M1, BACKLOG>(P, e, orow);
    }
    P.cm.rng.store_state(e, g);
}

template <int M1, bool BACKLOG>
__global__ void __launch_bounds__(256)
im_reset_kernel(ImParams P, const uint8_t *__restrict__ mask, int64_t *__restrict__ obs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    if (mask && !mask[e]) return;
    im_reset_one<M1, BACKLOG>(P, e, obs ? obs + e * (M1 * (P.lt_max + 1)) : nullptr);
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

#define IM_DISPATCH(M1V, BL, LAUNCH)                                   \
    switch (M1V) {                                                     \
        case 1: if (BL) LAUNCH(1, true); else LAUNCH(1, false); break; \
        case 2: if (BL) LAUNCH(2, true); else LAUNCH(2, false); break; \
        case 3: if (BL) LAUNCH(3, true); else LAUNCH(3, false); break; \
        case 4: if (BL) LAUNCH(4, true); else LAUNCH(4, false); break; \
        case 5: if (BL) LAUNCH(5, true); else LAUNCH(5, false); break; \
        case 6: if (BL) LAUNCH(6, true); else LAUNCH(6, false); break; \
        case 7: if (BL) LAUNCH(7, true); else LAUNCH(7, false); break; \
        case 8: if (BL) LAUNCH(8, true); else LAUNCH(8, false); break; \
        default: return hipErrorInvalidValue;                          \
    }

hipError_t im_step_launch(const ImParams &p, int M1, bool backlog, const int64_t *act,
                          int64_t *obs, double *rew, uint8_t *term, uint8_t *trunc,
                          int64_t *fobs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    const dim3 grid(grid_for(p.cm.N, 256)), block(256);
#define L_(M, B) hipLaunchKernelGGL((im_step_kernel<M, B>), grid, block, 0, s, p, act, obs, rew, term, trunc, fobs)
    IM_DISPATCH(M1, backlog, L_)
#undef L_
    return hipGetLastError();
}

hipError_t im_rollout_launch(const ImParams &p, int M1, bool backlog, int K, const int64_t *act,
                             int64_t *obs, double *rew, uint8_t *term, uint8_t *trunc,
                             hipStream_t s) {
    if (p.cm.N == 0 || K <= 0) return hipSuccess;
    const dim3 grid(grid_for(p.cm.N, 256)), block(256);
#define L_(M, B) hipLaunchKernelGGL((im_rollout_kernel<M, B>), grid, block, 0, s, p, K, act, obs, rew, term, trunc)
    IM_DISPATCH(M1, backlog, L_)
#undef L_
    return hipGetLastError();
}

hipError_t im_reset_launch(const ImParams &p, int M1, bool backlog, const uint8_t *mask,
                           int64_t *obs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    const dim3 grid(grid_for(p.cm.N, 256)), block(256);
#define L_(M, B) hipLaunchKernelGGL((im_reset_kernel<M, B>), grid, block, 0, s, p, mask, obs)
    IM_DISPATCH(M1, backlog, L_)
#undef L_
    return hipGetLastError();
}

}  // namespace invsim
