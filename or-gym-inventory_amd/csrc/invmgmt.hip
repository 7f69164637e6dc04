// InvManagementMasterEnv.step / reset (inventory_management.py:186-352) as
// HIP kernels for gfx950, templated on M1 = m-1 inventory stages (register
// arrays), backlog vs lost sales, and whether the episode period is lock-step
// uniform (TU).
//
// Work layout: one wave = 16 envs x 4 lanes (group_rng.hpp).  The 4 lanes of
// an env run the (cheap, integer) dynamics redundantly, evaluate 4 Poisson
// candidates in parallel, split the observation-window copy, and only the
// group leader writes state.  Observation rows are assembled in an LDS tile
// and written with 16-byte coalesced stores.
//
// Per-env HBM state (SoA rows of Npad, int64 like the reference):
//   I[M1]            on-hand inventory at the start of the period   (:203)
//   B[M1+1]          backlog carried into the period (backlog only)  (:208)
//   Rring[sum L_i]   fulfilled orders R; stage i keeps its last L_i in a ring,
//                    slot t mod L_i = R[t-L_i] = this period's arrival (:275)
//   alog32[D][Npad][M1] requested orders (action_log) ring of D = lt_max rows, 32-bit,
//                    an env's row contiguous
//                    (alog: int64 ring for the rare entries >= 2^32 - 1):
//                    exactly the observation window (:380)
//   period (only when not lock-step), PCG64
// Ring entries older than the episode are masked by the period counter, as the
// reference's zeroed history would be, so reset writes only I, B, period.
//
// A launch runs K >= 1 consecutive steps (invsim_step: K = 1; invsim_rollout:
// K) with PCG64, I, B and the period in registers.
#include "kernels.hpp"

namespace invsim {
namespace {

#ifdef INVSIM_TIMING
__device__ uint64_t g_tbuf[TB_WAVES * TB_PROBES];
#endif

// obs-window entries per lane kept in registers: the (lt_max - 1) * M1 entries
// of lt_max <= 10, capped at 36 (longer windows are copied ring -> LDS directly)
// Requested orders are >= 0 (np.maximum(action, 0), :250) and, for any sane
// policy, far below 2^32: the action_log ring keeps 4 bytes per entry, with a
// sentinel sending the rare wider value to the int64 ring (halves the step's
// largest read, the observation window)
constexpr uint32_t IM_WIDE = 0xFFFFFFFFu;

__device__ __forceinline__ int64_t alog_get(const ImParams &P, int64_t idx) {
    const uint32_t v = P.alog32[idx];
    return v == IM_WIDE ? P.alog[idx] : (int64_t)v;
}

constexpr int im_wlane(int m1) { return m1 * (9 < 36 / m1 ? 9 : 36 / m1); }   // whole rows

// numpy int64 array arithmetic wraps around (two's complement)
__device__ __forceinline__ int64_t wrap_add(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a + (uint64_t)b);
}
__device__ __forceinline__ int64_t wrap_sub(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a - (uint64_t)b);
}

// np.minimum(int64, float64).astype(int64) for the supplier-inventory cap (:265)
__device__ __forceinline__ int64_t min_via_f64(int64_t a, int64_t sup) {
    const double x = (double)a, y = (double)sup;
    return (int64_t)((x <= y) ? x : y);
}

// The step's global stores, issued after the obs tile store: gfx9 VMEM stores
// read their data VGPRs late and vmcnt also counts stores, so a store issued
// before the tile copy makes every later overwrite of its data registers wait
// for the store to complete.
template <int M1>
struct ImPending {
    int64_t R[M1], req[M1];
    int t;
};

template <int M1, bool BACKLOG, class G = Pcg>
struct ImState {
    G g;
    uint64_t u32;        // PCG64 32-bit buffer (dist 3 only)
    int64_t I[M1];
    int64_t B[M1 + 1];
};

// reset (:197-220): I = I0, B = 0; obs row = [I0, 0...] (lane j of the group
// writes every 4th element)
template <int M1, bool BACKLOG, class G = Pcg>
__device__ __forceinline__ void im_reset_regs(const ImParams &P, ImState<M1, BACKLOG, G> &s,
                                              int64_t *orow, int j) {
#pragma unroll
    for (int i = 0; i < M1; i++) s.I[i] = P.I0[i];
#pragma unroll
    for (int q = 0; q <= M1; q++) s.B[q] = 0;
    if (orow) {
        const int O = M1 * (P.lt_max + 1);
        for (int q = j; q < O; q += LPE) orow[q] = (q < M1) ? P.I0[q] : 0;
    }
}

// One step (:224-352) at period t < periods.  Returns truncated.
template <int M1, bool BACKLOG, bool NPD, class G = Pcg>
__device__ __forceinline__ bool im_step_regs(const ImParams &P, int64_t e, bool valid, int j, int t,
                                             ImState<M1, BACKLOG, G> &s,
                                             const int64_t *__restrict__ arow, int64_t *orow,
                                             const double *rhs, TableStage *ts, double apow, int64_t udem,
                                             double &reward, int64_t &dem_out, double *met, int64_t *irec,
                                             ImPending<M1> &pend) {
    const int64_t S = P.cm.Npad;
    const int D = P.lt_max;
    const bool leader = valid && j == 0;   // state writes
    // Phase A: every load of the step up front (actions, arrivals, this lane's
    // share of the observation window) so the latency overlaps the demand draw
    int64_t req[M1], ordreq[M1], R[M1], arr[M1];
#pragma unroll
    for (int i = 0; i < M1; i++) req[i] = arow[i];
#pragma unroll
    for (int i = 0; i < M1; i++) {                                  // arrivals R[t-L_i] (:271-277)
        // unconditional load (row 0 when L = 0: the ring always has a row) so the
        // step's loads are straight-line and their waits exact; masked below
        const int L = P.L[i];
        const int row = L > 0 ? P.ring_off[i] + (int)((uint32_t)t % (uint32_t)L) : 0;
        arr[i] = P.Rring[(int64_t)row * S + e];
        if (!(L > 0 && t >= L)) arr[i] = 0;
    }
    // window rows t+1-n .. t-1 of the action_log ring (:380): nw entries, lane j
    // takes entries q = j, j+4, ...
    const int t1 = t + 1;
    const int n = D > 0 ? (t1 < D ? t1 : D) : 0;
    const int nw = n > 0 ? (n - 1) * M1 : 0;
    const int slot0 = D > 0 ? (int)((uint32_t)(t1 - n) % (uint32_t)D) : 0;
    // action_log ring layout [slot][env][stage]: one env's row of a slot is M1
    // contiguous words, so a window row is one vector load (dwordx3 at M1 = 3)
    auto wrow = [&](int r) -> int64_t {
        int slot = slot0 + r;
        slot = slot >= D ? slot - D : slot;
        return ((int64_t)slot * S + e) * M1;
    };
    auto widx = [&](int q) -> int64_t {
        const int r = q / M1, i = q - r * M1;
        return wrow(r) + i;
    };
    constexpr int WL = im_wlane(M1);
    const bool wreg = orow && (D - 1) * M1 <= WL * LPE;   // launch-uniform
    uint32_t wv[WL];
#ifndef INVSIM_ABL_NO_WINDOW
    {   // unconditional (straight-line loads, exact vmcnt waits): entries past nw
        // (start of an episode) re-read the last valid one, or entry 0, always a
        // valid ring row; unused when !wreg
        static_assert(LPE == 1, "window rows are loaded whole per lane");
        const int rmax = nw > 0 ? nw / M1 - 1 : 0;   // last valid window row
#pragma unroll
        for (int r = 0; r < WL / M1; r++) {
            const uint32_t *src = P.alog32 + wrow(r < rmax ? r : rmax);
#pragma unroll
            for (int i = 0; i < M1; i++) wv[r * M1 + i] = src[i];
        }
    }
#endif
    TPROBE(1);   // step loads issued
    if (ts) ts->flush((int)threadIdx.x);
    // Phase B: demand, a function of the RNG stream only (:172, :280)
#ifdef INVSIM_ABL_NO_POISSON  // profiling ablation build only (wrong results)
    int64_t d = 20 + (int64_t)(s.g.lo & 3);
#else
    s.g.sub(0);
    if constexpr (G::kCounter) s.u32 = 0;    // fast stream: no 32-bit half carried between steps
    int64_t d = NPD ? np_demand(s.g, s.u32, P.nd) : (P.dist == 5) ? udem : env_poisson(s.g, P.pc, rhs);
#endif
    if (d < 0) d = 0;
    TPROBE(2);
    // Phase C: dynamics (identical in the 4 lanes)
#pragma unroll
    for (int i = 0; i < M1; i++) req[i] = req[i] > 0 ? req[i] : 0;  // :250
#pragma unroll
    for (int i = 0; i < M1; i++) {
        ordreq[i] = wrap_add(req[i], s.B[i + 1]);                   // :253-255
        const int64_t r = ordreq[i] < P.c[i] ? ordreq[i] : P.c[i];  // :263
        // :260-265 np.minimum(., [I[t,1:], inf]) in float64, then astype(int64):
        // the last stage's cap is +inf but the f64 round trip still rounds |r| > 2^53
        R[i] = (i + 1 < M1) ? min_via_f64(r, s.I[i + 1]) : (int64_t)(double)r;
    }
    int64_t Icur[M1];
#pragma unroll
    for (int i = 0; i < M1; i++) {
        const int L = P.L[i];
        Icur[i] = wrap_add(s.I[i], L == 0 ? R[i] : arr[i]);
        pend.R[i] = R[i];                                           // ring slot t mod L <- R[t] (:267)
    }
    pend.t = t;
    const int64_t dfill = wrap_add(d, s.B[0]);                      // :284-286
    const int64_t s0 = Icur[0] < dfill ? Icur[0] : dfill;           // :288
    Icur[0] = wrap_sub(Icur[0], s0);
    int64_t Sv[M1 + 1], U[M1 + 1];
    Sv[0] = s0;
#pragma unroll
    for (int i = 0; i < M1; i++) Sv[i + 1] = R[i];                  // :295
#pragma unroll
    for (int i = 1; i < M1; i++) Icur[i] = wrap_sub(Icur[i], R[i]); // :300 (reference quirk, kept)
    U[0] = wrap_sub(dfill, s0);                                     // :303
#pragma unroll
    for (int i = 0; i < M1; i++) U[i + 1] = wrap_sub(ordreq[i], R[i]); // :304
    double term[M1 + 1];                                            // :315-321
#pragma unroll
    for (int q = 0; q <= M1; q++) {
        const double Sj = (double)Sv[q];
        const int64_t inv = (q < M1) ? Icur[q] : 0;
        const double hold = P.hc[q] * (double)(inv > 0 ? inv : 0);
        term[q] = ((P.up[q] * Sj - P.uc[q] * Sj) - hold) - P.kc[q] * (double)U[q];
    }
    const double profit = np_sum<double>(M1 + 1, [&](int q) { return term[q]; });
    reward = apow * profit;                                         // :322
    TPROBE(6);
#pragma unroll
    for (int i = 0; i < M1; i++) s.I[i] = Icur[i];                  // :326
#pragma unroll
    for (int q = 0; q <= M1; q++) s.B[q] = BACKLOG ? U[q] : 0;      // :307-312
    dem_out = d;
    if (irec) {  // step info (inventory_management.py:334-345): S[t], U[t], then the
                 // f64 bits of period_profit, revenue, procurement, holding, penalty sums
        constexpr int W = 2 * (M1 + 1) + 5;
        int64_t *rr = irec + e * W;
#pragma unroll
        for (int q = 0; q <= M1; q++) {
            rr[q] = Sv[q];
            rr[M1 + 1 + q] = U[q];
        }
        const double rev = np_sum<double>(M1 + 1, [&](int q) { return P.up[q] * (double)Sv[q]; });
        const double pro = np_sum<double>(M1 + 1, [&](int q) { return P.uc[q] * (double)Sv[q]; });
        const double hol = np_sum<double>(M1 + 1, [&](int q) {
            const int64_t inv = (q < M1) ? Icur[q] : 0;
            return P.hc[q] * (double)(inv > 0 ? inv : 0);
        });
        const double pen = np_sum<double>(M1 + 1, [&](int q) { return P.kc[q] * (double)U[q]; });
        rr[2 * (M1 + 1) + 0] = __double_as_longlong(profit);
        rr[2 * (M1 + 1) + 1] = __double_as_longlong(rev);
        rr[2 * (M1 + 1) + 2] = __double_as_longlong(pro);
        rr[2 * (M1 + 1) + 3] = __double_as_longlong(hol);
        rr[2 * (M1 + 1) + 4] = __double_as_longlong(pen);
    }
    if (met) {   // evaluate_agent metrics (benchmark_InvManagementBacklogEnv.py:378-399)
        met[2] += (double)d;                                        // demand_realized
        met[3] += (double)Sv[0];                                    // sales[0]
        met[4] += (double)U[0];                                     // unfulfilled[0]
        int64_t es = 0;                                             // sum(max(0, ending_inventory))
#pragma unroll
        for (int i = 0; i < M1; i++) es = wrap_add(es, Icur[i] > 0 ? Icur[i] : 0);
        met[5] += (double)es;
    }
    if (orow) {                                                     // :354-391
        int64_t *w = orow + M1;
        if (j == 0) {
#pragma unroll
            for (int i = 0; i < M1; i++) orow[i] = Icur[i];
        }
        if (D > 0) {
            if (wreg) {
                // branch-free: the WL = (D-1)*M1 oldest slots get the window or 0,
                // then the tail slots are cleared before an early-episode newest row
                bool wide = false;
#pragma unroll
                for (int u = 0; u < WL; u++) {
                    const int q = j + u * LPE;
                    if (q < (D - 1) * M1) w[q] = (q < nw) ? (int64_t)wv[u] : 0;
                    wide |= (q < nw) && wv[u] == IM_WIDE;
                }
                if (wide) {   // rare: entries >= 2^32 - 1 come from the int64 ring
#pragma unroll
                    for (int u = 0; u < WL; u++) {
                        const int q = j + u * LPE;
                        if (q < nw && wv[u] == IM_WIDE) w[q] = P.alog[widx(q)];
                    }
                }
                if (n < D)
                    for (int q = (D - 1) * M1 + j; q < D * M1; q += LPE) w[q] = 0;
            } else {
#ifndef INVSIM_ABL_NO_WINDOW
                for (int q = j; q < nw; q += LPE) w[q] = alog_get(P, widx(q));
#endif
                for (int q = n * M1 + j; q < D * M1; q += LPE) w[q] = 0;
            }
        }
        if (j == 0 && D > 0) {
#pragma unroll
            for (int i = 0; i < M1; i++) w[(n - 1) * M1 + i] = req[i];   // newest row last (:380)
        }
    }
#pragma unroll
    for (int i = 0; i < M1; i++) pend.req[i] = req[i];              // action_log[t] (:268)
    TPROBE(3);
    return t1 >= P.periods;                                         // :350
}

template <int M1>
__device__ __forceinline__ void im_flush_pending(const ImParams &P, const ImPending<M1> &pend, int64_t e) {
    const int64_t S = P.cm.Npad;
    const int t = pend.t;
#pragma unroll
    for (int i = 0; i < M1; i++) {
        const int L = P.L[i];
        if (L > 0) st_store(P.Rring + (int64_t)(P.ring_off[i] + (int)((uint32_t)t % (uint32_t)L)) * S + e, pend.R[i]);
    }
    const int D = P.lt_max;
    if (D > 0) {
        const int wslot = (int)((uint32_t)t % (uint32_t)D);
#pragma unroll
        for (int i = 0; i < M1; i++) {
            const int64_t idx = ((int64_t)wslot * S + e) * M1 + i;
            const bool wide = pend.req[i] >= (int64_t)IM_WIDE;
            st_store(P.alog32 + idx, wide ? IM_WIDE : (uint32_t)pend.req[i]);
            if (wide) st_store(P.alog + idx, pend.req[i]);
        }
    }
}

// BaseStockAgent.get_action (benchmark_InvManagementBacklogEnv.py:152-198): order
// up to (L_i + 1) * mu * sf over the inventory position on hand + requested
// orders of the last L_i periods (action_log[max(0, t - L_i) : t, i]), in
// float64, clipped to [0, c_i], truncated to int64.
template <int M1, bool BACKLOG, class G = Pcg>
__device__ __forceinline__ void im_base_stock(const ImParams &P, const PolicyIO &pol, const ImState<M1, BACKLOG, G> &st,
                                              int t, int64_t e, int64_t (&act)[M1]) {
    const int64_t S = P.cm.Npad;
    const int D = P.lt_max;
#pragma unroll
    for (int i = 0; i < M1; i++) {
        const int L = P.L[i];
        int64_t pos = st.I[i];                                      // observation[:M1] = I[t]
        if (L > 0) {
            int64_t pipe = 0;
            for (int a = 1; a <= L; a++) {
                const int tau = t - a;
                if (tau >= 0)
                    pipe = wrap_add(pipe, alog_get(P, ((int64_t)((uint32_t)tau % (uint32_t)D) * S + e) * M1 + i));
            }
            pos = wrap_add(pos, pipe);
        }
        const double target = ((double)(L + 1) * pol.mu) * pol.sf;   // (lead_times + 1) * mu * sf
        double x = target - (double)pos;
        x = (x > 0) ? x : 0.0;                                      // np.maximum(0, .)
        x = (x < 0.0) ? 0.0 : x;                                    // np.clip(., low = 0, high = c)
        x = (x > (double)P.c[i]) ? (double)P.c[i] : x;
        act[i] = (int64_t)x;                                        // astype(int64)
    }
}

// Step k of a launch for the wave's envs: step (or NEXT_STEP reset) into the
// LDS obs tile, SAME_STEP final-obs/reset, then the tile's coalesced store.
template <int M1, bool BACKLOG, bool STEP_ONLY, bool POL, bool NPD, class G = Pcg>
__device__ __forceinline__ void im_launch_step(const ImParams &P, const StepIO<int64_t, int64_t> &io, int k,
                                               int64_t e, int64_t e0, int lane, bool valid, int nvalid,
                                               ImState<M1, BACKLOG, G> &st, int &t, bool &fault,
                                               int64_t *tile, int64_t *trow, const double *rhs,
                                               TableStage *ts, const double *pre_apow, const int64_t *pre_udem,
                                               const PolicyIO &pol, double *met) {
    const int j = lane & (LPE - 1);
    const bool leader = j == 0;
    const int64_t N = P.cm.N;
    const int O = M1 * (P.lt_max + 1);
    const int64_t oi = (int64_t)k * N + e;
    bool tr = false;
    bool stepped = false;
    double rew = 0.0;
    int64_t dem = 0;
    ImPending<M1> pend;
    if (!STEP_ONLY && ts) {   // all lanes write the table before the divergent branch
        ts->flush(lane);
        ts = nullptr;
    }
    if (!STEP_ONLY && t >= P.periods) {
        if (P.cm.autoreset == AR_NEXT_STEP) {
            im_reset_regs<M1, BACKLOG>(P, st, trow, j);
            if (valid && leader && (!POL || io.rew)) {
                out_store(io.rew + oi, 0.0);
                out_store(io.term + oi, (uint8_t)0);
                out_store(io.trunc + oi, (uint8_t)0);
            }
            t = 0;
        } else {
            fault = true;  // stepping past the horizon (reference: IndexError)
        }
    } else {
        // every lane steps (lanes past N read padded state columns and the last
        // env's actions); only valid lanes store
        double r;
        int64_t d;
        const int64_t ea = valid ? oi : (int64_t)k * N + (N - 1);
        // per-period scalars (alpha**t, user_D[t]: always a valid table), loaded
        // before any store of the step (vmcnt counts stores too) unless preloaded
        const double apow = pre_apow ? *pre_apow : P.alpha_pow[t];
        const int64_t udem = pre_udem ? *pre_udem : P.user_D[t];
        const int64_t *arow = io.act + ea * M1;
        int64_t pact[M1];
        if (POL) {
            if (pol.kind == POL_BASE_STOCK) {
                im_base_stock<M1, BACKLOG>(P, pol, st, t, e, pact);
            } else {
#pragma unroll
                for (int i = 0; i < M1; i++) pact[i] = pol.ci[i];
            }
            if (valid && pol.act_out) {
#pragma unroll
                for (int i = 0; i < M1; i++) out_store((int64_t *)pol.act_out + oi * M1 + i, pact[i]);
            }
            arow = pact;
        }
        tr = im_step_regs<M1, BACKLOG, NPD>(P, e, valid, j, t, st, arow, trow, rhs, ts, apow, udem, r, d,
                                            POL ? met : nullptr,
                                            (valid && leader && k == io.K - 1) ? (int64_t *)P.cm.info_rec : nullptr,
                                            pend);
        stepped = true;
        if (POL) {
            met[0] += r;                                            // episode_reward += reward
            met[1] += 1.0;                                          // episode_steps
        }
        rew = r;
        dem = d;
        t += 1;
    }
    wave_lds_sync();
    if (P.cm.autoreset == AR_SAME_STEP) {        // final obs out, then the reset obs in
        if (valid && tr && io.fobs)
            for (int q = j; q < O; q += LPE) io.fobs[e * O + q] = trow[q];
        wave_lds_sync();
        if (tr) {
            im_reset_regs<M1, BACKLOG>(P, st, trow, j);
            t = 0;
        }
        wave_lds_sync();
    }
#ifndef INVSIM_ABL_NO_OBS  // profiling ablation build only
    // obs tile: at most 64 * M1 * 11 int64 in register-window configurations
    if (!POL || io.obs)
        store_tile<(M1 * 11 * EPW * 8 + 16 * WAVE - 1) / (16 * WAVE)>(tile, io.obs + ((int64_t)k * N + e0) * O,
                                                                     (int64_t)nvalid * O, lane);
#endif
    // the step's own stores, after the tile copy (see ImPending)
    if (stepped && valid && leader) {
        im_flush_pending<M1>(P, pend, e);
        if (!POL || io.rew) {
            out_store(io.rew + oi, rew);
            out_store(io.term + oi, (uint8_t)0);
            out_store(io.trunc + oi, (uint8_t)(tr ? 1 : 0));
        }
        if (k == io.K - 1 && P.cm.info_demand) P.cm.info_demand[e] = dem;
    }
    TPROBE(4);
    wave_lds_sync();
}

template <int M1, bool BACKLOG, bool TU, bool ONE, bool POL, bool NPD, class G>
__global__ void __launch_bounds__(WAVE)
im_run_kernel(ImParams P, int t_u, StepIO<int64_t, int64_t> io, PolicyIO pol) {
    extern __shared__ __attribute__((aligned(16))) int64_t im_tile[];
    const int lane = threadIdx.x;
    const int j = lane & (LPE - 1);
    const bool leader = j == 0;
    const int64_t e0 = (int64_t)blockIdx.x * EPW;
    const int64_t e = e0 + (lane / LPE);
    const int64_t N = P.cm.N;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < EPW ? (N - e0) : EPW);
    const int O = M1 * (P.lt_max + 1);
    const int64_t S = P.cm.Npad;
    int64_t *trow = im_tile + (int64_t)(lane / LPE) * O;
    TPROBE(0);
    TPROBE_ID();
    if (ONE && TU && t_u >= P.periods) {
        // lock-step NEXT_STEP autoreset of the whole batch (the host refuses a
        // DISABLED overrun when the period is lock-step, and SAME_STEP resets in
        // the done step): no state to load, so a separate straight path
        if (valid) {
#pragma unroll
            for (int i = 0; i < M1; i++) P.I[i * S + e] = P.I0[i];
            if (BACKLOG) {
#pragma unroll
                for (int q = 0; q <= M1; q++) P.B[q * S + e] = 0;
            }
            out_store(io.rew + e, 0.0);
            out_store(io.term + e, (uint8_t)0);
            out_store(io.trunc + e, (uint8_t)0);
        }
        for (int q = 0; q < O; q++) trow[q] = (q < M1) ? P.I0[q] : 0;
        wave_lds_sync();
        store_tile(im_tile, io.obs + e0 * O, (int64_t)nvalid * O, lane);
        return;
    }
    // PTRS right-hand-side table -> LDS (after the obs tile), so the demand
    // draw's lookups do not queue behind the step's global loads (vmcnt is in order)
    // (fixed count of clamped loads issued first, written to LDS after the state
    // loads are in flight)
    // loads in the order their values are needed: period scalars, RHS table, PCG64, state
    const int t0 = TU ? t_u : (valid ? P.cm.period[e] : 0);   // padded lanes: any in-range period
    const int tc = t0 < P.periods ? t0 : 0;
    const double apow0 = P.alpha_pow[tc];
    const int64_t udem0 = P.user_D[tc];
    double *rhs_l = reinterpret_cast<double *>(im_tile + (int64_t)EPW * O);
    TableStage ts;
    ts.dst = rhs_l;
    {
        const bool has_tab = P.pc.nk > 0;
        const double *tsrc = has_tab ? P.rhs : P.alpha_pow;   // any valid pointer
        const int qm = has_tab ? P.pc.nk - 1 : 0;
#pragma unroll
        for (int u = 0; u < TableStage::NT; u++) ts.v[u] = tsrc[min(lane + u * WAVE, qm)];
    }

    // state rows are Npad wide, so every lane loads unconditionally (straight-line
    // loads keep the compiler's vmcnt waits exact); lanes past N take the last
    // env's PCG64 stream (an all-zero stream would never leave the PTRS loop)
    ImState<M1, BACKLOG, G> st;
    P.cm.rng.load(valid ? e : N - 1, st.g);
    st.g.set_step(P.cm.ph_step);
    st.u32 = (NPD && !G::kCounter) ? P.cm.u32buf[valid ? e : N - 1] : 0;
#pragma unroll
    for (int i = 0; i < M1; i++) st.I[i] = P.I[i * S + e];
#pragma unroll
    for (int q = 0; q <= M1; q++) st.B[q] = BACKLOG ? P.B[q * S + e] : 0;
    int t = t0;
    bool fault = false;
    constexpr int MD = 6;                       // metrics (invsim.h INVSIM_METRICS_*)
    double met[MD];
#pragma unroll
    for (int q = 0; q < MD; q++) met[q] = (POL && pol.metrics) ? pol.metrics[(valid ? e : N - 1) * MD + q] : 0.0;
    if (ONE) {
        im_launch_step<M1, BACKLOG, TU, false, NPD>(P, io, 0, e, e0, lane, valid, nvalid, st, t, fault, im_tile, trow,
                                               rhs_l, &ts, &apow0, &udem0, pol, met);
    } else {
        ts.flush(lane);
        for (int k = 0; k < io.K; k++) {
            st.g.set_step(P.cm.ph_step + (uint64_t)k);
            im_launch_step<M1, BACKLOG, false, POL, NPD>(P, io, k, e, e0, lane, valid, nvalid, st, t, fault, im_tile,
                                                    trow, rhs_l, nullptr, nullptr, nullptr, pol, met);
        }
    }
    if (valid && leader) {
        P.cm.rng.store_state(e, st.g);
        if (NPD && !G::kCounter) P.cm.u32buf[e] = st.u32;
#pragma unroll
        for (int i = 0; i < M1; i++) st_store(P.I + i * S + e, st.I[i]);
        if (BACKLOG) {
#pragma unroll
            for (int q = 0; q <= M1; q++) st_store(P.B + q * S + e, st.B[q]);
        }
        if (!TU) P.cm.period[e] = t;
        if (fault) atomicOr(P.cm.status, 1u);
        if (POL && pol.metrics) {
#pragma unroll
            for (int q = 0; q < MD; q++) pol.metrics[e * MD + q] = met[q];
        }
    }
    TWAIT();
    TPROBE(5);
}

template <int M1, bool BACKLOG>
__global__ void __launch_bounds__(256)
im_reset_kernel(ImParams P, const uint8_t *__restrict__ mask, int64_t *__restrict__ obs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    if (mask && !mask[e]) return;
    const int64_t S = P.cm.Npad;
    const int O = M1 * (P.lt_max + 1);
#pragma unroll
    for (int i = 0; i < M1; i++) P.I[i * S + e] = P.I0[i];
    if (BACKLOG) {
#pragma unroll
        for (int q = 0; q <= M1; q++) P.B[q * S + e] = 0;
    }
    P.cm.period[e] = 0;
    if (obs) {
        int64_t *orow = obs + e * O;
        for (int q = 0; q < O; q++) orow[q] = (q < M1) ? P.I0[q] : 0;
    }
}

// Cross-wave LDS handoff inside a workgroup: orders LDS traffic only (an
// __syncthreads() would also drain each wave's outstanding global loads and
// stores, s_waitcnt vmcnt(0), before the s_barrier)
__device__ __forceinline__ void wg_lds_sync() {
    TBAR_T0();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    TBAR_ADD();
}

// Single lock-step step (invsim_step, K = 1, t_u < periods, no SAME_STEP reset
// in this step) with the work of 64 envs split over two waves of one
// workgroup:
//   wave 0 (window)   the observation window rows t+1-n .. t-1 of the action_log
//                     ring into the LDS tile, and this step's demand d
//   wave 1 (dynamics) actions, arrivals, I, B; the demand-independent part of
//                     the dynamics, then (after the handoff of d through LDS)
//                     sales, backlog, reward, the tile's inventory and newest
//                     action row, and the state / output stores
// Both waves then store half of the observation tile.  Same arithmetic, in
// the same order, as im_step_regs (inventory_management.py:224-352).
// With the lookahead (AHEAD) the dynamics wave loads d from the cache itself,
// so it computes as soon as its own loads land, and the waves meet only once,
// when the tile is complete (the window wave leaves the newest row's words to
// the dynamics wave).
//
// Demand lookahead (P.ahead: two slots of [state hi, state lo, demand, 32-bit
// buffer] x Npad, alternating per launch).  The demand is a function of the
// env's generator stream only, so each launch also draws the NEXT step's
// demand.  AHEAD (slot `cur` holds every env's state one draw past the
// committed one, and that draw): wave 0 just loads d, and `gla` extra
// workgroups at the front of the grid (128 envs each, no barriers) draw the
// next demand from slot cur's state and write it to slot cur ^ 1 -- so the
// Poisson chain (~2.5 us) runs beside the step instead of before it.
// !AHEAD (first step after a seed / set_state / other kernel): wave 0 draws d
// inline from cm.rng, stores that state to slot cur, then draws the lookahead
// into slot cur ^ 1.  Either way every stream is consumed in the reference's
// order.  The committed state (after this step's draw) is left in slot cur,
// which the host flips to `cur ^ 1` of the new current slot; cm.rng is brought
// up to date from it (im_commit_kernel) only before something reads it: another
// kernel, get_state, a masked seed.
// RG = PhiloxGen (the fast stream, invmgmt_ph.hip): the same lookahead, but a
// draw is a function of (key, launch step) only, so the cache holds just the
// next step's demand (row 2 of a slot) and no generator state is read or written.
template <int M1, bool BACKLOG, bool NPD, bool AHEAD, class RG = Pcg>
__global__ void __launch_bounds__(2 * WAVE)
im_split_kernel(ImParams P, int t, StepIO<int64_t, int64_t> io, int cur, int la0, int gla) {
    extern __shared__ __attribute__((aligned(16))) int64_t im_tile[];
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    double *rhs_l = reinterpret_cast<double *>(im_tile + (int64_t)WAVE * M1 * (P.lt_max + 1));
    uint64_t *Acur = P.ahead ? P.ahead + (int64_t)cur * 4 * S : nullptr;
    uint64_t *Anxt = P.ahead ? P.ahead + (int64_t)(cur ^ 1) * 4 * S : nullptr;
    const int64_t udem = P.user_D[t];
    auto stage_table = [&](int lane) {
        TableStage ts;
        ts.dst = rhs_l;
        const bool has_tab = P.pc.nk > 0 && P.dist == 1;
        const double *tsrc = has_tab ? P.rhs : P.alpha_pow;    // any valid pointer
        const int qm = has_tab ? P.pc.nk - 1 : 0;
#pragma unroll
        for (int u = 0; u < TableStage::NT; u++) ts.v[u] = tsrc[min(lane + u * WAVE, qm)];
        return ts;
    };
    auto draw = [&](auto &g, uint64_t &u32) -> int64_t {
#ifdef INVSIM_ABL_NO_POISSON  // profiling ablation build only (wrong results)
        int64_t x = 20 + (int64_t)(g.lo & 3);
        g.next64();
#else
        int64_t x = NPD ? np_demand(g, u32, P.nd) : (P.dist == 5) ? udem : env_poisson(g, P.pc, rhs_l);
#endif
        return x < 0 ? 0 : x;
    };
    // DEC: with the lookahead the dynamics wave loads d itself and the waves
    // meet once (tile complete); otherwise d is handed over at a first barrier
#ifdef INVSIM_IM_SPLIT_DSYNC   // A/B build only: the round-5 handoff of d through LDS
    constexpr bool DEC = false;
#else
    constexpr bool DEC = AHEAD;
#endif
    const int bid = (int)blockIdx.x;
    TPROBE(0);
    TPROBE_ID();
    if (AHEAD && bid >= la0 && bid < la0 + gla) {   // ---- lookahead workgroup: 128 envs, one per lane
        const int64_t e = (int64_t)(bid - la0) * (2 * WAVE) + threadIdx.x;
        const bool valid = e < N;
        const int64_t ee = valid ? e : N - 1;
        TableStage ts = stage_table((int)(threadIdx.x & (WAVE - 1)));
        if constexpr (RG::kCounter) {   // the fast stream: the draw of launch step ph_step + 1
            RG g;
            P.cm.rng.load(ee, g);
            g.set_step(P.cm.ph_step + 1);
            g.sub(0);
            uint64_t u32 = 0;
            ts.flush((int)(threadIdx.x & (WAVE - 1)));
            const int64_t dn = draw(g, u32);
            if (valid) st_store(Anxt + 2 * S + e, (uint64_t)dn);
            return;
        }
        Pcg g;
        g.hi = Acur[ee];
        g.lo = Acur[S + ee];
        g.inc_hi = P.cm.rng.inc_hi[ee];
        g.inc_lo = P.cm.rng.inc_lo[ee];
        uint64_t u32 = NPD ? Acur[3 * S + ee] : 0;
        PtrsJumpLane jt;
        jt.load((int)(threadIdx.x & (WAVE - 1)));
        ts.flush((int)(threadIdx.x & (WAVE - 1)));   // each wave writes the whole (identical) table
        TPROBE(1);
        // slot cur keeps this state: the committed one once the slots flip
        int64_t dn;
#ifndef INVSIM_ABL_NO_POISSON
        if (!NPD && P.dist == 1 && P.pc.lam >= 10)   // PTRS with a compacted second round
            dn = np_poisson_ptrs_compact(
                g, P.pc, RhsTab{rhs_l}, true, jt,
                [](const PtrsConst &c, int) { return c; });
        else
#endif
            dn = draw(g, u32);
        TPROBE(2);
        if (valid) {
            st_store(Anxt + e, g.hi);
            st_store(Anxt + S + e, g.lo);
            st_store(Anxt + 2 * S + e, (uint64_t)dn);
            if (NPD) st_store(Anxt + 3 * S + e, u32);
        }
        TWAIT();
        TPROBE(5);
        return;
    }
    const int lane = threadIdx.x & (WAVE - 1);
    const bool demand_wave = threadIdx.x < WAVE;
    const int64_t e0 = (int64_t)(AHEAD && bid >= la0 ? bid - gla : bid) * WAVE;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < WAVE ? (N - e0) : WAVE);
    const int D = P.lt_max;
    const int O = M1 * (D + 1);
    int64_t *trow = im_tile + (int64_t)lane * O;
    int64_t *w = trow + M1;
    int64_t *dsh = reinterpret_cast<int64_t *>(rhs_l + RHS_LDS_MAX);
    const int t1 = t + 1;
    const int n = D > 0 ? (t1 < D ? t1 : D) : 0;                    // window rows incl. the newest
    const int nw = n > 0 ? (n - 1) * M1 : 0;
    // the tile halves each wave stores (16-byte aligned: an even int64 count)
    const int64_t tcount = (int64_t)nvalid * O;
    const int64_t thalf = ((tcount / 2) + 1) & ~(int64_t)1;
    constexpr int WL = im_wlane(M1);
    const bool wreg = (D - 1) * M1 <= WL;   // launch-uniform
    // window rows t+1-n .. t-1 (:380), loaded whole (see im_step_regs)
    const int slot0 = D > 0 ? (int)((uint32_t)(t1 - n) % (uint32_t)D) : 0;
    auto wrow = [&](int r) -> int64_t {
        int slot = slot0 + r;
        slot = slot >= D ? slot - D : slot;
        return ((int64_t)slot * S + e) * M1;
    };
    // DEC with a register window: the dynamics wave, whose own loads land
    // ~1.4 us before the window wave's (profiles/r06/split_dec), loads the
    // window rows RW .. RWN-1 and writes their tile words; the window wave the
    // rest.  RW = 6 of 9 measured fastest (Backlog 65 536 8.13 -> 7.81 us,
    // LostSales 32 768 6.19 -> 5.99 us; RW = 4, 5, 7 in between).  rmax: the last row that holds a logged order (earlier periods
    // re-read it: straight-line loads, entries past nw unused)
#ifndef INVSIM_IM_SPLIT_RW
#define INVSIM_IM_SPLIT_RW 6
#endif
    constexpr int RWN = WL / M1;
    constexpr int RW = INVSIM_IM_SPLIT_RW < RWN ? INVSIM_IM_SPLIT_RW : RWN;
    constexpr int WD = (RWN - RW) * M1 > 0 ? (RWN - RW) * M1 : 1;
    const bool wsplit = DEC && wreg && RW < RWN;
    const int u_dyn = wsplit ? RW * M1 : WL;   // log entries u_dyn <= u < nw: the dynamics wave's
    const int rmax = nw > 0 ? nw / M1 - 1 : 0;
    if (demand_wave) {
        const int64_t ee = valid ? e : N - 1;        // padded lanes: the last env's stream
        TableStage ts;
        RG g;
        uint64_t u32 = 0;
        int64_t d = 0;
        if (AHEAD) {
            if (!DEC) d = (int64_t)Acur[2 * S + ee];   // (DEC: the dynamics wave loads it)
        } else {
            ts = stage_table(lane);
            P.cm.rng.load(ee, g);
            g.set_step(P.cm.ph_step);
            g.sub(0);
            if (NPD && !RG::kCounter) u32 = P.cm.u32buf[ee];
        }
        uint32_t wv[WL];
        {
#pragma unroll
            for (int r = 0; r < RWN; r++) {
#ifdef INVSIM_ABL_NO_WINDOW   // profiling ablation build only (wrong results): no window read
#pragma unroll
                for (int i = 0; i < M1; i++) wv[r * M1 + i] = (uint32_t)(r + i);
#else
                if (r < RW || !wsplit) {
                    const uint32_t *src = P.alog32 + wrow(r < rmax ? r : rmax);
#pragma unroll
                    for (int i = 0; i < M1; i++) wv[r * M1 + i] = src[i];
                } else {
#pragma unroll
                    for (int i = 0; i < M1; i++) wv[r * M1 + i] = 0;   // (the dynamics wave's rows)
                }
#endif
            }
        }
        if (!AHEAD) {
            ts.flush(lane);
            d = draw(g, u32);
        }
        if (!DEC) dsh[lane] = d;
        if (D > 0) {   // the window part of the obs rows; the newest row is the dynamics wave's
            if (wreg) {
                bool wide = false;
#pragma unroll
                for (int u = 0; u < WL; u++) {
                    // (not the newest row, nw .. nw + M1 - 1: the dynamics wave
                    // writes it, with no barrier in between under DEC)
                    // (nor the log entries u_dyn .. nw - 1: the dynamics wave's under wsplit)
                    if (u < (D - 1) * M1 && !(u >= nw && u < nw + M1) && !(u >= u_dyn && u < nw))
                        w[u] = (u < nw) ? (int64_t)wv[u] : 0;
                    wide |= (u < nw) && (u < u_dyn) && wv[u] == IM_WIDE;
                }
                if (wide) {
#pragma unroll
                    for (int u = 0; u < WL; u++)
                        if (u < nw && u < u_dyn && wv[u] == IM_WIDE) w[u] = P.alog[wrow(u / M1) + u % M1];
                }
                if (n < D)
                    for (int q = (D - 1) * M1; q < D * M1; q++) w[q] = 0;
            } else {
                for (int q = 0; q < nw; q++) w[q] = alog_get(P, wrow(q / M1) + q % M1);
                for (int q = n * M1; q < D * M1; q++) w[q] = 0;
            }
        }
        if (!DEC) wg_lds_sync();   // d -> dynamics wave
        if (DEC) TWAIT();  // (TIMING build: probe 6 after the window rows land)
        TPROBE(6);       // the window wave past its first barrier (DEC: window rows in)
        if constexpr (!RG::kCounter) {
            if (!AHEAD && valid) {   // committed generator state: after this step's draw
                if (Acur) {          // into slot cur (the committed slot once the slots flip)
                    st_store(Acur + e, g.hi);
                    st_store(Acur + S + e, g.lo);
                    if (NPD) st_store(Acur + 3 * S + e, u32);
                } else {
                    P.cm.rng.store_state(e, g);
                    if (NPD) P.cm.u32buf[e] = u32;
                }
            }
        }
        wg_lds_sync();   // tile complete
        store_tile<(M1 * 11 * WAVE * 8 / 2 + 16 * WAVE - 1) / (16 * WAVE)>(im_tile, io.obs + e0 * O,
                                                                          thalf < tcount ? thalf : tcount, lane);
        if (!AHEAD && Anxt) {    // lookahead after an inline draw (first step after invalidation)
            if constexpr (RG::kCounter) {
                g.set_step(P.cm.ph_step + 1);
                g.sub(0);
                u32 = 0;
            }
            const int64_t dn = draw(g, u32);
            if (valid) {
                if constexpr (!RG::kCounter) {
                    st_store(Anxt + e, g.hi);
                    st_store(Anxt + S + e, g.lo);
                    if (NPD) st_store(Anxt + 3 * S + e, u32);
                }
                st_store(Anxt + 2 * S + e, (uint64_t)dn);
            }
        }
        TWAIT();
        TPROBE(5);   // the window wave's exit
        return;
    }
    // ---- dynamics wave
    TPROBE_AT(3, WAVE);
    const double apow = P.alpha_pow[t];
    const int64_t *arow = io.act + (valid ? e : N - 1) * M1;
    // episode sink (kernels.hpp EpSink): the running return and the group's
    // partials are loaded with the step's other loads
    double *const ep_part = P.cm.ep_ret ? P.cm.ep_part + 4 * (e0 / WAVE) : nullptr;
    EpPart epp;
    double ep_r = 0.0;
    if (ep_part) {
        epp.load(ep_part);
        ep_r = P.cm.ep_ret[valid ? e : N - 1];
    }
    int64_t req[M1], arr[M1], I[M1], B[M1 + 1];
    // DEC: this step's demand straight from the lookahead slot, so the dynamics
    // wave does not wait for the window wave's loads before its arithmetic
    const int64_t d_ahead = DEC ? (int64_t)Acur[2 * S + (valid ? e : N - 1)] : 0;
    uint32_t wd[WD];   // wsplit: window rows RW .. RWN-1
    if (wsplit) {
#pragma unroll
        for (int r = RW; r < RWN; r++) {
#ifdef INVSIM_ABL_NO_WINDOW
#pragma unroll
            for (int i = 0; i < M1; i++) wd[(r - RW) * M1 + i] = (uint32_t)(r + i);
#else
            const uint32_t *src = P.alog32 + wrow(r < rmax ? r : rmax);
#pragma unroll
            for (int i = 0; i < M1; i++) wd[(r - RW) * M1 + i] = src[i];
#endif
        }
    }
#pragma unroll
    for (int i = 0; i < M1; i++) req[i] = arow[i];
#pragma unroll
    for (int i = 0; i < M1; i++) {                                  // arrivals R[t-L_i] (:271-277)
        const int L = P.L[i];
        const int row = L > 0 ? P.ring_off[i] + (int)((uint32_t)t % (uint32_t)L) : 0;
        arr[i] = P.Rring[(int64_t)row * S + e];
        if (!(L > 0 && t >= L)) arr[i] = 0;
    }
#pragma unroll
    for (int i = 0; i < M1; i++) I[i] = P.I[i * S + e];
#pragma unroll
    for (int q = 0; q <= M1; q++) B[q] = BACKLOG ? P.B[q * S + e] : 0;
    int64_t ordreq[M1], R[M1], Icur[M1];
#pragma unroll
    for (int i = 0; i < M1; i++) req[i] = req[i] > 0 ? req[i] : 0;  // :250
#pragma unroll
    for (int i = 0; i < M1; i++) {
        ordreq[i] = wrap_add(req[i], B[i + 1]);                     // :253-255
        const int64_t r = ordreq[i] < P.c[i] ? ordreq[i] : P.c[i];  // :263
        R[i] = (i + 1 < M1) ? min_via_f64(r, I[i + 1]) : (int64_t)(double)r;   // :260-265
    }
#pragma unroll
    for (int i = 0; i < M1; i++) Icur[i] = wrap_add(I[i], P.L[i] == 0 ? R[i] : arr[i]);
#pragma unroll
    for (int i = 1; i < M1; i++) Icur[i] = wrap_sub(Icur[i], R[i]); // :300 (reference quirk, kept)
    int64_t Sv[M1 + 1], U[M1 + 1];
#pragma unroll
    for (int i = 0; i < M1; i++) {
        Sv[i + 1] = R[i];                                           // :295
        U[i + 1] = wrap_sub(ordreq[i], R[i]);                       // :304
    }
    if (!DEC) wg_lds_sync();   // d from the demand wave
    if (DEC) TWAIT();     // (TIMING build: probe 1 after the loads land)
    TPROBE_AT(1, WAVE);   // the dynamics wave: loads in, d handed over
    const int64_t d = DEC ? d_ahead : dsh[lane];
    const int64_t dfill = wrap_add(d, B[0]);                        // :284-286
    const int64_t s0 = Icur[0] < dfill ? Icur[0] : dfill;           // :288
    Icur[0] = wrap_sub(Icur[0], s0);
    Sv[0] = s0;
    U[0] = wrap_sub(dfill, s0);                                     // :303
    double term[M1 + 1];                                            // :315-321
#pragma unroll
    for (int q = 0; q <= M1; q++) {
        const double Sj = (double)Sv[q];
        const int64_t inv = (q < M1) ? Icur[q] : 0;
        const double hold = P.hc[q] * (double)(inv > 0 ? inv : 0);
        term[q] = ((P.up[q] * Sj - P.uc[q] * Sj) - hold) - P.kc[q] * (double)U[q];
    }
    const double profit = np_sum<double>(M1 + 1, [&](int q) { return term[q]; });
    const double reward = apow * profit;                            // :322
#pragma unroll
    for (int i = 0; i < M1; i++) trow[i] = Icur[i];                 // obs (:354-391)
    if (D > 0) {
#pragma unroll
        for (int i = 0; i < M1; i++) w[(n - 1) * M1 + i] = req[i];  // newest row last (:380)
    }
    if (wsplit) {   // its window rows (an entry >= 2^32 - 1 from the int64 side ring)
#pragma unroll
        for (int j = 0; j < (RWN - RW) * M1; j++) {
            const int u = RW * M1 + j;
            if (u < nw) w[u] = wd[j] == IM_WIDE ? P.alog[wrow(u / M1) + u % M1] : (int64_t)wd[j];
        }
    }
    wg_lds_sync();   // tile complete
    TPROBE_AT(2, WAVE);   // the dynamics wave: step computed, stores next
    {
        const int64_t h = thalf < tcount ? thalf : tcount;
        if (tcount > h)
            store_tile<(M1 * 11 * WAVE * 8 / 2 + 16 * WAVE - 1) / (16 * WAVE)>(im_tile + h, io.obs + e0 * O + h,
                                                                              tcount - h, lane);
    }
    if (valid) {
        if (P.cm.info_rec) {   // step info (:334-345), as im_step_regs
            constexpr int W = 2 * (M1 + 1) + 5;
            int64_t *rr = (int64_t *)P.cm.info_rec + e * W;
#pragma unroll
            for (int q = 0; q <= M1; q++) {
                rr[q] = Sv[q];
                rr[M1 + 1 + q] = U[q];
            }
            const double rev = np_sum<double>(M1 + 1, [&](int q) { return P.up[q] * (double)Sv[q]; });
            const double pro = np_sum<double>(M1 + 1, [&](int q) { return P.uc[q] * (double)Sv[q]; });
            const double hol = np_sum<double>(M1 + 1, [&](int q) {
                const int64_t inv = (q < M1) ? Icur[q] : 0;
                return P.hc[q] * (double)(inv > 0 ? inv : 0);
            });
            const double pen = np_sum<double>(M1 + 1, [&](int q) { return P.kc[q] * (double)U[q]; });
            rr[2 * (M1 + 1) + 0] = __double_as_longlong(profit);
            rr[2 * (M1 + 1) + 1] = __double_as_longlong(rev);
            rr[2 * (M1 + 1) + 2] = __double_as_longlong(pro);
            rr[2 * (M1 + 1) + 3] = __double_as_longlong(hol);
            rr[2 * (M1 + 1) + 4] = __double_as_longlong(pen);
        }
        ImPending<M1> pend;
#pragma unroll
        for (int i = 0; i < M1; i++) {
            pend.R[i] = R[i];                                           // ring slot t mod L <- R[t] (:267)
            pend.req[i] = req[i];                                       // action_log[t] (:268)
        }
        pend.t = t;
        im_flush_pending<M1>(P, pend, e);
        out_store(io.rew + e, reward);
        out_store(io.term + e, (uint8_t)0);
        out_store(io.trunc + e, (uint8_t)(t1 >= P.periods ? 1 : 0));   // :350
        if (P.cm.info_demand) P.cm.info_demand[e] = d;
#pragma unroll
        for (int i = 0; i < M1; i++) st_store(P.I + i * S + e, Icur[i]);   // :326
        if (BACKLOG) {
#pragma unroll
            for (int q = 0; q <= M1; q++) st_store(P.B + q * S + e, U[q]);   // :307-312
        }
    }
    if (ep_part) {   // after the stores: the butterfly runs while they drain
        EpLane a;
        if (valid) {
            a.r = ep_r;
            a.add(reward, t1 >= P.periods);               // terminated is always False (:350)
            P.cm.ep_ret[e] = a.r;
        }
        epp.flush(ep_part, a, t1 >= P.periods, lane);
    }
    TWAIT();
    TPROBE_AT(4, WAVE);   // the dynamics wave's exit (probe 3: its entry)
}

// K-step lock-step rollout (invsim_rollout, NEXT_STEP or DISABLED autoreset,
// Poisson demand) for 3 stages with compile-time lead times L0..L2 (the
// reference default [1, 5, 10]), one 128-thread workgroup per 64 envs:
//   wave 0 (demand)   draws the demands into an LDS ring of RD chunks of CH
//                     launch steps, ahead of the dynamics wave, as a flat
//                     per-lane loop (stream_flat_loop); a demand is a function
//                     of the env's stream only, and a NEXT_STEP reset step
//                     draws nothing (reset(), :186-222)
//   wave 1 (dynamics) the step (:224-352) with every window in registers,
//                     aligned by age: the fulfilled-order history of stage i
//                     (rw_i[a] = R[t - L_i + a], so the arrival is rw_i[0]) and
//                     the requested-order rows of the observation window
//                     (wv[a] = action_log[t - (D - 1) + a]).  A step reads only
//                     its actions (prefetched a step ahead) and writes the obs
//                     tile, reward, flags and the new ring slots (so the rings
//                     stay exact for every other kernel).
// Chunk handoff (c = 0, 1, ...): the demand wave fills buffer c & 1, then
// barrier c; the dynamics wave consumes chunk c after barrier c, so the
// demand wave's refill of a buffer follows the dynamics wave's use of it.
// Same arithmetic, in the same order, as im_step_regs.
// The demand wave of the rollout kernels (stream_flat_loop): Poisson demand
// (:280) of each launch step into the ring dbuf [RD * CH][WAVE], nb barriers
template <int CH, int RD, class RG, class Stage = NoStage>
__device__ __forceinline__ void im_stream_loop(const ImParams &P, RG &g, const double *rhs_l, int64_t *dbuf,
                                               int lane, int K, int nb, int t_start, Stage stage = Stage()) {
    StreamPos<RG> pos(P.cm.ph_step);
    stream_flat_loop<CH, RD, 1>(
        K, nb, t_start, P.periods,
        [&](int j, int, int64_t &d) {
#ifdef INVSIM_ABL_ROLL_NO_DRAW
            d = 20;
            return true;
#else
            pos.at(g, j, 0);
            return np_poisson_try(g, P.pc, rhs_l, d);
#endif
        },
        [&](int slot, int, int64_t d) { dbuf[slot * WAVE + lane] = d < 0 ? 0 : d; }, stage);
}

// The open-loop rollout's actions of chunk b, staged into the LDS ring
// act_l [2][CH][2 * M1][WAVE] (32-bit halves) by the demand wave with LDS-DMA
// loads (global_load_lds_dword: row q of step kk lands at + q * WAVE, lane l at
// + 4 l): chunk b is read by the dynamics wave between barriers b and b + 1, and
// its buffer (b & 1) was last read before barrier b - 1.
template <int CH, int M1>
struct ImActStage {
    const int64_t *act;
    uint32_t *act_l;
    int64_t N, el;
    int K, nch;
    __device__ __forceinline__ void operator()(int b) const {
        if (b >= nch) return;
#pragma unroll
        for (int kk = 0; kk < CH; kk++) {
            const int k = b * CH + kk;
            if (k < K) {
                const uint32_t *src = reinterpret_cast<const uint32_t *>(act + ((int64_t)k * N + el) * M1);
#pragma unroll
                for (int q = 0; q < 2 * M1; q++)
                    __builtin_amdgcn_global_load_lds(
                        (const void *)(src + q),
                        (__attribute__((address_space(3))) void *)(act_l + (((b & 1) * CH + kk) * 2 * M1 + q) * WAVE),
                        4, 0, 0);
            }
        }
    }
    __device__ __forceinline__ void wait() const { __builtin_amdgcn_s_waitcnt(0); }
};
constexpr int IM_AP_LDS = 256;   // alpha**t LDS table of the 3-role rollout (periods <= this)
// Open-loop actions staged by the demand wave (1) or loaded by the dynamics and
// obs waves themselves (0, the default: LostSales 32 768 envs, 30-step
// launches, 63.1-64.1 us against 64.9-65.5 staged, profiles/r04/stage_ab)
#ifndef IM_ROLL3O_STAGE
#define IM_ROLL3O_STAGE 0
#endif

// demand chunk of im_roll3_kernel: 4 launch steps (round 5; 65 536 envs, K = 30:
// 108.0-109.0 us against 112.1-113.0 with 8, equal at 262 144 envs,
// profiles/r05/roll3_ring/ab.txt; a smaller first chunk starts the dynamics
// wave sooner)
#ifndef IM_ROLL3_CH
#define IM_ROLL3_CH 4
#endif
#ifndef IM_ROLL3_RD
#define IM_ROLL3_RD 4
#endif
template <int L0, int L1, int L2>
struct ImLt3 {
    static constexpr int M1 = 3;
    static constexpr int D = (L0 > L1 ? (L0 > L2 ? L0 : L2) : (L1 > L2 ? L1 : L2));
    static constexpr int O = M1 * (D + 1);
    static constexpr int CH = IM_ROLL3_CH;                               // demand chunk (launch steps)
    static constexpr int RD = IM_ROLL3_RD;                               // demand ring depth (chunks)
    static constexpr int lt(int i) { return i == 0 ? L0 : i == 1 ? L1 : L2; }
    static constexpr int W(int i) { return lt(i) > 0 ? lt(i) : 1; }      // register window length
    static constexpr size_t lds() {   // + the episode sink's [3][WAVE] sums (EpLaneLds)
        return (size_t)WAVE * O * 8 + RHS_LDS_MAX * 8 + (size_t)RD * CH * WAVE * 8 + 3 * WAVE * 8;
    }
};

// POL (invsim_rollout_policy with BASE_STOCK or CONSTANT): the dynamics wave
// computes each step's order from its registers instead of loading it --
// BaseStockAgent.get_action (benchmark_InvManagementBacklogEnv.py:152-198) needs
// I[t] and the requested orders of the last L_i periods, ages 1 .. L_i of the
// window it already holds (plus the age-D row, wold) -- every output is
// optional, and the evaluate_agent sums accumulate in registers (as
// im_launch_step / im_step_regs, same order).
// waves_per_eu(2): at most 256 registers in all, so two dynamics waves share a
// SIMD (the policy variant sits at 256 VGPRs, and the compiler would otherwise
// take AGPRs beyond them: one wave per SIMD, measured 104 -> 166 us)
template <int L0, int L1, int L2, bool BACKLOG, bool POL, class RG = Pcg>
__global__ void __launch_bounds__(2 * WAVE) __attribute__((amdgpu_waves_per_eu(2)))
im_roll3_kernel(ImParams P, int t_start, StepIO<int64_t, int64_t> io, PolicyIO pol, int g0) {
    using G = ImLt3<L0, L1, L2>;
    constexpr int M1 = G::M1, D = G::D, O = G::O, CH = G::CH;
    extern __shared__ __attribute__((aligned(16))) int64_t im_tile[];
    double *rhs_l = reinterpret_cast<double *>(im_tile + WAVE * O);
    int64_t *dbuf = reinterpret_cast<int64_t *>(rhs_l + RHS_LDS_MAX);   // [RD * CH][WAVE]
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const int64_t e0 = ((int64_t)blockIdx.x + g0) * WAVE;   // g0: the launch's first group
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int64_t el = valid ? e : N - 1;          // padded lanes: the last env's data, never stored
    const int nvalid = (int)((N - e0) < WAVE ? (N - e0) : WAVE);
    const int K = io.K;
    const int nch = (K + CH - 1) / CH;
    if (threadIdx.x < WAVE) {   // ---- demand wave
        TableStage ts;
        ts.dst = rhs_l;
        {
            const bool has_tab = P.pc.nk > 0;
            const double *tsrc = has_tab ? P.rhs : P.alpha_pow;   // any valid pointer
            const int qm = has_tab ? P.pc.nk - 1 : 0;
#pragma unroll
            for (int u = 0; u < TableStage::NT; u++) ts.v[u] = tsrc[min(lane + u * WAVE, qm)];
        }
        RG g;
        P.cm.rng.load(el, g);
        ts.flush(lane);
        im_stream_loop<CH, G::RD>(P, g, rhs_l, dbuf, lane, K, nch, t_start);   // barriers 0 .. nch - 1
        if (valid) P.cm.rng.store_state(e, g);
        return;
    }
    // ---- dynamics wave
    int64_t *trow = im_tile + (int64_t)lane * O;
    int t = t_start;
    int64_t I[M1], B[M1 + 1];
#pragma unroll
    for (int i = 0; i < M1; i++) I[i] = P.I[i * S + el];
#pragma unroll
    for (int q = 0; q <= M1; q++) B[q] = BACKLOG ? P.B[q * S + el] : 0;
    // fulfilled-order windows: rw_i[a] = R[t - L_i + a] from ring slot (t + a) mod L_i
    // (rows older than the episode are masked at use by t >= L_i)
    int64_t rw[M1][D > 0 ? D : 1];                 // stage i uses rw[i][0 .. W(i))
#pragma unroll
    for (int i = 0; i < M1; i++) {
#pragma unroll
        for (int a = 0; a < G::W(i); a++) {
            const int L = G::lt(i);
            rw[i][a] = L > 0 ? P.Rring[(int64_t)(P.ring_off[i] + (int)((uint32_t)(t + a) % (uint32_t)L)) * S + el] : 0;
        }
    }
    // requested-order rows: wv[a] = action_log[t - (D - 1) + a], slot (t + 1 + a) mod D
    int64_t wv[D > 1 ? D - 1 : 1][M1];
#pragma unroll
    for (int a = 0; a + 1 < D; a++) {
        const int64_t base = ((int64_t)((uint32_t)(t + 1 + a) % (uint32_t)D) * S + el) * M1;
#pragma unroll
        for (int i = 0; i < M1; i++) {
            const uint32_t v = P.alog32[base + i];
            wv[a][i] = (int64_t)v;
            if (v == IM_WIDE) wv[a][i] = P.alog[base + i];
        }
    }
    int64_t nact[M1];
#pragma unroll
    for (int i = 0; i < M1; i++) nact[i] = POL ? 0 : io.act[el * M1 + i];
    // POL: the age-D requested-order row (slot t mod D, before step t overwrites it)
    int64_t wold[M1];
#pragma unroll
    for (int i = 0; i < M1; i++) {
        wold[i] = 0;
        if (POL && G::lt(i) == D) wold[i] = alog_get(P, ((int64_t)((uint32_t)t % (uint32_t)D) * S + el) * M1 + i);
    }
    constexpr int MD = 6;                                 // metrics (invsim.h INVSIM_METRICS_*)
    double met[MD];
#pragma unroll
    for (int q = 0; q < MD; q++) met[q] = (POL && pol.metrics) ? pol.metrics[el * MD + q] : 0.0;
    double napow = P.alpha_pow[t < P.periods ? t : 0];   // alpha**t of the next step, prefetched
    int64_t dlast = 0;
    bool last_real = false;
    // episode sink (kernels.hpp EpSink), accumulated in registers over the launch;
    // the group's partials are read only after the loop (they would hold 8
    // VGPRs through it: the policy kernel then needs AGPRs, one wave per SIMD)
    double *const ep_part = P.cm.ep_ret ? P.cm.ep_part + 4 * (e0 / WAVE) : nullptr;
    EpLaneLds ep;
    bool ep_done = false;
    if (ep_part) ep.init(reinterpret_cast<double *>(dbuf + G::RD * CH * WAVE), lane, valid ? P.cm.ep_ret[e] : 0.0);
    wg_lds_sync();   // barrier 0: chunk 0 ready
    for (int c = 0; c < nch; c++) {
        const int64_t *db = dbuf + (c % G::RD) * CH * WAVE;
        for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
            const int k = c * CH + kk;
            const int64_t oi = (int64_t)k * N + e;
            int64_t req[M1];
#pragma unroll
            for (int i = 0; i < M1; i++) req[i] = nact[i];
            const double apow = napow;
            {
                const int tn = (t >= P.periods) ? 0 : t + 1;     // the next launch step's period
                napow = P.alpha_pow[tn < P.periods ? tn : 0];
            }
            if (!POL && k + 1 < K) {               // prefetch the next step's actions
#pragma unroll
                for (int i = 0; i < M1; i++) nact[i] = io.act[((int64_t)(k + 1) * N + el) * M1 + i];
            }
            if (t >= P.periods) {                  // NEXT_STEP autoreset (:197-220)
#pragma unroll
                for (int i = 0; i < M1; i++) I[i] = P.I0[i];
#pragma unroll
                for (int q = 0; q <= M1; q++) B[q] = 0;
#pragma unroll
                for (int q = 0; q < O; q++) trow[q] = (q < M1) ? P.I0[q] : 0;
                if (valid && (!POL || io.rew)) {
                    out_store(io.rew + oi, 0.0);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)0);
                }
                if (ep_part) ep.add(0.0, false);   // the reset step's row: reward 0, no flag
                t = 0;
            } else {
                const int64_t d = db[kk * WAVE + lane];
                if (POL) {
                    if (pol.kind == POL_BASE_STOCK) {   // im_base_stock from the register windows
#pragma unroll
                        for (int i = 0; i < M1; i++) {
                            constexpr int DD = D;
                            int64_t pos = I[i];                                 // observation[:M1] = I[t]
                            int64_t pipe = 0;
#pragma unroll
                            for (int a = 1; a <= G::lt(i); a++) {               // action_log[max(0, t - L_i) : t, i]
                                const int64_t v = (a <= DD - 1) ? wv[(DD - 1 - a) >= 0 ? DD - 1 - a : 0][i] : wold[i];
                                if (t - a >= 0) pipe = wrap_add(pipe, v);
                            }
                            if (G::lt(i) > 0) pos = wrap_add(pos, pipe);
                            const double target = ((double)(G::lt(i) + 1) * pol.mu) * pol.sf;
                            double x = target - (double)pos;
                            x = (x > 0) ? x : 0.0;                              // np.maximum(0, .)
                            x = (x < 0.0) ? 0.0 : x;                            // np.clip(., 0, c)
                            x = (x > (double)P.c[i]) ? (double)P.c[i] : x;
                            req[i] = (int64_t)x;
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < M1; i++) req[i] = pol.ci[i];
                    }
                    if (valid && pol.act_out) {
#pragma unroll
                        for (int i = 0; i < M1; i++) out_store((int64_t *)pol.act_out + oi * M1 + i, req[i]);
                    }
                }
                int64_t ordreq[M1], R[M1], Icur[M1];
#pragma unroll
                for (int i = 0; i < M1; i++) req[i] = req[i] > 0 ? req[i] : 0;   // :250
#pragma unroll
                for (int i = 0; i < M1; i++) {
                    ordreq[i] = wrap_add(req[i], B[i + 1]);                     // :253-255
                    const int64_t r = ordreq[i] < P.c[i] ? ordreq[i] : P.c[i];  // :263
                    R[i] = (i + 1 < M1) ? min_via_f64(r, I[i + 1]) : (int64_t)(double)r;   // :260-265
                }
#pragma unroll
                for (int i = 0; i < M1; i++) {                                  // arrivals (:271-277)
                    const int L = G::lt(i);
                    const int64_t arr = (L > 0 && t >= L) ? rw[i][0] : 0;
                    Icur[i] = wrap_add(I[i], L == 0 ? R[i] : arr);
                }
#pragma unroll
                for (int i = 1; i < M1; i++) Icur[i] = wrap_sub(Icur[i], R[i]); // :300 (reference quirk, kept)
                int64_t Sv[M1 + 1], U[M1 + 1];
#pragma unroll
                for (int i = 0; i < M1; i++) {
                    Sv[i + 1] = R[i];                                           // :295
                    U[i + 1] = wrap_sub(ordreq[i], R[i]);                       // :304
                }
                const int64_t dfill = wrap_add(d, B[0]);                        // :284-286
                const int64_t s0 = Icur[0] < dfill ? Icur[0] : dfill;           // :288
                Icur[0] = wrap_sub(Icur[0], s0);
                Sv[0] = s0;
                U[0] = wrap_sub(dfill, s0);                                     // :303
                double term[M1 + 1];                                            // :315-321
#pragma unroll
                for (int q = 0; q <= M1; q++) {
                    const double Sj = (double)Sv[q];
                    const int64_t inv = (q < M1) ? Icur[q] : 0;
                    const double hold = P.hc[q] * (double)(inv > 0 ? inv : 0);
                    term[q] = ((P.up[q] * Sj - P.uc[q] * Sj) - hold) - P.kc[q] * (double)U[q];
                }
                const double profit = np_sum<double>(M1 + 1, [&](int q) { return term[q]; });
                const double reward = apow * profit;                            // :322
                if (POL) {   // evaluate_agent metrics (benchmark_InvManagementBacklogEnv.py:378-399)
                    met[2] += (double)d;                                        // demand_realized
                    met[3] += (double)Sv[0];                                    // sales[0]
                    met[4] += (double)U[0];                                     // unfulfilled[0]
                    int64_t es = 0;                                             // sum(max(0, ending_inventory))
#pragma unroll
                    for (int i = 0; i < M1; i++) es = wrap_add(es, Icur[i] > 0 ? Icur[i] : 0);
                    met[5] += (double)es;
                    met[0] += reward;                                           // episode_reward += reward
                    met[1] += 1.0;                                              // episode_steps
                }
                // observation (:354-391): I, then the window rows t+1-n .. t, zeros after
                const int n = (t + 1 < D) ? t + 1 : D;
#pragma unroll
                for (int i = 0; i < M1; i++) trow[i] = Icur[i];
#pragma unroll
                for (int a = 0; a + 1 < D; a++) {
                    const int r = a - D + n;                                    // obs row of wv[a]
                    if (r >= 0) {
#pragma unroll
                        for (int i = 0; i < M1; i++) trow[M1 + r * M1 + i] = wv[a][i];
                    }
                }
#pragma unroll
                for (int i = 0; i < M1; i++) trow[M1 + (n - 1) * M1 + i] = req[i];
                for (int q = M1 + n * M1; q < O; q++) trow[q] = 0;
                // the new ring slots: R[t] (:267), action_log[t] (:268)
                if (valid) {
#pragma unroll
                    for (int i = 0; i < M1; i++) {
                        const int L = G::lt(i);
                        if (L > 0) st_store(P.Rring + (int64_t)(P.ring_off[i] + (int)((uint32_t)t % (uint32_t)L)) * S + e, R[i]);
                    }
                    const int64_t wb = ((int64_t)((uint32_t)t % (uint32_t)D) * S + e) * M1;
#pragma unroll
                    for (int i = 0; i < M1; i++) {
                        const bool wide = req[i] >= (int64_t)IM_WIDE;
                        st_store(P.alog32 + wb + i, wide ? IM_WIDE : (uint32_t)req[i]);
                        if (wide) st_store(P.alog + wb + i, req[i]);
                    }
                    if (!POL || io.rew) {
                        out_store(io.rew + oi, reward);
                        out_store(io.term + oi, (uint8_t)0);
                        out_store(io.trunc + oi, (uint8_t)(t + 1 >= P.periods ? 1 : 0));   // :350
                    }
                }
                if (ep_part) {
                    const bool done = valid && t + 1 >= P.periods;
                    ep.add(valid ? reward : 0.0, done);
                    ep_done |= done;
                }
                // age the windows by one period
#pragma unroll
                for (int i = 0; i < M1; i++) {
                    const int L = G::lt(i);
                    if (L > 0) {
#pragma unroll
                        for (int a = 0; a + 1 < G::W(i); a++) rw[i][a] = rw[i][a + 1];
                        rw[i][G::W(i) - 1] = R[i];
                    }
                }
                if (POL && D > 1) {
#pragma unroll
                    for (int i = 0; i < M1; i++) wold[i] = wv[0][i];             // age D - 1 -> age D
                }
#pragma unroll
                for (int a = 0; a + 2 < D; a++) {
#pragma unroll
                    for (int i = 0; i < M1; i++) wv[a][i] = wv[a + 1][i];
                }
                if (D > 1) {
#pragma unroll
                    for (int i = 0; i < M1; i++) wv[D - 2][i] = req[i];
                }
#pragma unroll
                for (int i = 0; i < M1; i++) I[i] = Icur[i];                    // :326
#pragma unroll
                for (int q = 0; q <= M1; q++) B[q] = BACKLOG ? U[q] : 0;        // :307-312
                dlast = d;
                last_real = k == K - 1;
                t += 1;
            }
            wave_lds_sync();
#ifndef INVSIM_ABL_ROLL_NO_STORE
            if (!POL || io.obs)
                store_tile<(O * WAVE * 8 + 16 * WAVE - 1) / (16 * WAVE)>(im_tile, io.obs + ((int64_t)k * N + e0) * O,
                                                                        (int64_t)nvalid * O, lane);
#endif
            wave_lds_sync();
        }
        if (c + 1 < nch) wg_lds_sync();   // barrier c + 1
    }
    if (valid) {
#pragma unroll
        for (int i = 0; i < M1; i++) st_store(P.I + i * S + e, I[i]);
        if (BACKLOG) {
#pragma unroll
            for (int q = 0; q <= M1; q++) st_store(P.B + q * S + e, B[q]);
        }
        if (P.cm.info_demand && last_real) P.cm.info_demand[e] = dlast;
        if (POL && pol.metrics) {
#pragma unroll
            for (int q = 0; q < MD; q++) pol.metrics[e * MD + q] = met[q];
        }
        if (ep_part) P.cm.ep_ret[e] = ep.r;
    }
    if (ep_part) {
        EpPart epp;
        epp.load(ep_part);
        epp.flush(ep_part, ep.get(), __ballot(ep_done) != 0, lane);
    }
}

// im_roll3_kernel with the observation work moved to a third wave (for small
// batches, where a dynamics wave has a SIMD to itself and its instruction
// chain is the step time): one 192-thread workgroup per 64 envs, three roles
// pipelined over chunks of CH launch steps:
//   wave 0 (demand)   draws the demands up to RD chunks ahead into an LDS
//                     ring (stream_flat_loop); a demand is a function of the
//                     env's stream only, and a NEXT_STEP reset step draws
//                     nothing (:186-222)
//   wave 1 (dynamics) consumes chunk c: the step (:224-352) with the
//                     fulfilled-order history in registers aligned by age
//                     (rw_i[a] = R[t - L_i + a], so the arrival is rw_i[0]);
//                     stores reward, flags, the new R ring slots, and hands the
//                     end-of-step inventory of every step to wave 2 in LDS
//   wave 2 (obs)      builds the observations of chunk c - 1: the inventory
//                     from wave 1, the requested-order rows from its own copy
//                     of the actions (wv[a] = action_log[t - (D - 1) + a], in
//                     registers), the obs tile store, and the action_log ring
// Each role's next step's actions / alpha**t are loaded a step ahead, before
// the previous step's stores (vmcnt is in order).  One barrier per chunk: the
// demand wave fills dbuf[c & 1] before barrier c, the dynamics wave consumes it
// between barriers c and c + 1 and fills ibuf[c & 1], which the obs wave
// consumes between barriers c + 1 and c + 2.  Same arithmetic, in the same
// order, as im_step_regs.
#ifndef IM_ROLL3O_CH
#define IM_ROLL3O_CH 2   // swept on MI355X (LostSales 32768 envs): (CH, RD) = (2, 8) 65.6 us, (4, 4) 67.0, (4, 8) 66.5, (8, 4) 74.6
#endif
#ifndef IM_ROLL3O_RD
#define IM_ROLL3O_RD 8
#endif
template <int L0, int L1, int L2>
struct ImLt3o : ImLt3<L0, L1, L2> {
    static constexpr int CH = IM_ROLL3O_CH;                              // chunk (launch steps)
    static constexpr int RD = IM_ROLL3O_RD;                              // demand ring depth (chunks)
    static constexpr int M1 = 3, O = ImLt3<L0, L1, L2>::O;
    // tile, RHS table, demand ring, ibuf [2][CH][M1][WAVE] (inventory, dynamics ->
    // obs wave), abuf [2][CH][M1][WAVE] (requested orders, dynamics -> obs wave;
    // only with POL or staging), act_l [2][CH][2 M1][WAVE] u32 (actions, demand ->
    // dynamics wave; only when staging open-loop actions), alpha**t
    static constexpr size_t abuf_n(bool pol) { return (pol || IM_ROLL3O_STAGE) ? (size_t)2 * CH * M1 * WAVE : 0; }
    static constexpr size_t actl_n(bool pol) { return (IM_ROLL3O_STAGE && !pol) ? (size_t)2 * CH * 2 * M1 * WAVE : 0; }
    static constexpr size_t lds(bool pol) {
        return (size_t)WAVE * O * 8 + RHS_LDS_MAX * 8 + (size_t)RD * CH * WAVE * 8 + (size_t)2 * CH * M1 * WAVE * 8 +
               abuf_n(pol) * 8 + actl_n(pol) * 4 + IM_AP_LDS * 8 + 3 * WAVE * 8;   // + EpLaneLds sums
    }
};

// POL (invsim_rollout_policy, BASE_STOCK / CONSTANT): the dynamics wave
// computes each step's order from I and its own register history of the last
// L_i orders per stage (hv), and hands the orders to the obs wave in LDS (abuf)
// beside the inventory; outputs optional, metrics in registers (as im_roll3_kernel).
// G2 = 2 (INVSIM_IM_ROLL3O_G2=1, A/B): two 64-env groups per 6-wave
// workgroup.  The dispatcher puts waves w and w + 4 of a 6-wave workgroup on
// one SIMD and waves 2 and 3 on a SIMD each (tools/wave_placement,
// profiles/r03/launch/placement.txt), so the two dynamics waves take waves 2
// and 3 and every demand wave shares its SIMD with the other group's obs wave.
template <int L0, int L1, int L2, bool BACKLOG, bool POL, class RG = Pcg, int G2 = 1>
__global__ void __launch_bounds__(3 * WAVE * G2)
im_roll3o_kernel(ImParams P, int t_start, StepIO<int64_t, int64_t> io, PolicyIO pol) {
    using G = ImLt3o<L0, L1, L2>;
    constexpr int M1 = G::M1, D = G::D, O = G::O, CH = G::CH;
    extern __shared__ __attribute__((aligned(16))) int64_t im_lds3o[];
    const int w = threadIdx.x / WAVE;
    // G2 = 2: wave -> (role, group) = 0 (0,0) 1 (0,1) 2 (1,0) 3 (1,1) 4 (2,1) 5 (2,0)
    const int role = G2 == 1 ? w : (w >> 1);
    const int grp = G2 == 1 ? 0 : (w < 4 ? (w & 1) : ((w & 1) ^ 1));
    int64_t *im_tile = im_lds3o + (int64_t)grp * (int64_t)(G::lds(POL) / sizeof(int64_t));
    double *rhs_l = reinterpret_cast<double *>(im_tile + WAVE * O);
    int64_t *dbuf = reinterpret_cast<int64_t *>(rhs_l + RHS_LDS_MAX);   // [RD * CH][WAVE]
    int64_t *ibuf = dbuf + G::RD * CH * WAVE;                             // [2][CH][M1][WAVE]
    int64_t *abuf = ibuf + 2 * CH * M1 * WAVE;                            // [2][CH][M1][WAVE] (POL / staged)
    uint32_t *act_l = reinterpret_cast<uint32_t *>(abuf + G::abuf_n(POL));  // [2][CH][2 M1][WAVE] (staged)
    double *ap_l = reinterpret_cast<double *>(act_l + G::actl_n(POL));      // alpha**t, t < periods
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const int64_t e0 = ((int64_t)blockIdx.x * G2 + grp) * WAVE;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int64_t el = valid ? e : N - 1;          // padded lanes: the last env's data, never stored
    const int nvalid = (int)((N - e0) < WAVE ? (N - e0) : WAVE);
    const int K = io.K;
    const int nch = (K + CH - 1) / CH;
    TPROBE_W(0);
    TPROBE_W_ID();
    if (role == 0) {   // ---- demand wave
        TableStage ts;
        ts.dst = rhs_l;
        {
            const bool has_tab = P.pc.nk > 0;
            const double *tsrc = has_tab ? P.rhs : P.alpha_pow;   // any valid pointer
            const int qm = has_tab ? P.pc.nk - 1 : 0;
#pragma unroll
            for (int u = 0; u < TableStage::NT; u++) ts.v[u] = tsrc[min(lane + u * WAVE, qm)];
        }
        RG g;
        P.cm.rng.load(el, g);
        for (int q = lane; q < P.periods; q += WAVE) ap_l[q] = P.alpha_pow[q];   // before barrier 0
        ts.flush(lane);
        // barriers 0 .. nch - 1 (demand chunk c ready), nch (the obs wave's last chunk)
        if (POL || !IM_ROLL3O_STAGE) {
            im_stream_loop<CH, G::RD>(P, g, rhs_l, dbuf, lane, K, nch + 1, t_start);
        } else {
            const ImActStage<CH, M1> stage{io.act, act_l, N, el, K, nch};
            im_stream_loop<CH, G::RD>(P, g, rhs_l, dbuf, lane, K, nch + 1, t_start, stage);
        }
        if (valid) P.cm.rng.store_state(e, g);
        TWAIT();
        TPROBE_W(6);
        return;
    }
    if (role == 2) {   // ---- obs wave
        int64_t *trow = im_tile + (int64_t)lane * O;
        int t = t_start;
        // requested-order rows: wv[a] = action_log[t - (D - 1) + a], slot (t + 1 + a) mod D
        int64_t wv[D > 1 ? D - 1 : 1][M1];
#pragma unroll
        for (int a = 0; a + 1 < D; a++) {
            const int64_t base = ((int64_t)((uint32_t)(t + 1 + a) % (uint32_t)D) * S + el) * M1;
#pragma unroll
            for (int i = 0; i < M1; i++) {
                const uint32_t v = P.alog32[base + i];
                wv[a][i] = (int64_t)v;
                if (v == IM_WIDE) wv[a][i] = P.alog[base + i];
            }
        }
        constexpr bool HANDED = POL || IM_ROLL3O_STAGE;   // requested orders from the dynamics wave
        int64_t nact[M1];
#pragma unroll
        for (int i = 0; i < M1; i++) nact[i] = HANDED ? 0 : io.act[el * M1 + i];
        wg_lds_sync();   // barrier 0
        for (int c = 0; c < nch; c++) {
            wg_lds_sync();   // barrier c + 1: inventory chunk c ready
            const int64_t *ib = ibuf + (c & 1) * CH * M1 * WAVE;
            const int64_t *ab = abuf + (c & 1) * CH * M1 * WAVE;
            for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
                const int k = c * CH + kk;
                int64_t req[M1];
#pragma unroll
                for (int i = 0; i < M1; i++) req[i] = HANDED ? ab[(kk * M1 + i) * WAVE + lane] : nact[i];
                if (!HANDED && k + 1 < K) {            // the next step's actions
#pragma unroll
                    for (int i = 0; i < M1; i++) nact[i] = io.act[((int64_t)(k + 1) * N + el) * M1 + i];
                }
                if (t >= P.periods) {                  // NEXT_STEP autoreset: [I0, 0...] (:220)
#pragma unroll
                    for (int q = 0; q < O; q++) trow[q] = (q < M1) ? ib[(kk * M1 + q) * WAVE + lane] : 0;
                    t = 0;
                } else {
#pragma unroll
                    for (int i = 0; i < M1; i++) req[i] = req[i] > 0 ? req[i] : 0;   // :250
                    // observation (:354-391): I, then the window rows t+1-n .. t, zeros after
                    const int n = (t + 1 < D) ? t + 1 : D;
#pragma unroll
                    for (int i = 0; i < M1; i++) trow[i] = ib[(kk * M1 + i) * WAVE + lane];
#pragma unroll
                    for (int a = 0; a + 1 < D; a++) {
                        const int r = a - D + n;                                // obs row of wv[a]
                        if (r >= 0) {
#pragma unroll
                            for (int i = 0; i < M1; i++) trow[M1 + r * M1 + i] = wv[a][i];
                        }
                    }
#pragma unroll
                    for (int i = 0; i < M1; i++) trow[M1 + (n - 1) * M1 + i] = req[i];
                    for (int q = M1 + n * M1; q < O; q++) trow[q] = 0;
                    if (valid) {                                                // action_log[t] (:268)
                        const int64_t wb = ((int64_t)((uint32_t)t % (uint32_t)D) * S + e) * M1;
#pragma unroll
                        for (int i = 0; i < M1; i++) {
                            const bool wide = req[i] >= (int64_t)IM_WIDE;
                            st_store(P.alog32 + wb + i, wide ? IM_WIDE : (uint32_t)req[i]);
                            if (wide) st_store(P.alog + wb + i, req[i]);
                        }
                    }
#pragma unroll
                    for (int a = 0; a + 2 < D; a++) {
#pragma unroll
                        for (int i = 0; i < M1; i++) wv[a][i] = wv[a + 1][i];
                    }
                    if (D > 1) {
#pragma unroll
                        for (int i = 0; i < M1; i++) wv[D - 2][i] = req[i];
                    }
                    t += 1;
                }
                wave_lds_sync();
#ifndef INVSIM_ABL_ROLL_NO_STORE
                if (!POL || io.obs)
                    store_tile<(O * WAVE * 8 + 16 * WAVE - 1) / (16 * WAVE)>(im_tile, io.obs + ((int64_t)k * N + e0) * O,
                                                                            (int64_t)nvalid * O, lane);
#endif
                wave_lds_sync();
            }
        }
        TWAIT();
        TPROBE_W(6);
        return;
    }
    // ---- dynamics wave
    int t = t_start;
    int64_t I[M1], B[M1 + 1];
#pragma unroll
    for (int i = 0; i < M1; i++) I[i] = P.I[i * S + el];
#pragma unroll
    for (int q = 0; q <= M1; q++) B[q] = BACKLOG ? P.B[q * S + el] : 0;
    // fulfilled-order windows: rw_i[a] = R[t - L_i + a] from ring slot (t + a) mod L_i
    // (rows older than the episode are masked at use by t >= L_i)
    int64_t rw[M1][D > 0 ? D : 1];                 // stage i uses rw[i][0 .. W(i))
#pragma unroll
    for (int i = 0; i < M1; i++) {
#pragma unroll
        for (int a = 0; a < G::W(i); a++) {
            const int L = G::lt(i);
            rw[i][a] = L > 0 ? P.Rring[(int64_t)(P.ring_off[i] + (int)((uint32_t)(t + a) % (uint32_t)L)) * S + el] : 0;
        }
    }
    // POL: hv[i][a] = action_log[t - 1 - a, i], the last W(i) requested orders of stage i
    int64_t hv[M1][D > 0 ? D : 1];
#pragma unroll
    for (int i = 0; i < M1; i++) {
#pragma unroll
        for (int a = 0; a < G::W(i); a++)
            hv[i][a] = POL ? alog_get(P, ((int64_t)((uint32_t)(t - 1 - a + 256 * D) % (uint32_t)D) * S + el) * M1 + i) : 0;
    }
    constexpr int MD = 6;                                 // metrics (invsim.h INVSIM_METRICS_*)
    double met[MD];
#pragma unroll
    for (int q = 0; q < MD; q++) met[q] = (POL && pol.metrics) ? pol.metrics[el * MD + q] : 0.0;
    constexpr bool STAGED = !POL && IM_ROLL3O_STAGE;
    int64_t nact[M1];
#pragma unroll
    for (int i = 0; i < M1; i++) nact[i] = (POL || STAGED) ? 0 : io.act[el * M1 + i];
    int64_t dlast = 0;
    bool last_real = false;
    // episode sink (kernels.hpp EpSink), accumulated in registers over the launch;
    // the group's partials are read only after the loop (they would hold 8
    // VGPRs through it: the policy kernel then needs AGPRs, one wave per SIMD)
    double *const ep_part = P.cm.ep_ret ? P.cm.ep_part + 4 * (e0 / WAVE) : nullptr;
    EpLaneLds ep;
    bool ep_done = false;
    if (ep_part) ep.init(reinterpret_cast<double *>(ap_l + IM_AP_LDS), lane, valid ? P.cm.ep_ret[e] : 0.0);
    wg_lds_sync();   // barrier 0: demand chunk 0 (and its actions when staged, alpha**t) ready
    for (int c = 0; c < nch; c++) {
        const int64_t *db = dbuf + (c % G::RD) * CH * WAVE;
        int64_t *ib = ibuf + (c & 1) * CH * M1 * WAVE;
        int64_t *ab = abuf + (c & 1) * CH * M1 * WAVE;
        const uint32_t *al = act_l + (c & 1) * CH * 2 * M1 * WAVE;
        for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
            const int k = c * CH + kk;
            const int64_t oi = (int64_t)k * N + e;
            int64_t req[M1];
#pragma unroll
            for (int i = 0; i < M1; i++)
                req[i] = !STAGED ? nact[i]
                                 : (int64_t)((uint64_t)al[(kk * 2 * M1 + 2 * i) * WAVE + lane] |
                                             ((uint64_t)al[(kk * 2 * M1 + 2 * i + 1) * WAVE + lane] << 32));
            if (!POL && !STAGED && k + 1 < K) {    // prefetch the next step's actions
#pragma unroll
                for (int i = 0; i < M1; i++) nact[i] = io.act[((int64_t)(k + 1) * N + el) * M1 + i];
            }
            const double apow = ap_l[t < P.periods ? t : 0];
            if (t >= P.periods) {                  // NEXT_STEP autoreset (:197-220)
#pragma unroll
                for (int i = 0; i < M1; i++) I[i] = P.I0[i];
#pragma unroll
                for (int q = 0; q <= M1; q++) B[q] = 0;
#pragma unroll
                for (int i = 0; i < M1; i++) ib[(kk * M1 + i) * WAVE + lane] = I[i];
                if (valid && (!POL || io.rew)) {
                    out_store(io.rew + oi, 0.0);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)0);
                }
                if (ep_part) ep.add(0.0, false);   // the reset step's row: reward 0, no flag
                t = 0;
            } else {
                const int64_t d = db[kk * WAVE + lane];
                if (POL) {
                    if (pol.kind == POL_BASE_STOCK) {   // im_base_stock from the register history
#pragma unroll
                        for (int i = 0; i < M1; i++) {
                            int64_t pos = I[i];                                 // observation[:M1] = I[t]
                            int64_t pipe = 0;
#pragma unroll
                            for (int a = 0; a < G::lt(i); a++)                  // action_log[max(0, t - L_i) : t, i]
                                if (t - 1 - a >= 0) pipe = wrap_add(pipe, hv[i][a]);
                            if (G::lt(i) > 0) pos = wrap_add(pos, pipe);
                            const double target = ((double)(G::lt(i) + 1) * pol.mu) * pol.sf;
                            double x = target - (double)pos;
                            x = (x > 0) ? x : 0.0;                              // np.maximum(0, .)
                            x = (x < 0.0) ? 0.0 : x;                            // np.clip(., 0, c)
                            x = (x > (double)P.c[i]) ? (double)P.c[i] : x;
                            req[i] = (int64_t)x;
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < M1; i++) req[i] = pol.ci[i];
                    }
                    if (valid && pol.act_out) {
#pragma unroll
                        for (int i = 0; i < M1; i++) out_store((int64_t *)pol.act_out + oi * M1 + i, req[i]);
                    }
                }
                int64_t ordreq[M1], R[M1], Icur[M1];
#pragma unroll
                for (int i = 0; i < M1; i++) req[i] = req[i] > 0 ? req[i] : 0;   // :250
#pragma unroll
                for (int i = 0; i < M1; i++) {
                    ordreq[i] = wrap_add(req[i], B[i + 1]);                     // :253-255
                    const int64_t r = ordreq[i] < P.c[i] ? ordreq[i] : P.c[i];  // :263
                    R[i] = (i + 1 < M1) ? min_via_f64(r, I[i + 1]) : (int64_t)(double)r;   // :260-265
                }
#pragma unroll
                for (int i = 0; i < M1; i++) {                                  // arrivals (:271-277)
                    const int L = G::lt(i);
                    const int64_t arr = (L > 0 && t >= L) ? rw[i][0] : 0;
                    Icur[i] = wrap_add(I[i], L == 0 ? R[i] : arr);
                }
#pragma unroll
                for (int i = 1; i < M1; i++) Icur[i] = wrap_sub(Icur[i], R[i]); // :300 (reference quirk, kept)
                int64_t Sv[M1 + 1], U[M1 + 1];
#pragma unroll
                for (int i = 0; i < M1; i++) {
                    Sv[i + 1] = R[i];                                           // :295
                    U[i + 1] = wrap_sub(ordreq[i], R[i]);                       // :304
                }
                const int64_t dfill = wrap_add(d, B[0]);                        // :284-286
                const int64_t s0 = Icur[0] < dfill ? Icur[0] : dfill;           // :288
                Icur[0] = wrap_sub(Icur[0], s0);
                Sv[0] = s0;
                U[0] = wrap_sub(dfill, s0);                                     // :303
                double term[M1 + 1];                                            // :315-321
#pragma unroll
                for (int q = 0; q <= M1; q++) {
                    const double Sj = (double)Sv[q];
                    const int64_t inv = (q < M1) ? Icur[q] : 0;
                    const double hold = P.hc[q] * (double)(inv > 0 ? inv : 0);
                    term[q] = ((P.up[q] * Sj - P.uc[q] * Sj) - hold) - P.kc[q] * (double)U[q];
                }
                const double profit = np_sum<double>(M1 + 1, [&](int q) { return term[q]; });
                const double reward = apow * profit;                            // :322
                if (POL) {   // evaluate_agent metrics (benchmark_InvManagementBacklogEnv.py:378-399)
                    met[2] += (double)d;                                        // demand_realized
                    met[3] += (double)Sv[0];                                    // sales[0]
                    met[4] += (double)U[0];                                     // unfulfilled[0]
                    int64_t es = 0;                                             // sum(max(0, ending_inventory))
#pragma unroll
                    for (int i = 0; i < M1; i++) es = wrap_add(es, Icur[i] > 0 ? Icur[i] : 0);
                    met[5] += (double)es;
                    met[0] += reward;                                           // episode_reward += reward
                    met[1] += 1.0;                                              // episode_steps
#pragma unroll
                    for (int i = 0; i < M1; i++) {
#pragma unroll
                        for (int a = G::W(i) - 1; a >= 1; a--) hv[i][a] = hv[i][a - 1];
                        hv[i][0] = req[i];
                    }
                }
                if (POL || STAGED) {
#pragma unroll
                    for (int i = 0; i < M1; i++) ab[(kk * M1 + i) * WAVE + lane] = req[i];   // the order -> obs wave
                }
#pragma unroll
                for (int i = 0; i < M1; i++) ib[(kk * M1 + i) * WAVE + lane] = Icur[i];   // obs I (:366)
                // the new fulfilled-order ring slots R[t] (:267)
                if (valid) {
#pragma unroll
                    for (int i = 0; i < M1; i++) {
                        const int L = G::lt(i);
                        if (L > 0) st_store(P.Rring + (int64_t)(P.ring_off[i] + (int)((uint32_t)t % (uint32_t)L)) * S + e, R[i]);
                    }
                    if (!POL || io.rew) {
                        out_store(io.rew + oi, reward);
                        out_store(io.term + oi, (uint8_t)0);
                        out_store(io.trunc + oi, (uint8_t)(t + 1 >= P.periods ? 1 : 0));   // :350
                    }
                }
                if (ep_part) {
                    const bool done = valid && t + 1 >= P.periods;
                    ep.add(valid ? reward : 0.0, done);
                    ep_done |= done;
                }
                // age the windows by one period
#pragma unroll
                for (int i = 0; i < M1; i++) {
                    const int L = G::lt(i);
                    if (L > 0) {
#pragma unroll
                        for (int a = 0; a + 1 < G::W(i); a++) rw[i][a] = rw[i][a + 1];
                        rw[i][G::W(i) - 1] = R[i];
                    }
                }
#pragma unroll
                for (int i = 0; i < M1; i++) I[i] = Icur[i];                    // :326
#pragma unroll
                for (int q = 0; q <= M1; q++) B[q] = BACKLOG ? U[q] : 0;        // :307-312
                dlast = d;
                last_real = k == K - 1;
                t += 1;
            }
        }
        wg_lds_sync();   // barrier c + 1: inventory chunk c ready, demand chunk c + 1 ready
    }
    if (valid) {
#pragma unroll
        for (int i = 0; i < M1; i++) st_store(P.I + i * S + e, I[i]);
        if (BACKLOG) {
#pragma unroll
            for (int q = 0; q <= M1; q++) st_store(P.B + q * S + e, B[q]);
        }
        if (P.cm.info_demand && last_real) P.cm.info_demand[e] = dlast;
        if (POL && pol.metrics) {
#pragma unroll
            for (int q = 0; q < MD; q++) pol.metrics[e * MD + q] = met[q];
        }
        if (ep_part) P.cm.ep_ret[e] = ep.r;
    }
    if (ep_part) {
        EpPart epp;
        epp.load(ep_part);
        epp.flush(ep_part, ep.get(), __ballot(ep_done) != 0, lane);
    }
    TWAIT();
    TPROBE_W(6);
}

// cm.rng <- the committed slot of the lookahead cache (see im_split_kernel)
__global__ void __launch_bounds__(256) im_commit_kernel(ImParams P, int slot) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int64_t S = P.cm.Npad;
    const uint64_t *A = P.ahead + (int64_t)slot * 4 * S;
    P.cm.rng.hi[e] = A[e];
    P.cm.rng.lo[e] = A[S + e];
    if (P.cm.u32buf) P.cm.u32buf[e] = A[3 * S + e];
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// the lock-step split step kernel applies (both streams)
inline bool im_split_applies(const ImParams &p, int t_u, const PolicyIO *pol, const StepIO<int64_t, int64_t> &io) {
    return !pol && io.K == 1 && t_u >= 0 && t_u < p.periods && io.obs &&
           !(p.cm.autoreset == AR_SAME_STEP && t_u + 1 >= p.periods) && p.cm.kn.im_split;
}

// The lock-step NEXT_STEP reset step (one step at t_u >= periods): its output row
// is reward 0 with no flag, whose fold changes nothing (EpLane adds +0.0 to
// returns restarted at +0.0), so the episode sink needs no work for it
inline bool im_sink_noop(const ImParams &p, int t_u, const PolicyIO *pol, const StepIO<int64_t, int64_t> &io) {
    return !pol && io.K == 1 && t_u >= p.periods && p.cm.autoreset == AR_NEXT_STEP;
}

// the 2-/3-role rollout kernels of the reference's default lead times apply
// (open loop, or the in-kernel BaseStock / ConstantOrder agents)
inline bool im_roll_applies(const ImParams &p, int M1, int t_u, const PolicyIO *pol,
                            const StepIO<int64_t, int64_t> &io) {
    const bool pol_roll = pol && (pol->kind == POL_BASE_STOCK || pol->kind == POL_CONSTANT) && p.cm.kn.im_pol_roll;
    return (!pol || pol_roll) && io.K > 1 && t_u >= 0 && p.cm.autoreset != AR_SAME_STEP && p.dist == 1 &&
           !p.cm.info_rec && M1 == 3 && p.L[0] == 1 && p.L[1] == 5 && p.L[2] == 10 && p.lt_max == 10 &&
           p.cm.kn.im_roll;
}

template <class RG>
hipError_t im_roll_launch(const ImParams &p, bool backlog, int t_u, const PolicyIO *pol,
                          const StepIO<int64_t, int64_t> &io, hipStream_t s) {
    PolicyIO none{};
    const PolicyIO &pv = pol ? *pol : none;
    using G = ImLt3<1, 5, 10>;
    using G3 = ImLt3o<1, 5, 10>;
    const dim3 g3(grid_for(p.cm.N, WAVE));
    // up to one 2-role workgroup per SIMD pair (N <= 32768): the dynamics
    // wave's chain is the step time, so split it (measured on MI355X:
    // LostSales 32768 envs 87.5 -> 77.7 us per K = 30; at 65536 the
    // 2-role kernel is faster, 118 vs 152 us)
    const bool three = p.cm.N <= p.cm.kn.im_roll3o_max_n && p.periods <= IM_AP_LDS;   // alpha**t table in LDS
    // two groups per workgroup when the group count is even (every workgroup full)
    // two 64-env groups per 6-wave workgroup: the default for policy rollouts
    // (BaseStock at 32 768 envs: 63.1-64.8 against 66.5-67.7 us per 30 steps),
    // equal open loop (profiles/r03/launch/g2_stage.txt)
    const bool g2 = p.cm.kn.im_roll3o_g2 < 0 ? pol != nullptr : p.cm.kn.im_roll3o_g2 == 1;
    const bool two = three && g2 && (g3.x % 2) == 0;
    const dim3 g6(g3.x / 2);
    // INVSIM_IM_ROLL_SUB (default 65 536): the 2-role rollout as back-to-back
    // launches of at most that many envs (whole 64-env groups), each over its
    // own groups: one round of 1 024 workgroups (four per CU) per launch.
    // Measured at K = 30 (profiles/r06/roll_sub): 262 144 envs 618 -> 564 us,
    // 1 048 576 envs 2 433 -> 2 300 us; sub-launches of 131 072 envs (two
    // rounds each) are slower than one launch, of 16 384 far slower
    const int sub = p.cm.kn.im_roll_sub >= WAVE ? (int)std::min<int64_t>(p.cm.kn.im_roll_sub / WAVE, g3.x) : (int)g3.x;
#define R_(B, POL)                                                                                                    \
    do {                                                                                                              \
        if (two) hipLaunchKernelGGL((im_roll3o_kernel<1, 5, 10, B, POL, RG, 2>), g6, dim3(6 * WAVE), 2 * G3::lds(POL), s, p, t_u, io, pv); \
        else if (three) hipLaunchKernelGGL((im_roll3o_kernel<1, 5, 10, B, POL, RG>), g3, dim3(3 * WAVE), G3::lds(POL), s, p, t_u, io, pv); \
        else                                                                                                          \
            for (int g0 = 0; g0 < (int)g3.x; g0 += sub)                                                               \
                hipLaunchKernelGGL((im_roll3_kernel<1, 5, 10, B, POL, RG>), dim3(min(sub, (int)g3.x - g0)), dim3(2 * WAVE), \
                                   G::lds(), s, p, t_u, io, pv, g0);                                                  \
    } while (0)
    if (pol) {
        if (backlog) R_(true, true);
        else R_(false, true);
    } else {
        if (backlog) R_(true, false);
        else R_(false, false);
    }
#undef R_
    return hipGetLastError();
}

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

#ifdef INVSIM_IM_FAST_TU
// invmgmt_ph.hip: this file compiled a second time for the fast-stream run
// kernels (a TU of their own, so the two instantiation sets compile in parallel)
hipError_t im_run_launch_ph(const ImParams &p, int M1, bool backlog, int t_u, const PolicyIO *pol,
                            const StepIO<int64_t, int64_t> &io, bool &ahead, int &slot, bool &sunk, hipStream_t s) {
    sunk = im_sink_noop(p, t_u, pol, io);
    if (p.cm.N == 0 || io.K <= 0) return hipSuccess;
    const size_t lds = (size_t)EPW * M1 * (p.lt_max + 1) * sizeof(int64_t) + RHS_LDS_MAX * sizeof(double);
    const dim3 grid(grid_for(p.cm.N, EPW)), block(WAVE);
    PolicyIO none{};
    const PolicyIO &pv = pol ? *pol : none;
    const bool npd = p.dist >= 2 && p.dist <= 4;
    if (im_split_applies(p, t_u, pol, io)) {   // the split step kernel, with the demand-only lookahead
        const size_t lds2 = lds + WAVE * sizeof(int64_t);
        ImParams q = p;
        if (!p.cm.kn.im_ahead) q.ahead = nullptr;
        const bool hit = ahead && q.ahead;
        const int gla = hit ? (int)grid_for(p.cm.N, 2 * WAVE) : 0;
        const dim3 grid2(grid.x + gla), block2(2 * WAVE);
        const int cur = slot;
        const int la0 = p.cm.kn.im_la_last ? (int)grid.x : 0;
#define S_(M, B)                                                                                        \
    do {                                                                                                \
        if (npd) {                                                                                      \
            if (hit) hipLaunchKernelGGL((im_split_kernel<M, B, true, true, PhiloxGen>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla);  \
            else hipLaunchKernelGGL((im_split_kernel<M, B, true, false, PhiloxGen>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla);     \
        } else {                                                                                        \
            if (hit) hipLaunchKernelGGL((im_split_kernel<M, B, false, true, PhiloxGen>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla); \
            else hipLaunchKernelGGL((im_split_kernel<M, B, false, false, PhiloxGen>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla);    \
        }                                                                                               \
    } while (0)
        IM_DISPATCH(M1, backlog, S_)
#undef S_
        sunk = true;                  // the split kernel folds into the episode sink (if one is set)
        ahead = q.ahead != nullptr;   // every env drew launch step ph_step + 1 into slot cur ^ 1
        if (ahead) slot ^= 1;
        return hipGetLastError();
    }
    // any other launch moves the counter past the cached step: the cache is stale
    ahead = false;
    if (im_roll_applies(p, M1, t_u, pol, io)) {
        sunk = true;                  // so do the rollout kernels
        return im_roll_launch<PhiloxGen>(p, backlog, t_u, pol, io, s);
    }
#define K_(M, B, TU, ONE, POL)                                                                          \
    do {                                                                                                \
        if (npd)                                                                                        \
            hipLaunchKernelGGL((im_run_kernel<M, B, TU, ONE, POL, true, PhiloxGen>), grid, block, lds, s, p, t_u, io, pv);  \
        else                                                                                            \
            hipLaunchKernelGGL((im_run_kernel<M, B, TU, ONE, POL, false, PhiloxGen>), grid, block, lds, s, p, t_u, io, pv); \
    } while (0)
#define L_(M, B)                                             \
    do {                                                     \
        if (pol) {                                           \
            if (t_u >= 0) K_(M, B, true, false, true);       \
            else K_(M, B, false, false, true);               \
        } else if (io.K == 1) {                              \
            if (t_u >= 0) K_(M, B, true, true, false);       \
            else K_(M, B, false, true, false);               \
        } else {                                             \
            if (t_u >= 0) K_(M, B, true, false, false);      \
            else K_(M, B, false, false, false);              \
        }                                                    \
    } while (0)
    IM_DISPATCH(M1, backlog, L_)
#undef L_
#undef K_
    return hipGetLastError();
}

INVSIM_PTRS_STATS_TU(im_ph)
#else
hipError_t im_run_launch(const ImParams &p, int M1, bool backlog, int t_u, const PolicyIO *pol,
                         const StepIO<int64_t, int64_t> &io, bool &ahead, int &slot, bool &sunk, hipStream_t s) {
    sunk = im_sink_noop(p, t_u, pol, io);
    if (p.cm.N == 0 || io.K <= 0) return hipSuccess;
    const size_t lds = (size_t)EPW * M1 * (p.lt_max + 1) * sizeof(int64_t) + RHS_LDS_MAX * sizeof(double);
    const dim3 grid(grid_for(p.cm.N, EPW)), block(WAVE);
    PolicyIO none{};
    const PolicyIO &pv = pol ? *pol : none;
    const bool npd = p.dist >= 2 && p.dist <= 4;
    const bool ph = p.cm.philox != 0;       // fast stream: invmgmt_ph.hip (split / rollout / run kernels, no lookahead)
    if (ph) return im_run_launch_ph(p, M1, backlog, t_u, pol, io, ahead, slot, sunk, s);   // (a cache is the fast stream's)
    if (im_split_applies(p, t_u, pol, io)) {
        const size_t lds2 = lds + WAVE * sizeof(int64_t);
        const dim3 block2(2 * WAVE);
        ImParams q = p;
        if (!p.cm.kn.im_ahead) q.ahead = nullptr;
        if (ahead && !q.ahead) {      // lookahead switched off: commit, then draw inline
            const hipError_t ce = im_commit_launch(p, slot, s);
            ahead = false;
            if (ce != hipSuccess) return ce;
        }
        const bool hit = ahead && q.ahead;
        const int gla = hit ? (int)grid_for(p.cm.N, 2 * WAVE) : 0;   // lookahead workgroups
        const dim3 grid2(grid.x + gla);
        const int cur = slot;
        const int la0 = p.cm.kn.im_la_last ? (int)grid.x : 0;   // lookahead workgroups first (default) or last
#define S_(M, B)                                                                                        \
    do {                                                                                                \
        if (npd) {                                                                                      \
            if (hit) hipLaunchKernelGGL((im_split_kernel<M, B, true, true>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla);  \
            else hipLaunchKernelGGL((im_split_kernel<M, B, true, false>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla);     \
        } else {                                                                                        \
            if (hit) hipLaunchKernelGGL((im_split_kernel<M, B, false, true>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla); \
            else hipLaunchKernelGGL((im_split_kernel<M, B, false, false>), grid2, block2, lds2, s, q, t_u, io, cur, la0, gla);    \
        }                                                                                               \
    } while (0)
        IM_DISPATCH(M1, backlog, S_)
#undef S_
        sunk = true;                  // the split kernel folds into the episode sink (if one is set)
        if (q.ahead) {                // every env drew its next demand into slot cur ^ 1
            ahead = true;
            slot ^= 1;
        } else {
            ahead = false;
        }
        return hipGetLastError();
    }
    // the one-wave kernel draws from the committed state (brought into cm.rng
    // first): the cache is stale after it, unless this launch is the lock-step
    // autoreset (no draw)
    if (!(!pol && io.K == 1 && t_u >= p.periods) && ahead) {
        const hipError_t ce = im_commit_launch(p, slot, s);
        ahead = false;
        if (ce != hipSuccess) return ce;
    }
    // lock-step rollout of the reference's default lead times: register windows
    // and a demand wave (im_roll3_kernel / im_roll3o_kernel), open loop or with
    // the in-kernel BaseStock / ConstantOrder agents
    if (im_roll_applies(p, M1, t_u, pol, io)) {
        sunk = true;                  // so do the rollout kernels
        return im_roll_launch<Pcg>(p, backlog, t_u, pol, io, s);
    }
#define K_(M, B, TU, ONE, POL)                                                                         \
    do {                                                                                                \
        if (npd)                                                                                        \
            hipLaunchKernelGGL((im_run_kernel<M, B, TU, ONE, POL, true, Pcg>), grid, block, lds, s, p, t_u, io, pv);  \
        else                                                                                            \
            hipLaunchKernelGGL((im_run_kernel<M, B, TU, ONE, POL, false, Pcg>), grid, block, lds, s, p, t_u, io, pv); \
    } while (0)
#define L_(M, B)                                             \
    do {                                                     \
        if (pol) {                                           \
            if (t_u >= 0) K_(M, B, true, false, true);       \
            else K_(M, B, false, false, true);               \
        } else if (io.K == 1) {                              \
            if (t_u >= 0) K_(M, B, true, true, false);       \
            else K_(M, B, false, true, false);               \
        } else {                                             \
            if (t_u >= 0) K_(M, B, true, false, false);      \
            else K_(M, B, false, false, false);              \
        }                                                    \
    } while (0)
    IM_DISPATCH(M1, backlog, L_)
#undef L_
#undef K_
    return hipGetLastError();
}

hipError_t im_commit_launch(const ImParams &p, int slot, hipStream_t s) {
    if (p.cm.N == 0 || !p.ahead) return hipSuccess;
    hipLaunchKernelGGL(im_commit_kernel, dim3(grid_for(p.cm.N, 256)), dim3(256), 0, s, p, slot ^ 1);
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

INVSIM_PTRS_STATS_TU(im)
#endif  // INVSIM_IM_FAST_TU

}  // namespace invsim

#if defined(INVSIM_TIMING) && !defined(INVSIM_IM_FAST_TU)
extern "C" int invsim_debug_timing(void *dst, int64_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(invsim::g_tbuf), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int invsim_debug_timing_bar(void *dst, int64_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(invsim::g_tbar), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
#endif
