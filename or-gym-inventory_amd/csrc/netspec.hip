// NetInvMgmtMasterEnv.step / reset (network_management.py:301-635) specialised
// at compile time for the reference's own supply networks (net_topologies.hpp:
// the default graph of network_management.py:108-139 and the custom graph of
// network_management_custom.py:108-145).  capi.hip selects this kernel when a
// handle's compiled tables equal one of them, else the generic table-walking
// kernel of netinvmgmt.hip runs.  Both produce identical results.
//
// With the topology constexpr, every node/link loop unrolls and every per-env
// node/link value is a register: no table reads, no LDS scratch.  The order
// windows live in registers aligned by AGE: w[k][a-1] = R[t-a, link k] for
// a = 1..L_k (a = L_k is this period's arrival).  A step reads the ring once
// (all sum L entries, masked by the period like the reference's zeroed
// history), writes one slot per link; a K-step rollout shifts the registers
// and stores the whole ring once at the end.
//
// Arithmetic order is the generic kernel's (and the reference's), term by term.
#include "../../include/invsim.h"
#include "kernels.hpp"
#include "net_topologies.hpp"

namespace invsim {
namespace {

__device__ __forceinline__ double max0(double x) { return (x > 0) ? x : 0.0; }

template <class G, class RG = Pcg>
struct NetSt {
    RG g;
    double X[G::J];
    double U[G::RL];
    double Y[G::E];
    double w[G::sumL > 0 ? G::sumL : 1];   // age-aligned order windows (see above)
};

// slot of R[t - a] in link k's ring (t - a >= 0)
template <class G>
__device__ __forceinline__ int ring_row(int k, int t, int a) {
    return G::ring_off[k] + (int)((uint32_t)(t - a) % (uint32_t)G::L[k]);
}

template <class G, class RG = Pcg>
__device__ __forceinline__ void spec_reset(NetSt<G, RG> &s, float *orow) {
#pragma unroll
    for (int j = 0; j < G::J; j++) s.X[j] = G::I0[j];
#pragma unroll
    for (int r = 0; r < G::RL; r++) s.U[r] = 0.0;
#pragma unroll
    for (int k = 0; k < G::E; k++) s.Y[k] = 0.0;
#pragma unroll
    for (int q = 0; q < G::sumL; q++) s.w[q] = 0.0;
#pragma unroll
    for (int r = 0; r < G::RL; r++) orow[r] = 0.f;
#pragma unroll
    for (int j = 0; j < G::J; j++) orow[G::RL + j] = (float)G::I0[j];
#pragma unroll
    for (int q = 0; q < G::sumL; q++) orow[G::RL + G::J + q] = 0.f;
}

// market demand draws of one step, retail-link order: max(0, int(round(poisson(lam))))
// (:536-541)
template <class G, class RG>
__device__ __forceinline__ void spec_demand(RG &g, const PtrsConst (&pc)[G::RL], const double *rhs_l,
                                            double (&Dd)[G::RL]) {
#pragma unroll
    for (int r = 0; r < G::RL; r++) {
        g.sub((uint32_t)r);                                    // fast stream: market r's counter block
        const int64_t pd = np_poisson(g, pc[r], rhs_l + r * RHS_LDS_MAX);
        Dd[r] = (double)(pd > 0 ? pd : 0);
    }
}

// The demand wave of the rollout kernels (stream_flat_loop): the market demands
// of each launch step, retail-link order, into the ring dbuf [RD * CH][RL][WAVE]
template <class G, int CH, int RD, class RG>
__device__ __forceinline__ void net_demand_loop(RG &g, const PtrsConst (&pc)[G::RL], const double *rhs_l,
                                                double *dbuf, int lane, int K, int nb, int t_start, int T,
                                                uint64_t ph_step) {
    constexpr int RL = G::RL;
    StreamPos<RG> pos(ph_step);
    stream_flat_loop<CH, RD, RL>(
        K, nb, t_start, T,
        [&](int j, int r, int64_t &kd) {
            pos.at(g, j, r);
            PtrsConst c = pc[0];
            const double *rt = rhs_l;
#pragma unroll
            for (int q = 1; q < RL; q++)
                if (r == q) {
                    c = pc[q];
                    rt = rhs_l + q * RHS_LDS_MAX;
                }
#ifdef INVSIM_ABL_ROLL_NO_DRAW
            kd = 20;
            return true;
#else
            return np_poisson_try(g, c, rt, kd);
#endif
        },
        [&](int slot, int r, int64_t kd) {   // max(0, int(round(poisson(lam)))) (:536-541)
            dbuf[(slot * RL + r) * WAVE + lane] = (double)(kd > 0 ? kd : 0);
        });
}

// One step (:436-635) at period t < T given the step's market demands Dd; obs
// row into orow (LDS).  Returns the reward; Rn receives R[t] (the fulfilled
// orders) per link.
//
// spec_flow: phases 0-3 of the step (orders, pipeline, arrivals, market), the
// state update without the profit; Sr receives the market sales.
template <class G, class RG = Pcg>
__device__ __forceinline__ void spec_flow(const NetParams &P, NetSt<G, RG> &s, const float (&act)[G::E],
                                          const double (&Dd)[G::RL], const double (&wa)[G::E], double (&Rn)[G::E],
                                          double (&Sr)[G::RL]) {
    double cons[G::J];
#pragma unroll
    for (int j = 0; j < G::J; j++) cons[j] = 0.0;
    // 0) orders over sorted reorder links (:448-490)
#pragma unroll
    for (int k = 0; k < G::E; k++) {
        const double rq = rint((double)act[k]);               // round() half-to-even
        const double request = (rq > 0) ? rq : 0.0;            // max(0, .)
        double f;
        if (G::sup[k] < 0) {
            f = request;                                       // raw material: unlimited
        } else {
            const int sp = G::sup[k] < 0 ? 0 : G::sup[k];
            const double oav = max0(s.X[sp] - cons[sp]);
            double avail = oav;
            if (G::sup_is_factory[k]) {
                const double mpi = G::v[sp] * oav;
                const double mp = (mpi < G::C[sp]) ? mpi : G::C[sp];   // min(C, v*avail)
                avail = (mp < avail) ? mp : avail;
            }
            f = (avail < request) ? avail : request;           // min(request, avail)
            cons[sp] += f / G::v[sp];
        }
        Rn[k] = f;
    }
    // 1) pipeline (:494-511): arrival = R[t-L] (age L), or R[t] when L == 0
    double arrv[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) {
        arrv[k] = (G::L[k] == 0) ? Rn[k] : wa[k];
        s.Y[k] = s.Y[k] - arrv[k] + Rn[k];
    }
    // arrivals in predecessor adjacency order (:516-523); X[t+1] (:528)
#pragma unroll
    for (int j = 0; j < G::J; j++) {
        double acc = 0.0;
#pragma unroll
        for (int q = G::pred_ptr[j]; q < G::pred_ptr[j + 1]; q++) acc += arrv[G::pred_idx[q]];
        s.X[j] = (s.X[j] + acc) - cons[j];
    }
    // 2&3) market fulfilment in retail-link edge order (:536-566)
#pragma unroll
    for (int r = 0; r < G::RL; r++) {
        const double fill = Dd[r] + s.U[r];
        const int node = G::rl_node[r];
        const double inv = max0(s.X[node]);
        const double sale = (inv < fill) ? inv : fill;          // min(fill, inv)
        s.X[node] -= sale;
        Sr[r] = sale;
        s.U[r] = P.backlog ? fill - sale : 0.0;
    }
}

// spec_profit: phase 5, the period's total profit over the main nodes
// (:578-613, Python sum() order = adjacency order) from R[t], the market sales,
// X[t+1], Y[t+1] and U[t+1]; pj (nullable) receives each node's profit.
template <class G>
__device__ __forceinline__ double spec_profit(const double (&Rn)[G::E], const double (&Sr)[G::RL],
                                              const double (&X)[G::J], const double (&Y)[G::E],
                                              const double (&U)[G::RL], double *pjo) {
    double total = 0.0;
#pragma unroll
    for (int j = 0; j < G::J; j++) {
        double SR = 0.0, sold = 0.0;
#pragma unroll
        for (int q = G::succ_ptr[j]; q < G::succ_ptr[j + 1]; q++) {
            const int idx = G::succ_idx[q];
            const bool re = G::succ_kind[q] == 0;
            const double sv = re ? Rn[idx < G::E ? idx : 0] : Sr[idx < G::RL ? idx : 0];
            SR += (re ? G::lp[idx < G::E ? idx : 0] : G::rl_p[idx < G::RL ? idx : 0]) * sv;
            sold += sv;
        }
        double PC = 0.0, HCp = 0.0;
#pragma unroll
        for (int q = G::pred_ptr[j]; q < G::pred_ptr[j + 1]; q++) PC += G::lp[G::pred_idx[q]] * Rn[G::pred_idx[q]];
        const double HC_on = G::h[j] * max0(X[j]);
#pragma unroll
        for (int q = G::pred_ptr[j]; q < G::pred_ptr[j + 1]; q++) HCp += G::lg[G::pred_idx[q]] * max0(Y[G::pred_idx[q]]);
        const double HC = HC_on + HCp;
        double OC = 0.0;
        if (G::is_factory[j]) OC = (G::v[j] > 0) ? G::o[j] * (sold / G::v[j]) : 0.0;
        double UP = 0.0;
        if (G::is_retail[j]) {
#pragma unroll
            for (int q = G::succ_ptr[j]; q < G::succ_ptr[j + 1]; q++)
                if (G::succ_kind[q] == 1) UP += G::rl_b[G::succ_idx[q] < G::RL ? G::succ_idx[q] : 0] *
                                                U[G::succ_idx[q] < G::RL ? G::succ_idx[q] : 0];
        }
        const double pj = SR - PC - OC - HC - UP;
        if (pjo) pjo[j] = pj;
        total += pj;
    }
    return total;
}

// spec_core: the step without the observation, given each link's age-L window
// entry wa[k] = R[t - L_k] (the arrival; unused for L == 0).
template <class G, class RG = Pcg>
__device__ __forceinline__ double spec_core(const NetParams &P, double apow, NetSt<G, RG> &s,
                                            const float (&act)[G::E], const double (&Dd)[G::RL],
                                            const double (&wa)[G::E], double (&Rn)[G::E], double *met,
                                            double *irec) {
    double Sr[G::RL];
    spec_flow<G>(P, s, act, Dd, wa, Rn, Sr);
    if (irec) {  // step record: S[t, retail], U[t+1, retail], X[t+1, main] (network_management.py:536-571)
#pragma unroll
        for (int r = 0; r < G::RL; r++) {
            irec[r] = Sr[r];
            irec[G::RL + r] = s.U[r];
        }
#pragma unroll
        for (int j = 0; j < G::J; j++) irec[2 * G::RL + j] = s.X[j];
#pragma unroll
        for (int k = 0; k < G::E; k++) {
            irec[2 * G::RL + G::J + k] = Rn[k];              // R[t]
            irec[2 * G::RL + G::J + G::E + k] = s.Y[k];      // Y[t+1]
        }
    }
    if (met) {   // evaluate_agent metrics (benchmark_NetInvMgmtLostSalesEnv.py:264-300)
#pragma unroll
        for (int r = 0; r < G::RL; r++) {
            met[2] += Dd[r];                  // D[t, retail links]
            met[3] += Sr[r];                  // S[t, retail links]
            met[4] += s.U[r];                 // U[t+1, retail links]
        }
#pragma unroll
        for (int j = 0; j < G::J; j++) met[5 + j] += s.X[j];   // X[t+1, main nodes] per node
    }
    const double total = spec_profit<G>(Rn, Sr, s.X, s.Y, s.U, irec ? irec + 2 * G::RL + G::J + 2 * G::E : nullptr);
    return apow * total;                                       // :619
}

template <class G, bool WIN = true, class RG = Pcg>
__device__ __forceinline__ double spec_dyn(const NetParams &P, int t, double apow, NetSt<G, RG> &s,
                                           const float (&act)[G::E], const double (&Dd)[G::RL], float *orow,
                                           double (&Rn)[G::E], double *met, double *irec) {
    double wa[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) wa[k] = (G::L[k] > 0) ? s.w[G::L[k] > 0 ? G::ring_off[k] + G::L[k] - 1 : 0] : 0.0;
    const double rw = spec_core<G>(P, apow, s, act, Dd, wa, Rn, met, irec);
    // obs (:334-413): U[t+1], X[t+1], then per link with L > 0 the fulfilled
    // orders R[t+1-L .. t] oldest first (ages L-1 .. 1, then R[t])
#pragma unroll
    for (int r = 0; r < G::RL; r++) orow[r] = (float)s.U[r];
#pragma unroll
    for (int j = 0; j < G::J; j++) orow[G::RL + j] = (float)s.X[j];
#pragma unroll
    for (int k = 0; k < G::E; k++) {
        if (G::L[k] == 0) continue;
        if (WIN) {   // !WIN: another wave writes the older window entries
#pragma unroll
            for (int p = 0; p + 1 < G::L[k]; p++)
                orow[G::win_off[k] + p] = (float)s.w[G::ring_off[k] + (G::L[k] - 1 - p) - 1];
        }
        orow[G::win_off[k] + G::L[k] - 1] = (float)Rn[k];
    }
    (void)t;
    return rw;
}

// One step (:436-635) at period t < T: the demand draws, then the dynamics
template <class G, class RG = Pcg>
__device__ __forceinline__ double spec_step(const NetParams &P, const PtrsConst (&pc)[G::RL], const double *rhs_l,
                                            int t, double apow, NetSt<G, RG> &s, const float (&act)[G::E],
                                            float *orow, double (&Rn)[G::E], int64_t (&dem)[G::RL],
                                            double *met, double *irec) {
    double Dd[G::RL];
    spec_demand<G>(s.g, pc, rhs_l, Dd);
#pragma unroll
    for (int r = 0; r < G::RL; r++) dem[r] = (int64_t)Dd[r];
    return spec_dyn<G>(P, t, apow, s, act, Dd, orow, Rn, met, irec);
}

// shift the age-aligned windows by one period: age a+1 <- age a, age 1 <- R[t]
template <class G, class RG = Pcg>
__device__ __forceinline__ void spec_shift(NetSt<G, RG> &s, const double (&Rn)[G::E]) {
#pragma unroll
    for (int k = 0; k < G::E; k++) {
        if (G::L[k] == 0) continue;
#pragma unroll
        for (int a = G::L[k]; a >= 2; a--) s.w[G::ring_off[k] + a - 1] = s.w[G::ring_off[k] + a - 2];
        s.w[G::ring_off[k]] = Rn[k];
    }
}

template <class G, bool TU, bool ONE, bool POL, class RG>
__global__ void __launch_bounds__(WAVE)
net_spec_kernel(NetParams P, int t_u, StepIO<float, float> io, PolicyIO pol) {
    extern __shared__ __attribute__((aligned(16))) float ns_lds[];
    constexpr int O = G::O;
    constexpr int TILE_IT = (EPW * O * 4 + 16 * WAVE - 1) / (16 * WAVE);
    const int lane = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * EPW;
    const int64_t e = e0 + lane;
    const int64_t N = P.cm.N;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < EPW ? (N - e0) : EPW);
    const int64_t S = P.cm.Npad;
    const int64_t el = valid ? e : N - 1;      // lanes past N mirror env N-1 (loads only)
    float *tile = ns_lds;
    float *trow = tile + lane * O;
    double *rhs_l = reinterpret_cast<double *>(ns_lds + ((EPW * O + 3) / 4) * 4);

    int t = TU ? t_u : P.cm.period[el];
    NetSt<G, RG> st;
    if (ONE && TU && t >= P.T) {
        // lock-step NEXT_STEP autoreset of the whole batch (the host refuses a
        // DISABLED overrun when lock-step; SAME_STEP resets in the done step)
        spec_reset<G>(st, trow);
        if (valid) {
#pragma unroll
            for (int j = 0; j < G::J; j++) P.X[j * S + e] = G::I0[j];
#pragma unroll
            for (int r = 0; r < G::RL; r++) P.U[r * S + e] = 0.0;
#pragma unroll
            for (int k = 0; k < G::E; k++) P.Y[k * S + e] = 0.0;
            out_store(io.rew + e, 0.0);
            out_store(io.term + e, (uint8_t)0);
            out_store(io.trunc + e, (uint8_t)0);
        }
        wave_lds_sync();
        store_tile<TILE_IT>(tile, io.obs + e0 * O, (int64_t)nvalid * O, lane);
        return;
    }
    // every load up front, in the order the values are needed
    const int tc = (t < P.T) ? t : 0;
    double apow = P.alpha_pow[tc];
    PtrsConst pc[G::RL];
#pragma unroll
    for (int r = 0; r < G::RL; r++) pc[r] = P.rl_pc[r];
    constexpr int NT = RHS_LDS_MAX / WAVE;
    double tv[G::RL][NT];
#pragma unroll
    for (int r = 0; r < G::RL; r++) {
        const int qm = pc[r].nk > 0 ? pc[r].nk - 1 : 0;
        const double *src = pc[r].nk > 0 ? P.rhs + pc[r].toff : P.alpha_pow;   // any valid pointer
#pragma unroll
        for (int u = 0; u < NT; u++) tv[r][u] = src[min(lane + u * WAVE, qm)];
    }
    P.cm.rng.load(el, st.g);
#pragma unroll
    for (int j = 0; j < G::J; j++) st.X[j] = P.X[j * S + el];
#pragma unroll
    for (int r = 0; r < G::RL; r++) st.U[r] = P.U[r * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) st.Y[k] = P.Y[k * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) {
        if (G::L[k] == 0) continue;
#pragma unroll
        for (int a = 1; a <= G::L[k]; a++) {
            const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
            const double v = P.Rring[(int64_t)row * S + el];
            st.w[G::ring_off[k] + a - 1] = (t - a >= 0) ? v : 0.0;   // zeroed history (:315-321)
        }
    }
    float act[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) act[k] = POL ? pol.cf[k] : io.act[el * G::E + k];
    constexpr int MD = 5 + G::J;             // metrics: reward, steps, demand, sales, stockout, X per node
    double met[MD];
#pragma unroll
    for (int q = 0; q < MD; q++) met[q] = (POL && pol.metrics) ? pol.metrics[el * MD + q] : 0.0;
#pragma unroll
    for (int r = 0; r < G::RL; r++)
#pragma unroll
        for (int u = 0; u < NT; u++) rhs_l[r * RHS_LDS_MAX + lane + u * WAVE] = tv[r][u];
    wave_lds_sync();

    bool fault = false;
    bool dirty_all = false;                    // rollout: whole ring rewritten at the end
    const int t_start = t;
    double Rn[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) Rn[k] = 0.0;
    const int K = ONE ? 1 : io.K;
    for (int kk = 0; kk < K; kk++) {
        const int64_t oi = (int64_t)kk * N + e;
        st.g.set_step(P.cm.ph_step + (uint64_t)kk);
        if (kk > 0) {
            const int64_t ea = (int64_t)kk * N + el;
            if (!POL) {
#pragma unroll
                for (int k = 0; k < G::E; k++) act[k] = io.act[ea * G::E + k];
            }
            apow = P.alpha_pow[(t < P.T) ? t : 0];
        }
        bool tr = false;
        if (!(ONE && TU) && t >= P.T) {
            if (P.cm.autoreset == AR_NEXT_STEP) {
                spec_reset<G>(st, trow);
                dirty_all = true;
                if (valid && (!POL || io.rew)) {
                    out_store(io.rew + oi, 0.0);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)0);
                }
                t = 0;
            } else {
                fault = true;   // stepping past the horizon (DISABLED)
            }
        } else {
            int64_t dem[G::RL];
            double *irec = (valid && kk == K - 1 && P.cm.info_rec)
                               ? (double *)P.cm.info_rec + e * (2 * G::RL + 2 * G::J + 2 * G::E) : nullptr;
            const double r = spec_step<G>(P, pc, rhs_l, t, apow, st, act, trow, Rn, dem, POL ? met : nullptr, irec);
            tr = t + 1 >= P.T;
            if (POL) {
                met[0] += r;                    // episode_reward += reward
                met[1] += 1.0;
                if (valid && pol.act_out) {
#pragma unroll
                    for (int k = 0; k < G::E; k++) out_store((float *)pol.act_out + oi * G::E + k, act[k]);
                }
            }
            if (valid && (!POL || io.rew)) {
                out_store(io.rew + oi, r);
                out_store(io.term + oi, (uint8_t)0);
                out_store(io.trunc + oi, (uint8_t)(tr ? 1 : 0));
            }
            if (valid) {
                if (kk == K - 1 && P.cm.info_demand) {
#pragma unroll
                    for (int q = 0; q < G::RL; q++) P.cm.info_demand[e * G::RL + q] = dem[q];
                }
            }
            if (ONE) {
                // single step: the ring changes in one slot per link, R[t]
                if (valid) {
#pragma unroll
                    for (int k = 0; k < G::E; k++)
                        if (G::L[k] > 0)
                            st_store(P.Rring + (int64_t)(G::ring_off[k] + (int)((uint32_t)t % (uint32_t)G::L[k])) * S + e,
                                     Rn[k]);
                }
            } else {
                spec_shift<G>(st, Rn);
                dirty_all = true;
            }
            t += 1;
        }
        if (P.cm.autoreset == AR_SAME_STEP && tr) {          // final obs out, then the reset obs in
            wave_lds_sync();
            if (valid && io.fobs)
                for (int q = 0; q < O; q++) io.fobs[e * O + q] = trow[q];
            wave_lds_sync();
            spec_reset<G>(st, trow);
            dirty_all = true;
            t = 0;
        }
        wave_lds_sync();
        if (!POL || io.obs) store_tile<TILE_IT>(tile, io.obs + ((int64_t)kk * N + e0) * O, (int64_t)nvalid * O, lane);
        wave_lds_sync();
    }
    if (valid) {
        P.cm.rng.store_state(e, st.g);
#pragma unroll
        for (int j = 0; j < G::J; j++) st_store(P.X + j * S + e, st.X[j]);
#pragma unroll
        for (int r = 0; r < G::RL; r++) st_store(P.U + r * S + e, st.U[r]);
#pragma unroll
        for (int k = 0; k < G::E; k++) st_store(P.Y + k * S + e, st.Y[k]);
        if (!ONE && dirty_all) {
            // ring slot of R[t - a] = age-a window register (zeros before the episode)
#pragma unroll
            for (int k = 0; k < G::E; k++) {
                if (G::L[k] == 0) continue;
#pragma unroll
                for (int a = 1; a <= G::L[k]; a++)
                    st_store(P.Rring + (int64_t)(G::ring_off[k] +
                                                 (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k])) * S + e,
                             st.w[G::ring_off[k] + a - 1]);
            }
        }
        if (!TU) P.cm.period[e] = t;
        if (fault) atomicOr(P.cm.status, 1u);
        if (POL && pol.metrics) {
#pragma unroll
            for (int q = 0; q < MD; q++) pol.metrics[e * MD + q] = met[q];
        }
    }
    (void)t_start;
}

// Cross-wave LDS handoff inside a workgroup: orders LDS traffic only (an
// __syncthreads() would also drain each wave's outstanding global loads and
// stores, s_waitcnt vmcnt(0), before the s_barrier)
__device__ __forceinline__ void net_wg_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Single lock-step step (invsim_step: K = 1, t < T, no policy, no SAME_STEP
// reset in this step) with the demand lookahead.  The market demands of a step
// are Poisson draws of the env's own stream at fixed rates, and reset() draws
// nothing (:301-332), so every launch can already draw the NEXT step's demands.
// P.ahead: two slots of rows [state hi, state lo, demand per retail link] x
// Npad, alternating per launch.
//   HIT (slot cur holds each env's state RL draws past the committed one, and
//        those draws): the step workgroups load the demands; `gla` workgroups
//        at the front of the grid draw the next demands from slot cur's state
//        into slot cur ^ 1, so the Poisson chain runs beside the step.
//   !HIT: the step draws inline from cm.rng, leaves the state in slot cur, then
//        draws the lookahead into slot cur ^ 1.
// After the launch the committed state is slot cur; the host flips the slots,
// and cm.rng is brought up to date from it (net_commit_kernel) only before
// something reads it.  Streams are consumed in the reference's order;
// arithmetic as net_spec_kernel.
template <class G, bool HIT>
__global__ void __launch_bounds__(WAVE)
net_step1_kernel(NetParams P, int t, StepIO<float, float> io, int cur, int gla) {
    extern __shared__ __attribute__((aligned(16))) float ns_lds[];
    constexpr int O = G::O, RL = G::RL, NR = 2 + G::RL;
    constexpr int TILE_IT = (EPW * O * 4 + 16 * WAVE - 1) / (16 * WAVE);
    constexpr int NT = RHS_LDS_MAX / WAVE;
    const int lane = threadIdx.x;
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const uint64_t *Acur = P.ahead + (int64_t)cur * NR * S;
    uint64_t *Anxt = P.ahead + (int64_t)(cur ^ 1) * NR * S;
    double *rhs_l = reinterpret_cast<double *>(ns_lds + ((EPW * O + 3) / 4) * 4);
    PtrsConst pc[RL];
#pragma unroll
    for (int r = 0; r < RL; r++) pc[r] = P.rl_pc[r];
    auto stage = [&](double (&tv)[RL][NT]) {
#pragma unroll
        for (int r = 0; r < RL; r++) {
            const int qm = pc[r].nk > 0 ? pc[r].nk - 1 : 0;
            const double *src = pc[r].nk > 0 ? P.rhs + pc[r].toff : P.alpha_pow;   // any valid pointer
#pragma unroll
            for (int u = 0; u < NT; u++) tv[r][u] = src[min(lane + u * WAVE, qm)];
        }
    };
    auto flush = [&](const double (&tv)[RL][NT]) {
#pragma unroll
        for (int r = 0; r < RL; r++)
#pragma unroll
            for (int u = 0; u < NT; u++) rhs_l[r * RHS_LDS_MAX + lane + u * WAVE] = tv[r][u];
        wave_lds_sync();
    };
    const int bid = (int)blockIdx.x;
    if (HIT && bid < gla) {   // ---- lookahead workgroup: 64 envs, one per lane
        const int64_t e = (int64_t)bid * WAVE + lane;
        const bool valid = e < N;
        const int64_t el = valid ? e : N - 1;
        double tv[RL][NT];
        stage(tv);
        Pcg g;
        g.hi = Acur[el];
        g.lo = Acur[S + el];
        g.inc_hi = P.cm.rng.inc_hi[el];
        g.inc_lo = P.cm.rng.inc_lo[el];
        PtrsJumpLane jt;
        jt.load(lane);
        flush(tv);
        double Dd[RL];
#pragma unroll
        for (int r = 0; r < RL; r++) {   // spec_demand, PTRS with a compacted second round
            const double *rt = rhs_l + r * RHS_LDS_MAX;
            const int64_t pd =
                pc[r].lam >= 10
                    ? np_poisson_ptrs_compact(
                          g, pc[r], RhsTab{rt}, true, jt,
                          [](const PtrsConst &c, int) { return c; })
                    : np_poisson(g, pc[r], rt);
            Dd[r] = (double)(pd > 0 ? pd : 0);
        }
        if (valid) {
            st_store(Anxt + e, g.hi);
            st_store(Anxt + S + e, g.lo);
#pragma unroll
            for (int r = 0; r < RL; r++) st_store(Anxt + (2 + r) * S + e, (uint64_t)(int64_t)Dd[r]);
        }
        return;
    }
    const int64_t e0 = (int64_t)(bid - (HIT ? gla : 0)) * EPW;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < EPW ? (N - e0) : EPW);
    const int64_t el = valid ? e : N - 1;      // lanes past N mirror env N-1 (loads only)
    float *tile = ns_lds;
    float *trow = tile + lane * O;
    NetSt<G> st;
    double Dd[RL];
    double tv[RL][NT];
    if (HIT) {
#pragma unroll
        for (int r = 0; r < RL; r++) Dd[r] = (double)(int64_t)Acur[(2 + r) * S + el];
    } else {
        stage(tv);
        st.g = P.cm.rng.load(el);
    }
    const double apow = P.alpha_pow[t];
#pragma unroll
    for (int j = 0; j < G::J; j++) st.X[j] = P.X[j * S + el];
#pragma unroll
    for (int r = 0; r < RL; r++) st.U[r] = P.U[r * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) st.Y[k] = P.Y[k * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) {
        if (G::L[k] == 0) continue;
#pragma unroll
        for (int a = 1; a <= G::L[k]; a++) {
            const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
            const double v = P.Rring[(int64_t)row * S + el];
            st.w[G::ring_off[k] + a - 1] = (t - a >= 0) ? v : 0.0;   // zeroed history (:315-321)
        }
    }
    float act[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) act[k] = io.act[el * G::E + k];
    if (!HIT) {
        flush(tv);
        spec_demand<G>(st.g, pc, rhs_l, Dd);                   // :536-541
    }
    double Rn[G::E];
    double *irec = (valid && P.cm.info_rec) ? (double *)P.cm.info_rec + e * (2 * RL + 2 * G::J + 2 * G::E) : nullptr;
    const double r = spec_dyn<G>(P, t, apow, st, act, Dd, trow, Rn, nullptr, irec);
    if (valid) {
        out_store(io.rew + e, r);
        out_store(io.term + e, (uint8_t)0);
        out_store(io.trunc + e, (uint8_t)(t + 1 >= P.T ? 1 : 0));
        if (P.cm.info_demand) {
#pragma unroll
            for (int q = 0; q < RL; q++) P.cm.info_demand[e * RL + q] = (int64_t)Dd[q];
        }
    }
    wave_lds_sync();
    store_tile<TILE_IT>(tile, io.obs + e0 * O, (int64_t)nvalid * O, lane);
    if (valid) {
#pragma unroll
        for (int k = 0; k < G::E; k++)
            if (G::L[k] > 0)
                st_store(P.Rring + (int64_t)(G::ring_off[k] + (int)((uint32_t)t % (uint32_t)G::L[k])) * S + e, Rn[k]);
#pragma unroll
        for (int j = 0; j < G::J; j++) st_store(P.X + j * S + e, st.X[j]);
#pragma unroll
        for (int q = 0; q < RL; q++) st_store(P.U + q * S + e, st.U[q]);
#pragma unroll
        for (int k = 0; k < G::E; k++) st_store(P.Y + k * S + e, st.Y[k]);
    }
    if (!HIT) {   // committed state (after this step's draws) -> slot cur; the lookahead -> slot cur ^ 1
        if (valid) {
            st_store((uint64_t *)Acur + e, st.g.hi);
            st_store((uint64_t *)Acur + S + e, st.g.lo);
        }
        spec_demand<G>(st.g, pc, rhs_l, Dd);
        if (valid) {
            st_store(Anxt + e, st.g.hi);
            st_store(Anxt + S + e, st.g.lo);
#pragma unroll
            for (int q = 0; q < RL; q++) st_store(Anxt + (2 + q) * S + e, (uint64_t)(int64_t)Dd[q]);
        }
    }
}

// net_step1_kernel with the work of 64 envs split over two waves of one
// workgroup (the step's load -> compute -> store chain is the step time at the
// 32 768-env configuration):
//   wave 0 (window)   the observation's order windows: R[t-a] for ages
//                     1 .. L-1 of every link (52 of the default graph's 61
//                     ring entries), read, rounded to f32 and placed in the
//                     LDS tile
//   wave 1 (dynamics) X, U, Y, the arrivals (age L), actions and demands; the
//                     step with the tile's U, X and newest orders; the state,
//                     ring slot and output stores (and the inline draw /
//                     lookahead production when !HIT)
// Then both waves store half of the tile.  Lookahead workgroups (HIT) cover 128
// envs, one per thread.  Same arithmetic as net_spec_kernel.
// RG = PhiloxGen (the fast stream): a draw is a function of (key, launch step),
// so the cache holds only the next step's market demands (rows 2 ..), and no
// generator state is read or written.
template <class G, bool HIT, class RG = Pcg>
__global__ void __launch_bounds__(2 * WAVE)
net_step2_kernel(NetParams P, int t, StepIO<float, float> io, int cur, int gla) {
    extern __shared__ __attribute__((aligned(16))) float ns_lds[];
    constexpr int O = G::O, RL = G::RL, NR = 2 + G::RL;
    constexpr int NT = RHS_LDS_MAX / WAVE;
    constexpr int HALF_IT = (EPW * O * 4 / 2 + 16 * WAVE - 1) / (16 * WAVE) + 1;
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const uint64_t *Acur = P.ahead + (int64_t)cur * NR * S;
    uint64_t *Anxt = P.ahead + (int64_t)(cur ^ 1) * NR * S;
    double *rhs_l = reinterpret_cast<double *>(ns_lds + ((EPW * O + 3) / 4) * 4);
    PtrsConst pc[RL];
#pragma unroll
    for (int r = 0; r < RL; r++) pc[r] = P.rl_pc[r];
    auto stage = [&](double (&tv)[RL][NT]) {
#pragma unroll
        for (int r = 0; r < RL; r++) {
            const int qm = pc[r].nk > 0 ? pc[r].nk - 1 : 0;
            const double *src = pc[r].nk > 0 ? P.rhs + pc[r].toff : P.alpha_pow;   // any valid pointer
#pragma unroll
            for (int u = 0; u < NT; u++) tv[r][u] = src[min(lane + u * WAVE, qm)];
        }
    };
    auto flush = [&](const double (&tv)[RL][NT]) {   // each wave writes the whole (identical) table
#pragma unroll
        for (int r = 0; r < RL; r++)
#pragma unroll
            for (int u = 0; u < NT; u++) rhs_l[r * RHS_LDS_MAX + lane + u * WAVE] = tv[r][u];
        wave_lds_sync();
    };
    const int bid = (int)blockIdx.x;
    if (HIT && bid < gla) {   // ---- lookahead workgroup: 128 envs, one per thread
        const int64_t e = (int64_t)bid * (2 * WAVE) + threadIdx.x;
        const bool valid = e < N;
        const int64_t el = valid ? e : N - 1;
        double tv[RL][NT];
        stage(tv);
        if constexpr (RG::kCounter) {   // the fast stream: launch step ph_step + 1
            RG g;
            P.cm.rng.load(el, g);
            g.set_step(P.cm.ph_step + 1);
            flush(tv);
            double Dd[RL];
            spec_demand<G>(g, pc, rhs_l, Dd);
            if (valid) {
#pragma unroll
                for (int r = 0; r < RL; r++) st_store(Anxt + (2 + r) * S + e, (uint64_t)(int64_t)Dd[r]);
            }
            return;
        }
        Pcg g;
        g.hi = Acur[el];
        g.lo = Acur[S + el];
        g.inc_hi = P.cm.rng.inc_hi[el];
        g.inc_lo = P.cm.rng.inc_lo[el];
        PtrsJumpLane jt;
        jt.load(lane);
        flush(tv);
        double Dd[RL];
#pragma unroll
        for (int r = 0; r < RL; r++) {   // spec_demand, PTRS with a compacted second round
            const double *rt = rhs_l + r * RHS_LDS_MAX;
            const int64_t pd =
                pc[r].lam >= 10
                    ? np_poisson_ptrs_compact(
                          g, pc[r], RhsTab{rt}, true, jt,
                          [](const PtrsConst &c, int) { return c; })
                    : np_poisson(g, pc[r], rt);
            Dd[r] = (double)(pd > 0 ? pd : 0);
        }
        if (valid) {
            st_store(Anxt + e, g.hi);
            st_store(Anxt + S + e, g.lo);
#pragma unroll
            for (int r = 0; r < RL; r++) st_store(Anxt + (2 + r) * S + e, (uint64_t)(int64_t)Dd[r]);
        }
        return;
    }
    const int64_t e0 = (int64_t)(bid - (HIT ? gla : 0)) * EPW;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < EPW ? (N - e0) : EPW);
    const int64_t el = valid ? e : N - 1;      // lanes past N mirror env N-1 (loads only)
    float *tile = ns_lds;
    float *trow = tile + lane * O;
    const int64_t tcount = (int64_t)nvalid * O;
    const int64_t thalf = ((tcount / 2) + 3) & ~(int64_t)3;           // 16-B aligned split
    const int64_t h = thalf < tcount ? thalf : tcount;
    if (threadIdx.x < WAVE) {   // ---- window wave
        float wf[G::sumL > 0 ? G::sumL : 1];
#pragma unroll
        for (int k = 0; k < G::E; k++) {
            if (G::L[k] < 2) continue;
#pragma unroll
            for (int a = 1; a < G::L[k]; a++) {
                const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
                const double v = P.Rring[(int64_t)row * S + el];
                wf[G::ring_off[k] + a - 1] = (t - a >= 0) ? (float)v : 0.f;   // zeroed history (:315-321)
            }
        }
#pragma unroll
        for (int k = 0; k < G::E; k++) {
            if (G::L[k] < 2) continue;
#pragma unroll
            for (int p = 0; p + 1 < G::L[k]; p++) trow[G::win_off[k] + p] = wf[G::ring_off[k] + (G::L[k] - 1 - p) - 1];
        }
        net_wg_sync();   // tile complete
        store_tile<HALF_IT>(tile, io.obs + e0 * O, h, lane);
        return;
    }
    // ---- dynamics wave
    NetSt<G, RG> st;
    double Dd[RL];
    double tv[RL][NT];
    if (HIT) {
#pragma unroll
        for (int r = 0; r < RL; r++) Dd[r] = (double)(int64_t)Acur[(2 + r) * S + el];
    } else {
        stage(tv);
        P.cm.rng.load(el, st.g);
        st.g.set_step(P.cm.ph_step);
    }
    const double apow = P.alpha_pow[t];
#pragma unroll
    for (int j = 0; j < G::J; j++) st.X[j] = P.X[j * S + el];
#pragma unroll
    for (int r = 0; r < RL; r++) st.U[r] = P.U[r * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) st.Y[k] = P.Y[k * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) {   // only the arrivals: age L = R[t - L]
        if (G::L[k] == 0) continue;
        const int a = G::L[k];
        const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
        const double v = P.Rring[(int64_t)row * S + el];
        st.w[G::ring_off[k] + a - 1] = (t - a >= 0) ? v : 0.0;
    }
    float act[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) act[k] = io.act[el * G::E + k];
    if (!HIT) {
        flush(tv);
        spec_demand<G>(st.g, pc, rhs_l, Dd);                   // :536-541
    }
    double Rn[G::E];
    double *irec = (valid && P.cm.info_rec) ? (double *)P.cm.info_rec + e * (2 * RL + 2 * G::J + 2 * G::E) : nullptr;
    const double r = spec_dyn<G, false>(P, t, apow, st, act, Dd, trow, Rn, nullptr, irec);
    net_wg_sync();   // tile complete
    if (h < tcount) store_tile<HALF_IT>(tile + h, io.obs + e0 * O + h, tcount - h, lane);
    if (valid) {
        out_store(io.rew + e, r);
        out_store(io.term + e, (uint8_t)0);
        out_store(io.trunc + e, (uint8_t)(t + 1 >= P.T ? 1 : 0));
        if (P.cm.info_demand) {
#pragma unroll
            for (int q = 0; q < RL; q++) P.cm.info_demand[e * RL + q] = (int64_t)Dd[q];
        }
#pragma unroll
        for (int k = 0; k < G::E; k++)
            if (G::L[k] > 0)
                st_store(P.Rring + (int64_t)(G::ring_off[k] + (int)((uint32_t)t % (uint32_t)G::L[k])) * S + e, Rn[k]);
#pragma unroll
        for (int j = 0; j < G::J; j++) st_store(P.X + j * S + e, st.X[j]);
#pragma unroll
        for (int q = 0; q < RL; q++) st_store(P.U + q * S + e, st.U[q]);
#pragma unroll
        for (int k = 0; k < G::E; k++) st_store(P.Y + k * S + e, st.Y[k]);
    }
    if (!HIT) {   // committed state (after this step's draws) -> slot cur; the lookahead -> slot cur ^ 1
        if constexpr (!RG::kCounter) {
            if (valid) {
                st_store((uint64_t *)Acur + e, st.g.hi);
                st_store((uint64_t *)Acur + S + e, st.g.lo);
            }
        } else {
            st.g.set_step(P.cm.ph_step + 1);
        }
        spec_demand<G>(st.g, pc, rhs_l, Dd);
        if (valid) {
            if constexpr (!RG::kCounter) {
                st_store(Anxt + e, st.g.hi);
                st_store(Anxt + S + e, st.g.lo);
            }
#pragma unroll
            for (int q = 0; q < RL; q++) st_store(Anxt + (2 + q) * S + e, (uint64_t)(int64_t)Dd[q]);
        }
    }
}

// cm.rng <- the committed slot of the lookahead cache
__global__ void __launch_bounds__(256) net_commit_kernel(NetParams P, int slot, int nr) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int64_t S = P.cm.Npad;
    const uint64_t *A = P.ahead + (int64_t)slot * nr * S;
    P.cm.rng.hi[e] = A[e];
    P.cm.rng.lo[e] = A[S + e];
}


// K-step lock-step rollout (invsim_rollout without a policy, NEXT_STEP
// autoreset or no overrun, Poisson market demand) of a compiled network, one
// 128-thread workgroup per 64 envs:
//   wave 0 (demand)   draws the market demands (RL per step, retail-link order)
//                     into an LDS ring of RD chunks of CH launch steps, ahead
//                     of the dynamics wave (net_demand_loop).  A demand is a function
//                     of the env's stream only (the orders never touch it), and
//                     a NEXT_STEP reset step draws nothing (reset(), :301-332).
//   wave 1 (dynamics) spec_dyn with the windows in registers; a step's actions
//                     and alpha**t are loaded one step ahead, before the
//                     previous step's stores (vmcnt is in order: a load issued
//                     behind stores waits for them).
// Chunk handoff: chunk c is in the ring before barrier c; the dynamics wave
// consumes it between barriers c and c + 1, and the demand wave refills its
// slots only after barrier c + 1.  Same arithmetic, in the same order, as
// net_spec_kernel.
template <class G>
struct NetRoll {
    static constexpr int CH = 8;                                          // demand chunk (launch steps)
    static constexpr int RD = 4;                                          // demand ring depth (chunks)
    static constexpr size_t tile_bytes() { return (size_t)((EPW * G::O + 3) / 4) * 4 * sizeof(float); }
    static constexpr size_t lds() {
        return tile_bytes() + (size_t)G::RL * RHS_LDS_MAX * sizeof(double) + (size_t)RD * CH * G::RL * WAVE * sizeof(double);
    }
};

template <class G, class RG = Pcg>
__global__ void __launch_bounds__(2 * WAVE)
net_roll_kernel(NetParams P, int t_start, StepIO<float, float> io) {
    using R = NetRoll<G>;
    constexpr int O = G::O, CH = R::CH, RL = G::RL;
    constexpr int TILE_IT = (EPW * O * 4 + 16 * WAVE - 1) / (16 * WAVE);
    extern __shared__ __attribute__((aligned(16))) float nr_lds[];
    float *tile = nr_lds;
    double *rhs_l = reinterpret_cast<double *>(nr_lds + R::tile_bytes() / sizeof(float));
    double *dbuf = rhs_l + RL * RHS_LDS_MAX;                          // [RD * CH][RL][WAVE]
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const int64_t e0 = (int64_t)blockIdx.x * WAVE;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int64_t el = valid ? e : N - 1;       // padded lanes: the last env's data, never stored
    const int nvalid = (int)((N - e0) < WAVE ? (N - e0) : WAVE);
    const int K = io.K;
    const int nch = (K + CH - 1) / CH;
    if (threadIdx.x < WAVE) {   // ---- demand wave
        PtrsConst pc[RL];
#pragma unroll
        for (int r = 0; r < RL; r++) pc[r] = P.rl_pc[r];
        constexpr int NT = RHS_LDS_MAX / WAVE;
        double tv[RL][NT];
#pragma unroll
        for (int r = 0; r < RL; r++) {
            const int qm = pc[r].nk > 0 ? pc[r].nk - 1 : 0;
            const double *src = pc[r].nk > 0 ? P.rhs + pc[r].toff : P.alpha_pow;   // any valid pointer
#pragma unroll
            for (int u = 0; u < NT; u++) tv[r][u] = src[min(lane + u * WAVE, qm)];
        }
        RG g;
        P.cm.rng.load(el, g);
#pragma unroll
        for (int r = 0; r < RL; r++)
#pragma unroll
            for (int u = 0; u < NT; u++) rhs_l[r * RHS_LDS_MAX + lane + u * WAVE] = tv[r][u];
        wave_lds_sync();
        net_demand_loop<G, CH, R::RD>(g, pc, rhs_l, dbuf, lane, K, nch, t_start, P.T, P.cm.ph_step);   // barriers 0 .. nch - 1
        if (valid) P.cm.rng.store_state(e, g);
        return;
    }
    // ---- dynamics wave
    float *trow = tile + lane * O;
    int t = t_start;
    NetSt<G> st;
#pragma unroll
    for (int j = 0; j < G::J; j++) st.X[j] = P.X[j * S + el];
#pragma unroll
    for (int r = 0; r < RL; r++) st.U[r] = P.U[r * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) st.Y[k] = P.Y[k * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) {
        if (G::L[k] == 0) continue;
#pragma unroll
        for (int a = 1; a <= G::L[k]; a++) {
            const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
            const double v = P.Rring[(int64_t)row * S + el];
            st.w[G::ring_off[k] + a - 1] = (t - a >= 0) ? v : 0.0;   // zeroed history (:315-321)
        }
    }
    float nact[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) nact[k] = io.act[el * G::E + k];
    double napow = P.alpha_pow[t < P.T ? t : 0];
    double dlast[RL];
#pragma unroll
    for (int r = 0; r < RL; r++) dlast[r] = 0.0;
    bool last_real = false;
    double Rn[G::E];
    net_wg_sync();   // barrier 0: chunk 0 ready
    for (int c = 0; c < nch; c++) {
        const double *db = dbuf + (c % R::RD) * CH * RL * WAVE;
        for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
            const int k = c * CH + kk;
            const int64_t oi = (int64_t)k * N + e;
            float act[G::E];
#pragma unroll
            for (int q = 0; q < G::E; q++) act[q] = nact[q];
            const double apow = napow;
            {
                const int tn = (t >= P.T) ? 0 : t + 1;          // the next launch step's period
                napow = P.alpha_pow[tn < P.T ? tn : 0];
            }
            if (k + 1 < K) {                                    // the next step's actions
#pragma unroll
                for (int q = 0; q < G::E; q++) nact[q] = io.act[((int64_t)(k + 1) * N + el) * G::E + q];
            }
            if (t >= P.T) {                                     // NEXT_STEP autoreset (:301-332)
                spec_reset<G>(st, trow);
                if (valid) {
                    out_store(io.rew + oi, 0.0);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)0);
                }
                t = 0;
            } else {
                double Dd[RL];
#pragma unroll
                for (int r = 0; r < RL; r++) Dd[r] = db[(kk * RL + r) * WAVE + lane];
                const double rw = spec_dyn<G>(P, t, apow, st, act, Dd, trow, Rn, nullptr, nullptr);
                if (valid) {
                    out_store(io.rew + oi, rw);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)(t + 1 >= P.T ? 1 : 0));
                }
                spec_shift<G>(st, Rn);
#pragma unroll
                for (int r = 0; r < RL; r++) dlast[r] = Dd[r];
                last_real = k == K - 1;
                t += 1;
            }
            wave_lds_sync();
#ifndef INVSIM_ABL_ROLL_NO_STORE
            store_tile<TILE_IT>(tile, io.obs + ((int64_t)k * N + e0) * O, (int64_t)nvalid * O, lane);
#endif
            wave_lds_sync();
        }
        if (c + 1 < nch) net_wg_sync();   // barrier c + 1
    }
    if (valid) {
#pragma unroll
        for (int j = 0; j < G::J; j++) st_store(P.X + j * S + e, st.X[j]);
#pragma unroll
        for (int r = 0; r < RL; r++) st_store(P.U + r * S + e, st.U[r]);
#pragma unroll
        for (int k = 0; k < G::E; k++) st_store(P.Y + k * S + e, st.Y[k]);
        // ring slot of R[t - a] = age-a window register (zeros before the episode)
#pragma unroll
        for (int k = 0; k < G::E; k++) {
            if (G::L[k] == 0) continue;
#pragma unroll
            for (int a = 1; a <= G::L[k]; a++)
                st_store(P.Rring + (int64_t)(G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k])) * S + e,
                         st.w[G::ring_off[k] + a - 1]);
        }
        if (P.cm.info_demand && last_real) {
#pragma unroll
            for (int r = 0; r < RL; r++) P.cm.info_demand[e * RL + r] = (int64_t)dlast[r];
        }
    }
}

// net_roll_kernel with the observation work moved to a third wave (the
// rollout kernel of compiled networks at every batch size: measured faster
// at 32 768 and 65 536 envs).  One 192-thread workgroup per 64 envs, three
// roles pipelined over chunks of CH launch steps:
//   wave 0 (demand)   the market demands into a ring of RD chunks, chunk c
//                     complete before barrier c; a flat loop of one PTRS
//                     candidate per lane and iteration, so lanes run ahead of
//                     each other's rejections (up to the ring's depth) instead
//                     of every draw waiting for the wave's slowest lane
//   wave 1 (dynamics) consumes chunk c between barriers c and c + 1: spec_core
//                     with the fulfilled orders in an LDS ring per link and
//                     lane, slot (t mod L) (the arrival R[t - L] is read from
//                     the slot this step's R[t] then overwrites; ring rows
//                     older than the episode are masked at use by t >= L, so a
//                     reset zeroes nothing); hands U[t+1], X[t+1] and R[t] of
//                     every step to wave 2 as f32 (the obs dtype) in rec[c & 1]
//   wave 2 (obs)      builds the observations of chunk c between barriers c + 1
//                     and c + 2: the order windows (ages 1 .. L-1, f32, in
//                     registers aligned by age), the LDS tile and its store
// The dynamics wave no longer shifts 61 f64 window registers, converts them
// to f32 or stores the tile each step.  Same arithmetic, in the same order,
// as net_spec_kernel.
template <class G>
struct NetLpos {
    static constexpr int count() {
        int n = 0;
        for (int k = 0; k < G::E; k++) n += G::L[k] > 0 ? 1 : 0;
        return n;
    }
    static constexpr int sumL1() {   // obs window entries older than R[t]
        int n = 0;
        for (int k = 0; k < G::E; k++) n += G::L[k] > 0 ? G::L[k] - 1 : 0;
        return n;
    }
    // rank of link k among the links with L > 0 (its R[t] column in rec)
    static constexpr int rank(int k) {
        int n = 0;
        for (int q = 0; q < k; q++) n += G::L[q] > 0 ? 1 : 0;
        return n;
    }
    // first age-1 register of link k's f32 window (ages 1 .. L-1)
    static constexpr int woff(int k) {
        int n = 0;
        for (int q = 0; q < k; q++) n += G::L[q] > 0 ? G::L[q] - 1 : 0;
        return n;
    }
};

#ifndef NET_ROLL3_CH
#define NET_ROLL3_CH 2   // chunk of the 3-role rollout (LDS: two 192-thread workgroups per CU)
#endif
#ifndef NET_ROLL3_RD
#define NET_ROLL3_RD 8   // demand ring depth in chunks (>= 2): how far the demand wave may run ahead
#endif

template <class G, int CH_>
struct NetRoll3 {
    static constexpr int CH = CH_;
    static constexpr int NR = G::RL + G::J + NetLpos<G>::count();   // rec columns per step
    static constexpr size_t tile_bytes() { return (size_t)((EPW * G::O + 3) / 4) * 4 * sizeof(float); }
    static constexpr size_t rhs_bytes() { return (size_t)G::RL * RHS_LDS_MAX * sizeof(double); }
    static constexpr int RD = NET_ROLL3_RD;
    static constexpr size_t dbuf_bytes() { return (size_t)RD * CH * G::RL * WAVE * sizeof(double); }
    static constexpr size_t ring_bytes() { return (size_t)(G::sumL > 0 ? G::sumL : 1) * WAVE * sizeof(double); }
    static constexpr size_t rec_bytes() { return 2 * (size_t)CH * NR * WAVE * sizeof(float); }
    static constexpr size_t lds() { return tile_bytes() + rhs_bytes() + dbuf_bytes() + ring_bytes() + rec_bytes(); }
};

// POL (invsim_rollout_policy with CONSTANT, ConstantOrderAgent,
// benchmark_NetInvMgmtBacklogEnv.py:119-135): the dynamics wave takes the
// agent's fixed order instead of loading actions, every output is optional,
// and the evaluate_agent sums accumulate in registers (spec_core, as
// net_spec_kernel).
template <class G, int CH_, bool POL, class RG = Pcg>
__global__ void __launch_bounds__(3 * WAVE)
net_roll3o_kernel(NetParams P, int t_start, StepIO<float, float> io, PolicyIO pol) {
    using R3 = NetRoll3<G, CH_>;
    using LP = NetLpos<G>;
    constexpr int O = G::O, CH = R3::CH, RD = R3::RD, RL = G::RL, NR = R3::NR;
    constexpr int TILE_IT = (EPW * O * 4 + 16 * WAVE - 1) / (16 * WAVE);
    extern __shared__ __attribute__((aligned(16))) float n3_lds[];
    char *lb = reinterpret_cast<char *>(n3_lds);
    float *tile = n3_lds;
    double *rhs_l = reinterpret_cast<double *>(lb + R3::tile_bytes());
    double *dbuf = reinterpret_cast<double *>(lb + R3::tile_bytes() + R3::rhs_bytes());     // [RD * CH][RL][WAVE]
    double *ring = reinterpret_cast<double *>(lb + R3::tile_bytes() + R3::rhs_bytes() + R3::dbuf_bytes());
    float *rec = reinterpret_cast<float *>(lb + R3::tile_bytes() + R3::rhs_bytes() + R3::dbuf_bytes() +
                                           R3::ring_bytes());                              // [2][CH][NR][WAVE]
    const int lane = threadIdx.x & (WAVE - 1);
    const int role = threadIdx.x / WAVE;
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const int64_t e0 = (int64_t)blockIdx.x * WAVE;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int64_t el = valid ? e : N - 1;       // padded lanes: the last env's data, never stored
    const int nvalid = (int)((N - e0) < WAVE ? (N - e0) : WAVE);
    const int K = io.K;
    const int nch = (K + CH - 1) / CH;
    if (role == 0) {   // ---- demand wave
        PtrsConst pc[RL];
#pragma unroll
        for (int r = 0; r < RL; r++) pc[r] = P.rl_pc[r];
        constexpr int NT = RHS_LDS_MAX / WAVE;
        double tv[RL][NT];
#pragma unroll
        for (int r = 0; r < RL; r++) {
            const int qm = pc[r].nk > 0 ? pc[r].nk - 1 : 0;
            const double *src = pc[r].nk > 0 ? P.rhs + pc[r].toff : P.alpha_pow;   // any valid pointer
#pragma unroll
            for (int u = 0; u < NT; u++) tv[r][u] = src[min(lane + u * WAVE, qm)];
        }
        RG g;
        P.cm.rng.load(el, g);
#pragma unroll
        for (int r = 0; r < RL; r++)
#pragma unroll
            for (int u = 0; u < NT; u++) rhs_l[r * RHS_LDS_MAX + lane + u * WAVE] = tv[r][u];
        wave_lds_sync();
        // flat draw loop (stream_flat_loop): up to RD chunks ahead of the dynamics;
        // barriers 0 .. nch - 1 (demand chunk c ready), nch (the obs wave's last chunk)
        net_demand_loop<G, CH, RD>(g, pc, rhs_l, dbuf, lane, K, nch + 1, t_start, P.T, P.cm.ph_step);
        if (valid) P.cm.rng.store_state(e, g);
        return;
    }
    if (role == 2) {   // ---- obs wave
        float *trow = tile + lane * O;
        int t = t_start;
        // f32 order windows, ages 1 .. L-1: wf[woff(k) + a - 1] = R[t - a] (zeros before the episode)
        float wf[LP::sumL1() > 0 ? LP::sumL1() : 1];
#pragma unroll
        for (int k = 0; k < G::E; k++) {
            if (G::L[k] <= 1) continue;
#pragma unroll
            for (int a = 1; a < G::L[k]; a++) {
                const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
                const double v = P.Rring[(int64_t)row * S + el];
                wf[LP::woff(k) + a - 1] = (t - a >= 0) ? (float)v : 0.f;
            }
        }
        net_wg_sync();   // barrier 0
        for (int c = 0; c < nch; c++) {
            net_wg_sync();   // barrier c + 1: record chunk c ready
            const float *rb = rec + (c & 1) * CH * NR * WAVE;
            for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
                const int k = c * CH + kk;
#ifdef INVSIM_ABL_R3_NO_OBS
                continue;
#endif
                if (t >= P.T) {                    // NEXT_STEP autoreset: [0, I0, 0 ...] (:301-332)
#pragma unroll
                    for (int r = 0; r < RL; r++) trow[r] = 0.f;
#pragma unroll
                    for (int j = 0; j < G::J; j++) trow[RL + j] = (float)G::I0[j];
#pragma unroll
                    for (int q = 0; q < G::sumL; q++) trow[RL + G::J + q] = 0.f;
#pragma unroll
                    for (int q = 0; q < LP::sumL1(); q++) wf[q] = 0.f;
                    t = 0;
                } else {
                    // obs (:334-413): U[t+1], X[t+1], then per link with L > 0
                    // R[t+1-L .. t] oldest first (ages L-1 .. 1, then R[t])
#pragma unroll
                    for (int q = 0; q < RL + G::J; q++) trow[q] = rb[(kk * NR + q) * WAVE + lane];
#pragma unroll
                    for (int kl = 0; kl < G::E; kl++) {
                        if (G::L[kl] == 0) continue;
                        const float rn = rb[(kk * NR + RL + G::J + LP::rank(kl)) * WAVE + lane];
#pragma unroll
                        for (int p = 0; p + 1 < G::L[kl]; p++)
                            trow[G::win_off[kl] + p] = wf[LP::woff(kl) + (G::L[kl] - 1 - p) - 1];
                        trow[G::win_off[kl] + G::L[kl] - 1] = rn;
                        // age the window: age a + 1 <- age a, age 1 <- R[t]
#pragma unroll
                        for (int a = G::L[kl] - 1; a >= 2; a--) wf[LP::woff(kl) + a - 1] = wf[LP::woff(kl) + a - 2];
                        if (G::L[kl] > 1) wf[LP::woff(kl)] = rn;
                    }
                    t += 1;
                }
                wave_lds_sync();
#ifndef INVSIM_ABL_ROLL_NO_STORE
                if (!POL || io.obs) store_tile<TILE_IT>(tile, io.obs + ((int64_t)k * N + e0) * O, (int64_t)nvalid * O, lane);
#endif
                wave_lds_sync();
            }
        }
        return;
    }
    // ---- dynamics wave
    double *rg = ring + lane;                   // [sumL][WAVE]: R[t'] of link k at row ring_off[k] + t' mod L
    int t = t_start;
    NetSt<G> st;
#pragma unroll
    for (int j = 0; j < G::J; j++) st.X[j] = P.X[j * S + el];
#pragma unroll
    for (int r = 0; r < RL; r++) st.U[r] = P.U[r * S + el];
#pragma unroll
    for (int k = 0; k < G::E; k++) st.Y[k] = P.Y[k * S + el];
    {
        double rv[G::sumL > 0 ? G::sumL : 1];
#pragma unroll
        for (int q = 0; q < G::sumL; q++) rv[q] = P.Rring[(int64_t)q * S + el];
#pragma unroll
        for (int q = 0; q < G::sumL; q++) rg[q * WAVE] = rv[q];
    }
    float nact[G::E];
#pragma unroll
    for (int k = 0; k < G::E; k++) nact[k] = POL ? pol.cf[k] : io.act[el * G::E + k];
    constexpr int MD = 5 + G::J;             // metrics: reward, steps, demand, sales, stockout, X per node
    double met[MD];
#pragma unroll
    for (int q = 0; q < MD; q++) met[q] = (POL && pol.metrics) ? pol.metrics[el * MD + q] : 0.0;
    double napow = P.alpha_pow[t < P.T ? t : 0];
    double dlast[RL];
#pragma unroll
    for (int r = 0; r < RL; r++) dlast[r] = 0.0;
    bool last_real = false;
    double Rn[G::E];
    net_wg_sync();   // barrier 0: demand chunk 0 ready
    for (int c = 0; c < nch; c++) {
        const double *db = dbuf + (c % RD) * CH * RL * WAVE;
        float *rb = rec + (c & 1) * CH * NR * WAVE;
        for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
            const int k = c * CH + kk;
            const int64_t oi = (int64_t)k * N + e;
            float act[G::E];
#pragma unroll
            for (int q = 0; q < G::E; q++) act[q] = nact[q];
            const double apow = napow;
            {
                const int tn = (t >= P.T) ? 0 : t + 1;          // the next launch step's period
                napow = P.alpha_pow[tn < P.T ? tn : 0];
            }
            if (!POL && k + 1 < K) {                            // the next step's actions
#pragma unroll
                for (int q = 0; q < G::E; q++) nact[q] = io.act[((int64_t)(k + 1) * N + el) * G::E + q];
            }
            if (t >= P.T) {                                     // NEXT_STEP autoreset (:301-332)
#pragma unroll
                for (int j = 0; j < G::J; j++) st.X[j] = G::I0[j];
#pragma unroll
                for (int r = 0; r < RL; r++) st.U[r] = 0.0;
#pragma unroll
                for (int q = 0; q < G::E; q++) st.Y[q] = 0.0;
                if (valid && (!POL || io.rew)) {
                    out_store(io.rew + oi, 0.0);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)0);
                }
                t = 0;
            } else {
                double Dd[RL], wa[G::E];
#pragma unroll
                for (int r = 0; r < RL; r++) Dd[r] = db[(kk * RL + r) * WAVE + lane];
#pragma unroll
                for (int q = 0; q < G::E; q++) {               // arrival R[t - L] (zero before the episode)
                    if (G::L[q] == 0) {
                        wa[q] = 0.0;
                        continue;
                    }
                    const double v = rg[(G::ring_off[q] + (int)((uint32_t)t % (uint32_t)G::L[q])) * WAVE];
                    wa[q] = (t >= G::L[q]) ? v : 0.0;
                }
                const double rw = spec_core<G>(P, apow, st, act, Dd, wa, Rn, POL ? met : nullptr, nullptr);
                if (POL) {
                    met[0] += rw;                                       // episode_reward += reward
                    met[1] += 1.0;
                    if (valid && pol.act_out) {
#pragma unroll
                        for (int q = 0; q < G::E; q++) out_store((float *)pol.act_out + oi * G::E + q, act[q]);
                    }
                }
#pragma unroll
                for (int q = 0; q < G::E; q++)
                    if (G::L[q] > 0) rg[(G::ring_off[q] + (int)((uint32_t)t % (uint32_t)G::L[q])) * WAVE] = Rn[q];
#pragma unroll
                for (int r = 0; r < RL; r++) rb[(kk * NR + r) * WAVE + lane] = (float)st.U[r];
#pragma unroll
                for (int j = 0; j < G::J; j++) rb[(kk * NR + RL + j) * WAVE + lane] = (float)st.X[j];
#pragma unroll
                for (int q = 0; q < G::E; q++)
                    if (G::L[q] > 0) rb[(kk * NR + RL + G::J + LP::rank(q)) * WAVE + lane] = (float)Rn[q];
                if (valid && (!POL || io.rew)) {
                    out_store(io.rew + oi, rw);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)(t + 1 >= P.T ? 1 : 0));
                }
#pragma unroll
                for (int r = 0; r < RL; r++) dlast[r] = Dd[r];
                last_real = k == K - 1;
                t += 1;
            }
        }
        net_wg_sync();   // barrier c + 1: demand chunk c + 1 and record chunk c ready
    }
    if (valid) {
#pragma unroll
        for (int j = 0; j < G::J; j++) st_store(P.X + j * S + e, st.X[j]);
#pragma unroll
        for (int r = 0; r < RL; r++) st_store(P.U + r * S + e, st.U[r]);
#pragma unroll
        for (int k = 0; k < G::E; k++) st_store(P.Y + k * S + e, st.Y[k]);
        // ring rows older than the episode are stored as zeros (the reference's zeroed history)
#pragma unroll
        for (int k = 0; k < G::E; k++) {
            if (G::L[k] == 0) continue;
#pragma unroll
            for (int a = 1; a <= G::L[k]; a++) {
                const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
                const double v = rg[row * WAVE];
                st_store(P.Rring + (int64_t)row * S + e, (t - a >= 0) ? v : 0.0);
            }
        }
        if (P.cm.info_demand && last_real) {
#pragma unroll
            for (int r = 0; r < RL; r++) P.cm.info_demand[e * RL + r] = (int64_t)dlast[r];
        }
        if (POL && pol.metrics) {
#pragma unroll
            for (int q = 0; q < MD; q++) pol.metrics[e * MD + q] = met[q];
        }
    }
}

// ---------------------------------------------------------------- 4 roles
// net_roll3o_kernel with the period's profit on a wave of its own, for batches
// up to 256 workgroups (one per CU: the record below takes the LDS).  At small
// shards every role has a SIMD to itself and the dynamics wave's instruction
// chain is the step time: ~425 instructions, 240 of them f64, about half of
// those the per-node profit sums (spec_profit).  One 256-thread workgroup per
// 64 envs:
//   wave 0 (demand)   as net_roll3o_kernel's
//   wave 1 (flow)     spec_flow (orders, pipeline, arrivals, market) with the
//                     order rings in LDS; hands R[t], the market sales,
//                     X[t+1], Y[t+1] and U[t+1] of every step to waves 2 and 3
//                     in the f64 record rec4[c & 1]
//   wave 2 (obs)      as net_roll3o_kernel's, from rec4 (rounded to f32)
//   wave 3 (profit)   spec_profit and apow * total from rec4, and the reward,
//                     terminated and truncated outputs, one chunk behind the
//                     flow wave
// Same arithmetic, in the same order, as net_spec_kernel.
template <class G>
struct NetRoll4 {
    static constexpr int CH = NET_ROLL3_CH, RD = NET_ROLL3_RD;
    static constexpr int NR4 = 2 * G::E + 2 * G::RL + G::J;            // rec4 columns: R, Sr, X, Y, U
    static constexpr int AP = 256;                                     // alpha**t in LDS (T <= AP)
    static constexpr size_t tile_bytes() { return (size_t)((EPW * G::O + 3) / 4) * 4 * sizeof(float); }
    static constexpr size_t rhs_bytes() { return (size_t)G::RL * RHS_LDS_MAX * sizeof(double); }
    static constexpr size_t dbuf_bytes() { return (size_t)RD * CH * G::RL * WAVE * sizeof(double); }
    static constexpr size_t ring_bytes() { return (size_t)(G::sumL > 0 ? G::sumL : 1) * WAVE * sizeof(double); }
    static constexpr size_t rec_bytes() { return 2 * (size_t)CH * NR4 * WAVE * sizeof(double); }
    static constexpr size_t lds() {
        return tile_bytes() + rhs_bytes() + dbuf_bytes() + ring_bytes() + rec_bytes() + AP * sizeof(double);
    }
    // rec4 column of R[t] link k, the sales of market r, X[t+1] node j, Y[t+1] link k, U[t+1] market r
    static constexpr int cR(int k) { return k; }
    static constexpr int cS(int r) { return G::E + r; }
    static constexpr int cX(int j) { return G::E + G::RL + j; }
    static constexpr int cY(int k) { return G::E + G::RL + G::J + k; }
    static constexpr int cU(int r) { return 2 * G::E + G::RL + G::J + r; }
};

template <class G, class RG = Pcg>
__global__ void __launch_bounds__(4 * WAVE)
net_roll4_kernel(NetParams P, int t_start, StepIO<float, float> io) {
    using R4 = NetRoll4<G>;
    using LP = NetLpos<G>;
    constexpr int O = G::O, CH = R4::CH, RD = R4::RD, RL = G::RL, NR4 = R4::NR4, E = G::E, J = G::J;
    constexpr int TILE_IT = (EPW * O * 4 + 16 * WAVE - 1) / (16 * WAVE);
    extern __shared__ __attribute__((aligned(16))) float n4_lds[];
    char *lb = reinterpret_cast<char *>(n4_lds);
    float *tile = n4_lds;
    double *rhs_l = reinterpret_cast<double *>(lb + R4::tile_bytes());
    double *dbuf = reinterpret_cast<double *>(lb + R4::tile_bytes() + R4::rhs_bytes());     // [RD * CH][RL][WAVE]
    double *ring = reinterpret_cast<double *>(lb + R4::tile_bytes() + R4::rhs_bytes() + R4::dbuf_bytes());
    double *rec = reinterpret_cast<double *>(lb + R4::tile_bytes() + R4::rhs_bytes() + R4::dbuf_bytes() +
                                             R4::ring_bytes());                              // [2][CH][NR4][WAVE]
    double *ap_l = rec + 2 * CH * NR4 * WAVE;                                                // alpha**t, t < T
    const int lane = threadIdx.x & (WAVE - 1);
    const int role = threadIdx.x / WAVE;
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const int64_t e0 = (int64_t)blockIdx.x * WAVE;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int64_t el = valid ? e : N - 1;       // padded lanes: the last env's data, never stored
    const int nvalid = (int)((N - e0) < WAVE ? (N - e0) : WAVE);
    const int K = io.K;
    const int nch = (K + CH - 1) / CH;
    if (role == 0) {   // ---- demand wave
        PtrsConst pc[RL];
#pragma unroll
        for (int r = 0; r < RL; r++) pc[r] = P.rl_pc[r];
        constexpr int NT = RHS_LDS_MAX / WAVE;
        double tv[RL][NT];
#pragma unroll
        for (int r = 0; r < RL; r++) {
            const int qm = pc[r].nk > 0 ? pc[r].nk - 1 : 0;
            const double *src = pc[r].nk > 0 ? P.rhs + pc[r].toff : P.alpha_pow;   // any valid pointer
#pragma unroll
            for (int u = 0; u < NT; u++) tv[r][u] = src[min(lane + u * WAVE, qm)];
        }
        RG g;
        P.cm.rng.load(el, g);
        for (int x = lane; x < P.T; x += WAVE) ap_l[x] = P.alpha_pow[x];   // before barrier 0
#pragma unroll
        for (int r = 0; r < RL; r++)
#pragma unroll
            for (int u = 0; u < NT; u++) rhs_l[r * RHS_LDS_MAX + lane + u * WAVE] = tv[r][u];
        wave_lds_sync();
        net_demand_loop<G, CH, RD>(g, pc, rhs_l, dbuf, lane, K, nch + 1, t_start, P.T, P.cm.ph_step);
        if (valid) P.cm.rng.store_state(e, g);
        return;
    }
    if (role == 2) {   // ---- obs wave
        float *trow = tile + lane * O;
        int t = t_start;
        float wf[LP::sumL1() > 0 ? LP::sumL1() : 1];
#pragma unroll
        for (int k = 0; k < E; k++) {
            if (G::L[k] <= 1) continue;
#pragma unroll
            for (int a = 1; a < G::L[k]; a++) {
                const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
                const double v = P.Rring[(int64_t)row * S + el];
                wf[LP::woff(k) + a - 1] = (t - a >= 0) ? (float)v : 0.f;
            }
        }
        net_wg_sync();   // barrier 0
        for (int c = 0; c < nch; c++) {
            net_wg_sync();   // barrier c + 1: record chunk c ready
            const double *rb = rec + (c & 1) * CH * NR4 * WAVE;
            for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
                const int k = c * CH + kk;
                if (t >= P.T) {                    // NEXT_STEP autoreset: [0, I0, 0 ...] (:301-332)
#pragma unroll
                    for (int r = 0; r < RL; r++) trow[r] = 0.f;
#pragma unroll
                    for (int j = 0; j < J; j++) trow[RL + j] = (float)G::I0[j];
#pragma unroll
                    for (int q = 0; q < G::sumL; q++) trow[RL + J + q] = 0.f;
#pragma unroll
                    for (int q = 0; q < LP::sumL1(); q++) wf[q] = 0.f;
                    t = 0;
                } else {
#pragma unroll
                    for (int r = 0; r < RL; r++) trow[r] = (float)rb[(kk * NR4 + R4::cU(r)) * WAVE + lane];
#pragma unroll
                    for (int j = 0; j < J; j++) trow[RL + j] = (float)rb[(kk * NR4 + R4::cX(j)) * WAVE + lane];
#pragma unroll
                    for (int kl = 0; kl < E; kl++) {
                        if (G::L[kl] == 0) continue;
                        const float rn = (float)rb[(kk * NR4 + R4::cR(kl)) * WAVE + lane];
#pragma unroll
                        for (int p = 0; p + 1 < G::L[kl]; p++)
                            trow[G::win_off[kl] + p] = wf[LP::woff(kl) + (G::L[kl] - 1 - p) - 1];
                        trow[G::win_off[kl] + G::L[kl] - 1] = rn;
#pragma unroll
                        for (int a = G::L[kl] - 1; a >= 2; a--) wf[LP::woff(kl) + a - 1] = wf[LP::woff(kl) + a - 2];
                        if (G::L[kl] > 1) wf[LP::woff(kl)] = rn;
                    }
                    t += 1;
                }
                wave_lds_sync();
                store_tile<TILE_IT>(tile, io.obs + ((int64_t)k * N + e0) * O, (int64_t)nvalid * O, lane);
                wave_lds_sync();
            }
        }
        return;
    }
    if (role == 3) {   // ---- profit wave
        int t = t_start;
        net_wg_sync();   // barrier 0
        for (int c = 0; c < nch; c++) {
            net_wg_sync();   // barrier c + 1: record chunk c ready
            const double *rb = rec + (c & 1) * CH * NR4 * WAVE;
            for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
                const int64_t oi = (int64_t)(c * CH + kk) * N + e;
                if (t >= P.T) {                    // the NEXT_STEP reset step: reward 0, no flag
                    if (valid) {
                        out_store(io.rew + oi, 0.0);
                        out_store(io.term + oi, (uint8_t)0);
                        out_store(io.trunc + oi, (uint8_t)0);
                    }
                    t = 0;
                    continue;
                }
                double Rn[E], Sr[RL], X[J], Y[E], U[RL];
#pragma unroll
                for (int k = 0; k < E; k++) Rn[k] = rb[(kk * NR4 + R4::cR(k)) * WAVE + lane];
#pragma unroll
                for (int r = 0; r < RL; r++) Sr[r] = rb[(kk * NR4 + R4::cS(r)) * WAVE + lane];
#pragma unroll
                for (int j = 0; j < J; j++) X[j] = rb[(kk * NR4 + R4::cX(j)) * WAVE + lane];
#pragma unroll
                for (int k = 0; k < E; k++) Y[k] = rb[(kk * NR4 + R4::cY(k)) * WAVE + lane];
#pragma unroll
                for (int r = 0; r < RL; r++) U[r] = rb[(kk * NR4 + R4::cU(r)) * WAVE + lane];
                const double rw = ap_l[t] * spec_profit<G>(Rn, Sr, X, Y, U, nullptr);   // :619
                if (valid) {
                    out_store(io.rew + oi, rw);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)(t + 1 >= P.T ? 1 : 0));
                }
                t += 1;
            }
        }
        return;
    }
    // ---- flow wave
    double *rg = ring + lane;                   // [sumL][WAVE]: R[t'] of link k at row ring_off[k] + t' mod L
    int t = t_start;
    NetSt<G> st;
#pragma unroll
    for (int j = 0; j < J; j++) st.X[j] = P.X[j * S + el];
#pragma unroll
    for (int r = 0; r < RL; r++) st.U[r] = P.U[r * S + el];
#pragma unroll
    for (int k = 0; k < E; k++) st.Y[k] = P.Y[k * S + el];
    {
        double rv[G::sumL > 0 ? G::sumL : 1];
#pragma unroll
        for (int q = 0; q < G::sumL; q++) rv[q] = P.Rring[(int64_t)q * S + el];
#pragma unroll
        for (int q = 0; q < G::sumL; q++) rg[q * WAVE] = rv[q];
    }
    float nact[E];
#pragma unroll
    for (int k = 0; k < E; k++) nact[k] = io.act[el * E + k];
    double Rn[E];
    net_wg_sync();   // barrier 0: demand chunk 0 ready
    for (int c = 0; c < nch; c++) {
        const double *db = dbuf + (c % RD) * CH * RL * WAVE;
        double *rb = rec + (c & 1) * CH * NR4 * WAVE;
        for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
            const int k = c * CH + kk;
            float act[E];
#pragma unroll
            for (int q = 0; q < E; q++) act[q] = nact[q];
            if (k + 1 < K) {                                    // the next step's actions
#pragma unroll
                for (int q = 0; q < E; q++) nact[q] = io.act[((int64_t)(k + 1) * N + el) * E + q];
            }
            if (t >= P.T) {                                     // NEXT_STEP autoreset (:301-332)
#pragma unroll
                for (int j = 0; j < J; j++) st.X[j] = G::I0[j];
#pragma unroll
                for (int r = 0; r < RL; r++) st.U[r] = 0.0;
#pragma unroll
                for (int q = 0; q < E; q++) st.Y[q] = 0.0;
                t = 0;
            } else {
                double Dd[RL], wa[E], Sr[RL];
#pragma unroll
                for (int r = 0; r < RL; r++) Dd[r] = db[(kk * RL + r) * WAVE + lane];
#pragma unroll
                for (int q = 0; q < E; q++) {                  // arrival R[t - L] (zero before the episode)
                    if (G::L[q] == 0) {
                        wa[q] = 0.0;
                        continue;
                    }
                    const double v = rg[(G::ring_off[q] + (int)((uint32_t)t % (uint32_t)G::L[q])) * WAVE];
                    wa[q] = (t >= G::L[q]) ? v : 0.0;
                }
                spec_flow<G>(P, st, act, Dd, wa, Rn, Sr);
#pragma unroll
                for (int q = 0; q < E; q++)
                    if (G::L[q] > 0) rg[(G::ring_off[q] + (int)((uint32_t)t % (uint32_t)G::L[q])) * WAVE] = Rn[q];
#pragma unroll
                for (int q = 0; q < E; q++) {
                    rb[(kk * NR4 + R4::cR(q)) * WAVE + lane] = Rn[q];
                    rb[(kk * NR4 + R4::cY(q)) * WAVE + lane] = st.Y[q];
                }
#pragma unroll
                for (int r = 0; r < RL; r++) {
                    rb[(kk * NR4 + R4::cS(r)) * WAVE + lane] = Sr[r];
                    rb[(kk * NR4 + R4::cU(r)) * WAVE + lane] = st.U[r];
                }
#pragma unroll
                for (int j = 0; j < J; j++) rb[(kk * NR4 + R4::cX(j)) * WAVE + lane] = st.X[j];
                t += 1;
            }
        }
        net_wg_sync();   // barrier c + 1: demand chunk c + 1 and record chunk c ready
    }
    if (valid) {
#pragma unroll
        for (int j = 0; j < J; j++) st_store(P.X + j * S + e, st.X[j]);
#pragma unroll
        for (int r = 0; r < RL; r++) st_store(P.U + r * S + e, st.U[r]);
#pragma unroll
        for (int k = 0; k < E; k++) st_store(P.Y + k * S + e, st.Y[k]);
        // ring rows older than the episode are stored as zeros (the reference's zeroed history)
#pragma unroll
        for (int k = 0; k < E; k++) {
            if (G::L[k] == 0) continue;
#pragma unroll
            for (int a = 1; a <= G::L[k]; a++) {
                const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
                const double v = rg[row * WAVE];
                st_store(P.Rring + (int64_t)row * S + e, (t - a >= 0) ? v : 0.0);
            }
        }
    }
}

// ---------------------------------------------------------------- small shards
// The K-step rollout for small per-GPU shards (config 5 split over 8 GPUs:
// 4 096 envs per rank).  There the 3-role kernel runs one dynamics wave per
// 64 envs on 64 of the 1 024 SIMDs, and each of those waves issues the whole
// step, ~425 instructions of which 240 are f64 (half rate on MI355X: 8 cycles
// per wave instruction), one env per lane: 1.3 us per step, with the demand
// draws and the observation work hidden beside it (ablation builds,
// profiles/r06/net_small/ablation.txt).  Fewer envs per wave do not shorten
// that chain; spreading ONE env's edge work over lanes does.
//
// net_rollq_kernel: one 16-lane DPP row per env, 4 envs per dynamics wave.
// Lane l of an env's row is reorder link l (l < E) and main node l (l < J):
//   * order fulfilment (:448-490): every link lane evaluates its own order in
//     the same instructions.  Links of one supplier are consecutive and
//     draw on the supplier's running consumption in link order, so the
//     lanes run in rounds by their rank within the supplier: round r's lanes
//     take the consumption of lane l - 1 (DPP row_shr:1) from round r - 1 --
//     a segmented clamp-scan in the reference's order;
//   * pipeline and arrivals (:494-528): each link lane keeps its own order
//     ring in LDS and updates its pipeline Y; node lane j gathers its
//     predecessor links' arrivals (ds_bpermute within the row) and adds them
//     in predecessor-adjacency order, then subtracts the supplier
//     consumption of its last link;
//   * market fulfilment (:536-566) on the lane of the market's node;
//   * profit (:578-613): link lanes form lp * R and lg * max(0, Y); node lane
//     j gathers its successors' and predecessors' terms in the same sum
//     orders as spec_core and forms its node profit; the period total is a
//     sequential scan over the node lanes in node order (row_shr:1, J - 1
//     steps), the reference's `total_profit_period += node_profit`.
// Every sum keeps spec_core's operand order, so results are bit-identical.
// Roles per 16-env workgroup: wave 0 draws the demands (net_demand_loop, one
// env per lane), wave 1 builds the observations one chunk behind (as
// net_roll3o_kernel's obs wave), waves 2-5 are the dynamics waves.
template <class G>
struct NetQ {
    static constexpr int QE = 16;                              // envs per workgroup
    static constexpr int QW = 4;                               // dynamics waves (4 envs each)
    static_assert(G::E <= 16 && G::J <= 16, "one 16-lane row per env");
    static constexpr int sup_rank(int k) {                     // rank of link k among its supplier's links
        int r = 0;
        for (int q = 0; q < k; q++) r += (G::sup[k] >= 0 && G::sup[q] == G::sup[k]) ? 1 : 0;
        return r;
    }
    static constexpr bool sup_consecutive() {                  // a supplier's links are adjacent
        for (int k = 1; k < G::E; k++)
            if (G::sup[k] >= 0 && sup_rank(k) > 0 && G::sup[k - 1] != G::sup[k]) return false;
        return true;
    }
    static_assert(sup_consecutive(), "the clamp-scan takes a supplier's links as consecutive lanes");
    static constexpr int rmax() {
        int m = 0;
        for (int k = 0; k < G::E; k++) m = sup_rank(k) + 1 > m ? sup_rank(k) + 1 : m;
        return m;
    }
    static constexpr int last_link(int j) {                    // the supplier's last link, or -1
        int l = -1;
        for (int k = 0; k < G::E; k++) l = G::sup[k] == j ? k : l;
        return l;
    }
    static constexpr int market(int j) {                       // the market of node j, or -1
        int m = -1;
        for (int r = 0; r < G::RL; r++) m = G::rl_node[r] == j ? r : m;
        return m;
    }
    static constexpr bool one_market_per_node() {
        for (int j = 0; j < G::J; j++) {
            int n = 0;
            for (int r = 0; r < G::RL; r++) n += G::rl_node[r] == j ? 1 : 0;
            if (n > 1) return false;
        }
        return true;
    }
    static_assert(one_market_per_node(), "a node lane serves at most one market");
    static constexpr int pmax() {
        int m = 0;
        for (int j = 0; j < G::J; j++) m = G::pred_ptr[j + 1] - G::pred_ptr[j] > m ? G::pred_ptr[j + 1] - G::pred_ptr[j] : m;
        return m;
    }
    static constexpr int smax() {
        int m = 0;
        for (int j = 0; j < G::J; j++) m = G::succ_ptr[j + 1] - G::succ_ptr[j] > m ? G::succ_ptr[j + 1] - G::succ_ptr[j] : m;
        return m;
    }
    static constexpr int NR = G::RL + G::J + NetLpos<G>::count();   // obs record columns per step
    // chunk of 4 launch steps: the dynamics lanes load chunk c + 1's actions at
    // the start of chunk c, 4-7 steps before their use (a load one step ahead
    // waits, in vmcnt order, behind the previous step's stores)
    static constexpr int CH = 4, RD = 4;
    static constexpr int AP = 256;                             // alpha**t in LDS (T <= AP)
    static constexpr size_t tile_bytes() { return (size_t)((QE * G::O + 3) / 4) * 4 * sizeof(float); }
    static constexpr size_t rhs_bytes() { return (size_t)G::RL * RHS_LDS_MAX * sizeof(double); }
    static constexpr size_t dbuf_bytes() { return (size_t)RD * CH * G::RL * WAVE * sizeof(double); }
    static constexpr size_t ring_bytes() { return (size_t)(G::sumL > 0 ? G::sumL : 1) * QE * sizeof(double); }
    static constexpr size_t rec_bytes() { return 2 * (size_t)CH * NR * WAVE * sizeof(float); }
    static constexpr size_t lds() {
        return tile_bytes() + rhs_bytes() + dbuf_bytes() + ring_bytes() + rec_bytes() + AP * sizeof(double);
    }
};

// a per-lane constant: f(i) of this lane's index i (< n), else dflt (a select chain, once per launch)
template <int n, class T, class F>
__device__ __forceinline__ T lane_const(int i, T dflt, F f) {
    T v = dflt;
#pragma unroll
    for (int q = 0; q < n; q++)
        if (i == q) v = f(q);
    return v;
}

// lane (row base + src)'s value (ds_bpermute within the env's row)
__device__ __forceinline__ double row_get(double v, int rowbase, int src) { return __shfl(v, rowbase + src); }

// lane l - 1's value within a 16-lane row (DPP row_shr:1; lane 0 of a row gets 0)
__device__ __forceinline__ double row_shr1(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x111, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x111, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

template <class G, class RG = Pcg>
__global__ void __launch_bounds__(6 * WAVE)
net_rollq_kernel(NetParams P, int t_start, StepIO<float, float> io) {
    using Q = NetQ<G>;
    using LP = NetLpos<G>;
    constexpr int O = G::O, CH = Q::CH, RD = Q::RD, RL = G::RL, NR = Q::NR, QE = Q::QE, E = G::E, J = G::J;
    constexpr int TILE_IT = (QE * O * 4 + 16 * WAVE - 1) / (16 * WAVE);
    extern __shared__ __attribute__((aligned(16))) float nq_lds[];
    char *lb = reinterpret_cast<char *>(nq_lds);
    float *tile = nq_lds;
    double *rhs_l = reinterpret_cast<double *>(lb + Q::tile_bytes());
    double *dbuf = reinterpret_cast<double *>(lb + Q::tile_bytes() + Q::rhs_bytes());       // [RD * CH][RL][WAVE]
    double *ring = reinterpret_cast<double *>(lb + Q::tile_bytes() + Q::rhs_bytes() + Q::dbuf_bytes());   // [sumL][QE]
    float *rec = reinterpret_cast<float *>(lb + Q::tile_bytes() + Q::rhs_bytes() + Q::dbuf_bytes() +
                                           Q::ring_bytes());                                // [2][CH][NR][WAVE]
    double *ap_l = reinterpret_cast<double *>(lb + Q::tile_bytes() + Q::rhs_bytes() + Q::dbuf_bytes() +
                                              Q::ring_bytes() + Q::rec_bytes());            // alpha**t, t < T
    const int lane = threadIdx.x & (WAVE - 1);
    const int w = threadIdx.x / WAVE;
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const int64_t e0 = (int64_t)blockIdx.x * QE;
    const int nvalid = (int)((N - e0) < QE ? (N - e0) : QE);
    const int K = io.K;
    const int nch = (K + CH - 1) / CH;
    if (w < 2) {
        // one env per lane (lanes >= QE repeat lane & (QE - 1)'s env and store nothing)
        const int q = lane & (QE - 1);
        const int64_t e = e0 + q;
        const bool valid = lane < QE && e < N;
        const int64_t el = e < N ? e : N - 1;
        if (w == 0) {   // ---- demand wave (as net_roll3o_kernel's)
            PtrsConst pc[RL];
#pragma unroll
            for (int r = 0; r < RL; r++) pc[r] = P.rl_pc[r];
            constexpr int NT = RHS_LDS_MAX / WAVE;
            double tv[RL][NT];
#pragma unroll
            for (int r = 0; r < RL; r++) {
                const int qm = pc[r].nk > 0 ? pc[r].nk - 1 : 0;
                const double *src = pc[r].nk > 0 ? P.rhs + pc[r].toff : P.alpha_pow;   // any valid pointer
#pragma unroll
                for (int u = 0; u < NT; u++) tv[r][u] = src[min(lane + u * WAVE, qm)];
            }
            RG g;
            P.cm.rng.load(el, g);
#pragma unroll
            for (int r = 0; r < RL; r++)
#pragma unroll
                for (int u = 0; u < NT; u++) rhs_l[r * RHS_LDS_MAX + lane + u * WAVE] = tv[r][u];
            wave_lds_sync();
            net_demand_loop<G, CH, RD>(g, pc, rhs_l, dbuf, lane, K, nch + 1, t_start, P.T, P.cm.ph_step);
            if (valid) P.cm.rng.store_state(e, g);
            return;
        }
        // ---- obs wave (as net_roll3o_kernel's, QE envs)
        float *trow = tile + q * O;
        int t = t_start;
        float wf[LP::sumL1() > 0 ? LP::sumL1() : 1];
#pragma unroll
        for (int k = 0; k < E; k++) {
            if (G::L[k] <= 1) continue;
#pragma unroll
            for (int a = 1; a < G::L[k]; a++) {
                const int row = G::ring_off[k] + (int)((uint32_t)(t - a + 256 * G::L[k]) % (uint32_t)G::L[k]);
                const double v = P.Rring[(int64_t)row * S + el];
                wf[LP::woff(k) + a - 1] = (t - a >= 0) ? (float)v : 0.f;
            }
        }
        net_wg_sync();   // barrier 0
        for (int c = 0; c < nch; c++) {
            net_wg_sync();   // barrier c + 1: record chunk c ready
            const float *rb = rec + (c & 1) * CH * NR * WAVE;
            for (int kk = 0; kk < CH && c * CH + kk < K; kk++) {
                const int k = c * CH + kk;
#ifdef INVSIM_ABL_R3_NO_OBS
                continue;
#endif
                if (lane < QE) {
                    if (t >= P.T) {                    // NEXT_STEP autoreset: [0, I0, 0 ...] (:301-332)
#pragma unroll
                        for (int r = 0; r < RL; r++) trow[r] = 0.f;
#pragma unroll
                        for (int j = 0; j < J; j++) trow[RL + j] = (float)G::I0[j];
#pragma unroll
                        for (int x = 0; x < G::sumL; x++) trow[RL + J + x] = 0.f;
#pragma unroll
                        for (int x = 0; x < LP::sumL1(); x++) wf[x] = 0.f;
                    } else {
#pragma unroll
                        for (int x = 0; x < RL + J; x++) trow[x] = rb[(kk * NR + x) * WAVE + q];
#pragma unroll
                        for (int kl = 0; kl < E; kl++) {
                            if (G::L[kl] == 0) continue;
                            const float rn = rb[(kk * NR + RL + J + LP::rank(kl)) * WAVE + q];
#pragma unroll
                            for (int p = 0; p + 1 < G::L[kl]; p++)
                                trow[G::win_off[kl] + p] = wf[LP::woff(kl) + (G::L[kl] - 1 - p) - 1];
                            trow[G::win_off[kl] + G::L[kl] - 1] = rn;
#pragma unroll
                            for (int a = G::L[kl] - 1; a >= 2; a--) wf[LP::woff(kl) + a - 1] = wf[LP::woff(kl) + a - 2];
                            if (G::L[kl] > 1) wf[LP::woff(kl)] = rn;
                        }
                    }
                }
                t = (t >= P.T) ? 0 : t + 1;
                wave_lds_sync();
#ifndef INVSIM_ABL_ROLL_NO_STORE
                store_tile<TILE_IT>(tile, io.obs + ((int64_t)k * N + e0) * O, (int64_t)nvalid * O, lane);
#endif
                wave_lds_sync();
            }
        }
        return;
    }
    // ---- dynamics waves: env row (lane >> 4), lane l = link l / node l of that env
    const int l = lane & 15;
    const int rowbase = lane & ~15;
    const int q = (w - 2) * 4 + (lane >> 4);                 // env within the workgroup
    const int64_t e = e0 + q;
    const bool valid = e < N;
    const int64_t el = valid ? e : N - 1;
    // link-lane constants (lanes >= E: a raw-material link that orders nothing)
    const bool is_link = l < E;
    const int lk = is_link ? l : 0;
    const int sup = lane_const<E>(l, -1, [](int k) { return G::sup[k]; });
    const int supc = sup < 0 ? 0 : sup;
    const bool sfac = lane_const<E>(l, 0, [](int k) { return G::sup_is_factory[k]; }) != 0;
    const double Csp = lane_const<E>(l, 0.0, [](int k) { return G::C[G::sup[k] < 0 ? 0 : G::sup[k]]; });
    const double vsp = lane_const<E>(l, 1.0, [](int k) { return G::v[G::sup[k] < 0 ? 0 : G::sup[k]]; });
    const int Lk = lane_const<E>(l, 0, [](int k) { return G::L[k]; });
    const int roff = lane_const<E>(l, 0, [](int k) { return G::ring_off[k]; });
    const double lpk = lane_const<E>(l, 0.0, [](int k) { return G::lp[k]; });
    const double lgk = lane_const<E>(l, 0.0, [](int k) { return G::lg[k]; });
    const int rank = lane_const<E>(l, 0, [](int k) { return Q::sup_rank(k); });
    const int reccol = lane_const<E>(l, -1, [](int k) { return G::L[k] > 0 ? RL + J + LP::rank(k) : -1; });
    // node-lane constants
    const bool is_node = l < J;
    const double I0j = lane_const<J>(l, 0.0, [](int j) { return G::I0[j]; });
    const double hj = lane_const<J>(l, 0.0, [](int j) { return G::h[j]; });
    const double oj = lane_const<J>(l, 0.0, [](int j) { return G::o[j]; });
    const double vj = lane_const<J>(l, 1.0, [](int j) { return G::v[j]; });
    const bool facj = lane_const<J>(l, 0, [](int j) { return G::is_factory[j]; }) != 0;
    const bool retj = lane_const<J>(l, 0, [](int j) { return G::is_retail[j]; }) != 0;
    const int lastl = lane_const<J>(l, -1, [](int j) { return Q::last_link(j); });
    const int mkt = lane_const<J>(l, -1, [](int j) { return Q::market(j); });
    const int mk = mkt < 0 ? 0 : mkt;
    const double rlp = lane_const<RL>(mk, 0.0, [](int r) { return G::rl_p[r]; });
    const double rlb = lane_const<RL>(mk, 0.0, [](int r) { return G::rl_b[r]; });
    constexpr int PM = Q::pmax() > 0 ? Q::pmax() : 1, SM = Q::smax() > 0 ? Q::smax() : 1;
    const int npred = lane_const<J>(l, 0, [](int j) { return G::pred_ptr[j + 1] - G::pred_ptr[j]; });
    const int nsucc = lane_const<J>(l, 0, [](int j) { return G::succ_ptr[j + 1] - G::succ_ptr[j]; });
    int pidx[PM], sidx[PM > SM ? PM : SM], skind[SM];
#pragma unroll
    for (int x = 0; x < PM; x++)
        pidx[x] = lane_const<J>(l, 0, [x](int j) {
            return G::pred_ptr[j] + x < G::pred_ptr[j + 1] ? G::pred_idx[G::pred_ptr[j] + x] : 0;
        });
#pragma unroll
    for (int x = 0; x < SM; x++) {
        sidx[x] = lane_const<J>(l, 0, [x](int j) {
            return G::succ_ptr[j] + x < G::succ_ptr[j + 1] ? G::succ_idx[G::succ_ptr[j] + x] : 0;
        });
        skind[x] = lane_const<J>(l, 0, [x](int j) {
            return G::succ_ptr[j] + x < G::succ_ptr[j + 1] ? G::succ_kind[G::succ_ptr[j] + x] : 0;
        });
    }
    // state: X (node lanes), U (the node's market), Y (link lanes), order ring (link lanes, LDS)
    int t = t_start;
    double X = is_node ? P.X[(int64_t)l * S + el] : 0.0;
    double U = (is_node && mkt >= 0) ? P.U[(int64_t)mk * S + el] : 0.0;
    double Y = is_link ? P.Y[(int64_t)lk * S + el] : 0.0;
    double *rg = ring + q;                                   // [sumL][QE]
    for (int a = 0; a < (is_link ? Lk : 0); a++) rg[(roff + a) * QE] = P.Rring[(int64_t)(roff + a) * S + el];
    int pos = Lk > 0 ? (int)((uint32_t)t % (uint32_t)Lk) : 0;   // ring slot of R[t - L] / R[t]
    if (w == 2)
        for (int x = lane; x < P.T; x += WAVE) ap_l[x] = P.alpha_pow[x];   // before barrier 0
    // this chunk's actions (acur) and the next one's (anxt), link lanes
    float acur[CH], anxt[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) acur[i] = io.act[((int64_t)(i < K ? i : K - 1) * N + el) * E + lk];
    net_wg_sync();   // barrier 0: demand chunk 0 ready (and every ring row and alpha**t in LDS)
    for (int c = 0; c < nch; c++) {
        const double *db = dbuf + (c % RD) * CH * RL * WAVE;
        float *rb = rec + (c & 1) * CH * NR * WAVE;
#pragma unroll
        for (int i = 0; i < CH; i++) {
            const int kn = (c + 1) * CH + i;
            anxt[i] = io.act[((int64_t)(kn < K ? kn : K - 1) * N + el) * E + lk];
        }
#pragma unroll
        for (int kk = 0; kk < CH; kk++) {
            const int k = c * CH + kk;
            if (k >= K) break;
            const int64_t oi = (int64_t)k * N + e;
            const float act = acur[kk];
            const double apow = ap_l[t < P.T ? t : 0];
            if (t >= P.T) {                                   // NEXT_STEP autoreset (:301-332)
                X = I0j;
                U = 0.0;
                Y = 0.0;
                if (valid && l == J - 1) {
                    out_store(io.rew + oi, 0.0);
                    out_store(io.term + oi, (uint8_t)0);
                    out_store(io.trunc + oi, (uint8_t)0);
                }
                t = 0;
                pos = 0;
                continue;
            }
#ifdef INVSIM_ABL_Q_NO_DYN   // profiling ablation only (wrong results): the dynamics waves idle
            t += 1;
            continue;
#endif
            // 0) orders (:448-490): a clamp-scan over each supplier's consecutive link lanes.
            // Branch-free: every lane evaluates every round and keeps its own round's
            // result (selects), so the row gathers are not split by exec-mask branches
            const double Xs = row_get(X, rowbase, supc);      // the supplier's on-hand X[t]
            const double rq = rint((double)act);
            const double request = (rq > 0) ? rq : 0.0;
            double cons = 0.0, Rn = 0.0;
#pragma unroll
            for (int r = 0; r < Q::rmax(); r++) {
                const double cin = (r == 0) ? 0.0 : row_shr1(cons);
                const double oav = max0(Xs - cin);
                double avail = oav;
                const double mpi = vsp * oav;
                const double mp = (mpi < Csp) ? mpi : Csp;
                avail = (sfac && mp < avail) ? mp : avail;
                const double f = (avail < request) ? avail : request;
                const double cn = cin + f / vsp;
                const bool mine = rank == r;
                Rn = mine ? (sup < 0 ? request : f) : Rn;     // raw material: unlimited
                cons = (mine && sup >= 0) ? cn : cons;
            }
            Rn = is_link ? Rn : 0.0;
            // 1) pipeline (:494-511): arrival R[t - L] (age L) from the lane's ring, or R[t] when L == 0
            const int slot = (roff + pos) * QE;               // lanes with L == 0 touch their row 0 (unused)
            const double wa = rg[slot];
            const double arrv = (Lk == 0) ? Rn : ((t >= Lk) ? wa : 0.0);
            if (Lk > 0) rg[slot] = Rn;                        // R[t] replaces R[t - L] in the same slot
            pos = (pos + 1 >= Lk) ? 0 : pos + 1;
            Y = Y - arrv + Rn;
            const double lpR = lpk * Rn;                      // purchasing / sales term of the link
            const double lgY = lgk * max0(Y);                 // pipeline holding term of the link
            // every row gather of the node phase at once (all depend only on the link phase)
            double g_arr[PM], g_lpR[PM], g_lgY[PM], g_sR[SM], g_sP[SM];
#pragma unroll
            for (int x = 0; x < PM; x++) {
                g_arr[x] = row_get(arrv, rowbase, pidx[x]);
                g_lpR[x] = row_get(lpR, rowbase, pidx[x]);
                g_lgY[x] = row_get(lgY, rowbase, pidx[x]);
            }
#pragma unroll
            for (int x = 0; x < SM; x++) {
                g_sR[x] = row_get(Rn, rowbase, sidx[x]);
                g_sP[x] = row_get(lpR, rowbase, sidx[x]);
            }
            const double cj = row_get(cons, rowbase, lastl < 0 ? 0 : lastl);
            // arrivals in predecessor order (:516-523), X[t+1] (:528).  Masked terms add
            // +0.0, which leaves these sums unchanged: they start at +0.0 and so are never -0.0
            double acc = 0.0;
#pragma unroll
            for (int x = 0; x < PM; x++) acc += (x < npred) ? g_arr[x] : 0.0;
            X = (X + acc) - (lastl < 0 ? 0.0 : cj);
            // 2&3) market fulfilment (:536-566) on the market's node lane
            const bool has_m = mkt >= 0 && is_node;
            const double fill = db[(kk * RL + mk) * WAVE + q] + U;
            const double inv = max0(X);
            const double sale = (inv < fill) ? inv : fill;
            X = has_m ? X - sale : X;
            const double Sr = has_m ? sale : 0.0;
            U = has_m ? (P.backlog ? fill - sale : 0.0) : U;
            // 5) node profit (:578-613) in spec_core's sum orders
            double SR = 0.0, sold = 0.0;
#pragma unroll
            for (int x = 0; x < SM; x++) {
                const bool in = x < nsucc, re = skind[x] == 0;
                SR += in ? (re ? g_sP[x] : rlp * Sr) : 0.0;
                sold += in ? (re ? g_sR[x] : Sr) : 0.0;
            }
            double PC = 0.0, HCp = 0.0;
#pragma unroll
            for (int x = 0; x < PM; x++) PC += (x < npred) ? g_lpR[x] : 0.0;
            const double HC_on = hj * max0(X);
#pragma unroll
            for (int x = 0; x < PM; x++) HCp += (x < npred) ? g_lgY[x] : 0.0;
            const double HC = HC_on + HCp;
            const double OC = facj ? ((vj > 0) ? oj * (sold / vj) : 0.0) : 0.0;
            const double UP = (retj && mkt >= 0) ? 0.0 + rlb * U : 0.0;
            const double pj = is_node ? SR - PC - OC - HC - UP : 0.0;
            // total_profit_period: a sequential scan over the node lanes in node order
            double tot = 0.0 + pj;
#pragma unroll
            for (int j = 1; j < J; j++) {
                const double prev = row_shr1(tot);
                tot = (l == j) ? prev + pj : tot;
            }
            const double rw = apow * tot;                     // :619, on lane J - 1
            // the obs wave's record: U[t+1], X[t+1], R[t] of the links with L > 0
            if (is_node && mkt >= 0) rb[(kk * NR + mk) * WAVE + q] = (float)U;
            if (is_node) rb[(kk * NR + RL + l) * WAVE + q] = (float)X;
            if (reccol >= 0) rb[(kk * NR + reccol) * WAVE + q] = (float)Rn;
            if (valid && l == J - 1) {
                out_store(io.rew + oi, rw);
                out_store(io.term + oi, (uint8_t)0);
                out_store(io.trunc + oi, (uint8_t)(t + 1 >= P.T ? 1 : 0));
            }
            t += 1;
        }
#pragma unroll
        for (int i = 0; i < CH; i++) acur[i] = anxt[i];
        net_wg_sync();   // barrier c + 1: demand chunk c + 1 and record chunk c ready
    }
    if (valid) {
        if (is_node) st_store(P.X + (int64_t)l * S + e, X);
        if (is_node && mkt >= 0) st_store(P.U + (int64_t)mk * S + e, U);
        if (is_link) st_store(P.Y + (int64_t)lk * S + e, Y);
        // ring rows older than the episode are stored as zeros (the reference's zeroed history)
        for (int a = 1; a <= (is_link ? Lk : 0); a++) {
            const int row = roff + (int)((uint32_t)(t - a + 256 * Lk) % (uint32_t)Lk);
            const double v = rg[row * QE];
            st_store(P.Rring + (int64_t)row * S + e, (t - a >= 0) ? v : 0.0);
        }
    }
}

}  // namespace

template <class G>
static bool topo_eq(const invsim_netinvmgmt_spec &h) {
    if (h.n_main != G::J || h.n_reorder != G::E || h.n_retail != G::RL) return false;
    for (int j = 0; j < G::J; j++)
        if (h.I0[j] != G::I0[j] || h.h[j] != G::h[j] || h.C[j] != G::C[j] || h.o[j] != G::o[j] ||
            h.v[j] != G::v[j] || h.is_factory[j] != G::is_factory[j] || h.is_retail[j] != G::is_retail[j])
            return false;
    for (int k = 0; k < G::E; k++)
        if (h.sup[k] != G::sup[k] || h.pur[k] != G::pur[k] || h.sup_is_factory[k] != G::sup_is_factory[k] ||
            h.L[k] != G::L[k] || h.lp[k] != G::lp[k] || h.lg[k] != G::lg[k])
            return false;
    for (int r = 0; r < G::RL; r++)
        if (h.rl_node[r] != G::rl_node[r] || h.rl_p[r] != G::rl_p[r] || h.rl_b[r] != G::rl_b[r] ||
            h.rl_user[r] != 0)
            return false;
    for (int j = 0; j <= G::J; j++)
        if (h.succ_ptr[j] != G::succ_ptr[j] || h.pred_ptr[j] != G::pred_ptr[j]) return false;
    for (int q = 0; q < G::NSUCC; q++)
        if (h.succ_kind[q] != G::succ_kind[q] || h.succ_idx[q] != G::succ_idx[q]) return false;
    for (int q = 0; q < G::NPRED; q++)
        if (h.pred_idx[q] != G::pred_idx[q]) return false;
    return true;
}

int net_spec_match(const invsim_netinvmgmt_spec &h) {
    // the specialised kernels draw Poisson market demand only
    for (int r = 0; h.rl_dist && r < h.n_retail; r++)
        if (!h.rl_user[r] && h.rl_dist[r] != 1) return NET_SPEC_NONE;
    if (topo_eq<NetTopoDefault>(h)) return NET_SPEC_DEFAULT;
    if (topo_eq<NetTopoCustom>(h)) return NET_SPEC_CUSTOM;
    return NET_SPEC_NONE;
}

template <class G>
static size_t spec_lds_bytes() {
    return (size_t)((EPW * G::O + 3) / 4) * 4 * sizeof(float) + (size_t)G::RL * RHS_LDS_MAX * sizeof(double);
}

template <class G>
static hipError_t spec_launch(const NetParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                              bool &ahead, int &slot, hipStream_t s) {
    const size_t lds = spec_lds_bytes<G>();
    const dim3 grid((unsigned)((p.cm.N + EPW - 1) / EPW)), block(WAVE);
    PolicyIO none{};
    const PolicyIO &pv = pol ? *pol : none;
    // fast stream: the split step kernel with a demand-only lookahead, the
    // rollout kernels with counter-positioned draws, net_spec_kernel otherwise
    const bool ph = p.cm.philox != 0;
    if (p.ahead && p.cm.kn.net_ahead && !pol && io.K == 1 && t_u >= 0 && t_u < p.T && io.obs &&
        !(p.cm.autoreset == AR_SAME_STEP && t_u + 1 >= p.T)) {
        const bool hit = ahead;
        const int gla = hit ? (int)((p.cm.N + WAVE - 1) / WAVE) : 0;
        const dim3 grid2(grid.x + gla);
        if (p.cm.kn.net_split || ph) {
            const int gl2 = hit ? (int)((p.cm.N + 2 * WAVE - 1) / (2 * WAVE)) : 0;
            const dim3 g2(grid.x + gl2), b2(2 * WAVE);
            if (ph) {
                if (hit) hipLaunchKernelGGL((net_step2_kernel<G, true, PhiloxGen>), g2, b2, lds, s, p, t_u, io, slot, gl2);
                else hipLaunchKernelGGL((net_step2_kernel<G, false, PhiloxGen>), g2, b2, lds, s, p, t_u, io, slot, gl2);
            } else {
                if (hit) hipLaunchKernelGGL((net_step2_kernel<G, true>), g2, b2, lds, s, p, t_u, io, slot, gl2);
                else hipLaunchKernelGGL((net_step2_kernel<G, false>), g2, b2, lds, s, p, t_u, io, slot, gl2);
            }
        } else {
            if (hit) hipLaunchKernelGGL((net_step1_kernel<G, true>), grid2, block, lds, s, p, t_u, io, slot, gla);
            else hipLaunchKernelGGL((net_step1_kernel<G, false>), grid2, block, lds, s, p, t_u, io, slot, gla);
        }
        ahead = true;
        slot ^= 1;
        return hipGetLastError();
    }
    // the other kernels draw from cm.rng: commit the cache first (the lock-step
    // NEXT_STEP autoreset launch draws nothing and keeps it)
    if (ph) {
        ahead = false;   // the fast stream's cache (demands only) is for a counter value now passed
    } else if (ahead && !(!pol && io.K == 1 && t_u >= p.T)) {
        const hipError_t ce = net_commit_launch(p, slot, s);
        ahead = false;
        if (ce != hipSuccess) return ce;
    }
#define K_(TU, ONE, POL)                                                                                   \
    do {                                                                                                   \
        if (ph) hipLaunchKernelGGL((net_spec_kernel<G, TU, ONE, POL, PhiloxGen>), grid, block, lds, s, p, t_u, io, pv); \
        else hipLaunchKernelGGL((net_spec_kernel<G, TU, ONE, POL, Pcg>), grid, block, lds, s, p, t_u, io, pv);         \
    } while (0)
    // ... and the in-kernel ConstantOrder agent on the 3-role kernel
    const bool pol_roll = pol && pol->kind == POL_CONSTANT && p.cm.kn.net_pol_roll;
    if ((!pol || pol_roll) && io.K > 1 && t_u >= 0 && !p.cm.info_rec && p.cm.kn.net_roll &&
        (p.cm.autoreset == AR_NEXT_STEP || (p.cm.autoreset == AR_DISABLED && t_u + io.K <= p.T))) {
        const dim3 gr((unsigned)((p.cm.N + WAVE - 1) / WAVE));
        using R3 = NetRoll3<G, NET_ROLL3_CH>;
        // small batches, open loop: the profit on a fourth wave (one workgroup per CU)
        if (!pol && p.cm.N <= p.cm.kn.net_roll4_max_n && !p.cm.info_demand && p.T <= NetRoll4<G>::AP &&
            p.cm.N > p.cm.kn.net_rollq_max_n) {
            if (ph) hipLaunchKernelGGL((net_roll4_kernel<G, PhiloxGen>), gr, dim3(4 * WAVE), NetRoll4<G>::lds(), s, p, t_u, io);
            else hipLaunchKernelGGL((net_roll4_kernel<G, Pcg>), gr, dim3(4 * WAVE), NetRoll4<G>::lds(), s, p, t_u, io);
            return hipGetLastError();
        }
        // small shards, open loop: the edge work of an env spread over a 16-lane row
        if (!pol && p.cm.N <= p.cm.kn.net_rollq_max_n && !p.cm.info_demand && p.T <= NetQ<G>::AP) {
            const dim3 gq((unsigned)((p.cm.N + NetQ<G>::QE - 1) / NetQ<G>::QE));
            if (ph) hipLaunchKernelGGL((net_rollq_kernel<G, PhiloxGen>), gq, dim3(6 * WAVE), NetQ<G>::lds(), s, p, t_u, io);
            else hipLaunchKernelGGL((net_rollq_kernel<G, Pcg>), gq, dim3(6 * WAVE), NetQ<G>::lds(), s, p, t_u, io);
            return hipGetLastError();
        }
        // the 3-role net_roll3o_kernel by default (measured on MI355X, 30-step
        // launches: 32 768 envs 69 vs 97 us, 65 536 envs 140 vs 185 us against
        // net_roll_kernel)
#define RK_(RG)                                                                                                       \
    do {                                                                                                              \
        if (pol) hipLaunchKernelGGL((net_roll3o_kernel<G, NET_ROLL3_CH, true, RG>), gr, dim3(3 * WAVE), R3::lds(), s, p, t_u, io, pv); \
        else if (p.cm.kn.net_roll3) hipLaunchKernelGGL((net_roll3o_kernel<G, NET_ROLL3_CH, false, RG>), gr, dim3(3 * WAVE), R3::lds(), s, p, t_u, io, pv); \
        else hipLaunchKernelGGL((net_roll_kernel<G, RG>), gr, dim3(2 * WAVE), NetRoll<G>::lds(), s, p, t_u, io);    \
    } while (0)
        if (ph) RK_(PhiloxGen);
        else RK_(Pcg);
#undef RK_
        return hipGetLastError();
    }
    if (pol) {
        if (t_u >= 0) K_(true, false, true);
        else K_(false, false, true);
    } else if (io.K == 1) {
        if (t_u >= 0) K_(true, true, false);
        else K_(false, true, false);
    } else {
        if (t_u >= 0) K_(true, false, false);
        else K_(false, false, false);
    }
#undef K_
    return hipGetLastError();
}

hipError_t net_commit_launch(const NetParams &p, int slot, hipStream_t s) {
    if (p.cm.N == 0 || !p.ahead) return hipSuccess;
    hipLaunchKernelGGL(net_commit_kernel, dim3((unsigned)((p.cm.N + 255) / 256)), dim3(256), 0, s, p, slot ^ 1,
                       2 + p.RL);
    return hipGetLastError();
}

hipError_t net_spec_launch(int which, const NetParams &p, int t_u, const PolicyIO *pol,
                           const StepIO<float, float> &io, bool &ahead, int &slot, hipStream_t s) {
    if (p.cm.N == 0 || io.K <= 0) return hipSuccess;
    switch (which) {
        case NET_SPEC_DEFAULT: return spec_launch<NetTopoDefault>(p, t_u, pol, io, ahead, slot, s);
        case NET_SPEC_CUSTOM: return spec_launch<NetTopoCustom>(p, t_u, pol, io, ahead, slot, s);
        default: return hipErrorInvalidValue;
    }
}

INVSIM_PTRS_STATS_TU(netspec)

}  // namespace invsim
