// NetInvMgmtMasterEnv.step / reset (network_management.py:301-635) as a
// topology-interpreting HIP kernel for gfx950: one thread per env, one wave
// per workgroup, the graph compiled by the host into index tables that every
// lane walks in lock-step (indices are wave-uniform: table reads are scalar
// loads).  Per-env node/link values live in LDS at [row][lane] (conflict-free)
// for the whole launch, so K steps touch HBM state once.
//
// Per-env HBM state (SoA rows of Npad, f64 like the reference DataFrames):
//   X[J] on-hand inventory, U[RL] unfulfilled market demand, Y[E] pipeline,
//   Rring[sum L] fulfilled orders per link (slot t mod L_e = R[t-L_e], the
//   delivery arriving this period; the same ring is the obs window),
//   period (only when not lock-step), PCG64.
#include "kernels.hpp"

namespace invsim {
namespace {

__device__ __forceinline__ double max0(double x) { return (x > 0) ? x : 0.0; }  // max(0, x)

struct NetScratch {
    double *X, *U, *Y;                     // persistent across the launch
    double *cons, *arr, *Rn, *arrv, *Sr, *Dd;  // per step
};

__device__ __forceinline__ NetScratch scratch_of(const NetParams &P, double *base) {
    NetScratch s;
    const int J = P.J, E = P.E, RL = P.RL;
    s.X = base;
    s.U = s.X + J * WAVE;
    s.Y = s.U + RL * WAVE;
    s.cons = s.Y + E * WAVE;
    s.arr = s.cons + J * WAVE;
    s.Rn = s.arr + J * WAVE;
    s.arrv = s.Rn + E * WAVE;
    s.Sr = s.arrv + E * WAVE;
    s.Dd = s.Sr + RL * WAVE;
    return s;
}
__host__ __device__ inline int scratch_rows(int J, int E, int RL) { return 3 * J + 3 * E + 3 * RL; }

#define LV(a, i) (a)[(i) * WAVE]

// reset (:301-332): X = I0, U = Y = 0; obs = [0(RL), I0(J), 0(sumL)]
__device__ __forceinline__ void net_reset_lds(const NetParams &P, NetScratch &s, float *orow) {
    for (int j = 0; j < P.J; j++) LV(s.X, j) = P.I0[j];
    for (int r = 0; r < P.RL; r++) LV(s.U, r) = 0.0;
    for (int k = 0; k < P.E; k++) LV(s.Y, k) = 0.0;
    if (orow) {
        int o = 0;
        for (int r = 0; r < P.RL; r++) orow[o++] = 0.f;
        for (int j = 0; j < P.J; j++) orow[o++] = (float)P.I0[j];
        for (int q = 0; q < P.sumL; q++) orow[o++] = 0.f;
    }
}

// One step (:436-635) at period t < T.  Returns truncated.
// All LPE lanes of the env run it (redundant node/link arithmetic in private
// LDS scratch, lane-group Poisson draws); lane j == 0 writes state and the
// U/X part of the obs row, lane j writes the order windows of links k = j mod LPE.
template <class RG>
__device__ bool net_step_lds(const NetParams &P, int64_t e, int gl, int t, RG &g, uint64_t &u32, NetScratch &s,
                             const float *__restrict__ arow, float *orow, double &reward, int64_t *dem,
                             double *irec) {
    const int64_t S = P.cm.Npad;
    const int J = P.J, E = P.E, RL = P.RL;
    const bool leader = gl == 0;
    // market demand draws first (retail-link order, :536-541): RNG-only work
    for (int r = 0; r < RL; r++) {
        double dd;
        if (P.rl_user[r]) {
            const int idx = t < P.T - 1 ? t : P.T - 1;
            dd = rint(P.user_D[(int64_t)r * P.T + idx]);       // max(0, int(round(x)))
            if (!(dd > 0)) dd = 0.0;
        } else {
            const PtrsConst &pc = P.rl_pc[r];
            g.sub((uint32_t)r);                                // fast stream: market r's counter block
            const int dk = P.rl_dist ? P.rl_dist[r] : 1;       // the edge's numpy method (:257-263)
            const int64_t pd = dk == 1 ? env_poisson(g, pc, P.rhs ? P.rhs + pc.toff : nullptr)
                                       : np_demand(g, u32, P.rl_nd[r]);
            dd = (double)(pd > 0 ? pd : 0);
        }
        LV(s.Dd, r) = dd;
        if (dem && leader) dem[e * RL + r] = (int64_t)dd;
    }
    for (int j = 0; j < J; j++) {
        LV(s.cons, j) = 0.0;
        LV(s.arr, j) = 0.0;
    }
    // 0) orders over sorted reorder links (:448-490)
    for (int k = 0; k < E; k++) {
        const double rq = rint((double)arow[k]);           // round() half-to-even
        const double request = (rq > 0) ? rq : 0.0;        // max(0, .)
        const int sp = P.sup[k];
        double f;
        if (sp < 0) {
            f = request;                                   // raw material: unlimited
        } else {
            const double oav = max0(LV(s.X, sp) - LV(s.cons, sp));
            double avail = oav;
            if (P.sup_is_factory[k]) {
                const double mpi = P.v[sp] * oav;
                const double mp = (mpi < P.C[sp]) ? mpi : P.C[sp];   // min(C, v*avail)
                avail = (mp < avail) ? mp : avail;
            }
            f = (avail < request) ? avail : request;       // min(request, avail)
            LV(s.cons, sp) += f / P.v[sp];
        }
        LV(s.Rn, k) = f;
    }
    // 1) pipeline Y[t+1] = Y[t] - R[t-L] + R[t] (:494-511); ring slot t mod L <- R[t]
    for (int k = 0; k < E; k++) {
        const int L = P.L[k];
        double a = 0.0;
        if (L == 0) {
            a = LV(s.Rn, k);
        } else {
            const int64_t row = P.ring_off[k] + (int)((uint32_t)t % (uint32_t)L);
            if (t >= L) a = P.Rring[row * S + e];
            if (leader) P.Rring[row * S + e] = LV(s.Rn, k);
        }
        LV(s.arrv, k) = a;
        LV(s.Y, k) = LV(s.Y, k) - a + LV(s.Rn, k);
    }
    // arrivals in predecessor adjacency order (:516-523); X[t+1] (:528)
    for (int j = 0; j < J; j++) {
        double acc = 0.0;
        for (int q = P.pred_ptr[j]; q < P.pred_ptr[j + 1]; q++) acc += LV(s.arrv, P.pred_idx[q]);
        LV(s.X, j) = (LV(s.X, j) + acc) - LV(s.cons, j);
    }
    // 2&3) market fulfilment in retail-link edge order (:536-566)
    for (int r = 0; r < RL; r++) {
        const double fill = LV(s.Dd, r) + LV(s.U, r);
        const int node = P.rl_node[r];
        const double inv = max0(LV(s.X, node));
        const double sale = (inv < fill) ? inv : fill;     // min(fill, inv)
        LV(s.X, node) -= sale;
        LV(s.Sr, r) = sale;
        LV(s.U, r) = P.backlog ? fill - sale : 0.0;
    }
    double *rr = (irec && leader) ? irec + e * (2 * RL + 2 * J + 2 * E) : nullptr;
    if (rr) {  // step record: S[t, retail], U[t+1, retail], X[t+1], R[t], Y[t+1] (P[t] below)
        for (int r = 0; r < RL; r++) {
            rr[r] = LV(s.Sr, r);
            rr[RL + r] = LV(s.U, r);
        }
        for (int j = 0; j < J; j++) rr[2 * RL + j] = LV(s.X, j);
        for (int k = 0; k < E; k++) {
            rr[2 * RL + J + k] = LV(s.Rn, k);
            rr[2 * RL + J + E + k] = LV(s.Y, k);
        }
    }
    // 5) profit per main node (:578-613), Python sum() order = adjacency order
    double total = 0.0;
    for (int j = 0; j < J; j++) {
        double SR = 0.0, sold = 0.0;
        for (int q = P.succ_ptr[j]; q < P.succ_ptr[j + 1]; q++) {
            const int idx = P.succ_idx[q];
            const bool re = P.succ_kind[q] == 0;
            const double sv = re ? LV(s.Rn, idx) : LV(s.Sr, idx);
            SR += (re ? P.lp[idx] : P.rl_p[idx]) * sv;
            sold += sv;
        }
        double PC = 0.0, HCp = 0.0;
        for (int q = P.pred_ptr[j]; q < P.pred_ptr[j + 1]; q++) PC += P.lp[P.pred_idx[q]] * LV(s.Rn, P.pred_idx[q]);
        const double HC_on = P.h[j] * max0(LV(s.X, j));
        for (int q = P.pred_ptr[j]; q < P.pred_ptr[j + 1]; q++)
            HCp += P.lg[P.pred_idx[q]] * max0(LV(s.Y, P.pred_idx[q]));
        const double HC = HC_on + HCp;
        double OC = 0.0;
        if (P.is_factory[j]) OC = (P.v[j] > 0) ? P.o[j] * (sold / P.v[j]) : 0.0;
        double UP = 0.0;
        if (P.is_retail[j])
            for (int q = P.succ_ptr[j]; q < P.succ_ptr[j + 1]; q++)
                if (P.succ_kind[q] == 1) UP += P.rl_b[P.succ_idx[q]] * LV(s.U, P.succ_idx[q]);
        const double pj = SR - PC - OC - HC - UP;
        if (rr) rr[2 * RL + J + 2 * E + j] = pj;                // P[t, node]
        total += pj;
    }
    reward = P.alpha_pow[t] * total;                        // :619
    // obs (:334-413): U[t+1] (RL), X[t+1] (J), then for each link with L>0 in
    // sorted order the fulfilled orders R[t+1-L .. t] right-aligned, zero before t=0
    if (orow) {
        if (leader) {
            int o = 0;
            for (int r = 0; r < RL; r++) orow[o++] = (float)LV(s.U, r);
            for (int q = 0; q < J; q++) orow[o++] = (float)LV(s.X, q);
        }
        for (int k = gl; k < E; k += LPE) {
            const int L = P.L[k];
            if (L == 0) continue;
            float *w = orow + P.win_off[k];
            for (int p = 0; p < L - 1; p++) {
                const int age = L - 1 - p;                  // R[t - age]
                double v = 0.0;
                if (t - age >= 0) {
                    const int64_t row = P.ring_off[k] + (int)((uint32_t)(t - age) % (uint32_t)L);
                    v = P.Rring[row * S + e];
                }
                w[p] = (float)v;
            }
            w[L - 1] = (float)LV(s.Rn, k);
        }
    }
    return t + 1 >= P.T;
}

// POL: closed-loop rollout (invsim_rollout_policy) with the CONSTANT agent
// (ConstantOrderAgent, benchmark_NetInvMgmtBacklogEnv.py:119-135) on any graph:
// every output optional, evaluate_agent metrics (as net_spec_kernel) summed
// into pol.metrics in place.
template <bool TU, bool POL, class RG>
__global__ void __launch_bounds__(WAVE)
net_run_kernel(NetParams P, int t_u, StepIO<float, float> io, PolicyIO pol) {
    extern __shared__ __attribute__((aligned(16))) double net_lds[];
    const int lane = threadIdx.x;
    const int gl = lane & (LPE - 1);
    const bool leader = gl == 0;
    const int64_t e0 = (int64_t)blockIdx.x * EPW;
    const int64_t e = e0 + lane / LPE;
    const int64_t N = P.cm.N;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < EPW ? (N - e0) : EPW);
    const int O = P.RL + P.J + P.sumL;
    const int64_t S = P.cm.Npad;
    const int rows = scratch_rows(P.J, P.E, P.RL);
    NetScratch s = scratch_of(P, net_lds + lane);   // private scratch per lane
    float *tile = reinterpret_cast<float *>(net_lds + (int64_t)rows * WAVE);
    float *trow = tile + (int64_t)(lane / LPE) * O;

    RG g;
    uint64_t u32 = 0;         // numpy's buffered 32-bit half (integers markets)
    int t = t_u;
    if (valid) {
        P.cm.rng.load(e, g);
        if (P.cm.u32buf && !RG::kCounter) u32 = P.cm.u32buf[e];
        for (int j = 0; j < P.J; j++) LV(s.X, j) = P.X[j * S + e];
        for (int r = 0; r < P.RL; r++) LV(s.U, r) = P.U[r * S + e];
        for (int k = 0; k < P.E; k++) LV(s.Y, k) = P.Y[k * S + e];
        if (!TU) t = P.cm.period[e];
    }
    bool fault = false;
    for (int k = 0; k < io.K; k++) {
        const int64_t oi = (int64_t)k * N + e;
        bool tr = false;
        g.set_step(P.cm.ph_step + (uint64_t)k);
        if (valid) {
            if (t >= P.T) {
                if (P.cm.autoreset == AR_NEXT_STEP) {
                    net_reset_lds(P, s, leader ? trow : nullptr);
                    if (leader && (!POL || io.rew)) {
                        io.rew[oi] = 0.0;
                        io.term[oi] = 0;
                        io.trunc[oi] = 0;
                    }
                    t = 0;
                } else {
                    fault = true;
                }
            } else {
                double r;
                if (RG::kCounter) u32 = 0;          // fast stream: no half carried between steps
                tr = net_step_lds(P, e, gl, t, g, u32, s, POL ? pol.cf : io.act + oi * P.E, trow, r,
                                  k == io.K - 1 ? P.cm.info_demand : nullptr,
                                  k == io.K - 1 ? (double *)P.cm.info_rec : nullptr);
                if (leader && (!POL || io.rew)) {
                    io.rew[oi] = r;
                    io.term[oi] = 0;
                    io.trunc[oi] = tr ? 1 : 0;
                }
                if (POL && leader) {
                    if (pol.act_out)
                        for (int q = 0; q < P.E; q++) ((float *)pol.act_out)[oi * P.E + q] = pol.cf[q];
                    if (pol.metrics) {   // evaluate_agent metrics (benchmark_NetInvMgmtLostSalesEnv.py:264-300)
                        double *met = pol.metrics + e * (5 + P.J);
                        met[0] += r;                                   // episode_reward
                        met[1] += 1.0;
                        double m2 = met[2], m3 = met[3], m4 = met[4];
                        for (int q = 0; q < P.RL; q++) {
                            m2 += LV(s.Dd, q);                         // D[t, retail links]
                            m3 += LV(s.Sr, q);                         // S[t, retail links]
                            m4 += LV(s.U, q);                          // U[t+1, retail links]
                        }
                        met[2] = m2;
                        met[3] = m3;
                        met[4] = m4;
                        for (int j = 0; j < P.J; j++) met[5 + j] += LV(s.X, j);   // X[t+1] per node
                    }
                }
                t += 1;
            }
        }
        __syncthreads();
        if (P.cm.autoreset == AR_SAME_STEP) {        // final obs out, then the reset obs in
            if (valid && tr && io.fobs)
                for (int q = gl; q < O; q += LPE) io.fobs[e * O + q] = trow[q];
            __syncthreads();
            if (valid && tr) {
                net_reset_lds(P, s, leader ? trow : nullptr);
                t = 0;
            }
            __syncthreads();
        }
        if (!POL || io.obs) store_tile(tile, io.obs + ((int64_t)k * N + e0) * O, (int64_t)nvalid * O, lane);
        __syncthreads();
    }
    if (valid && leader) {
        P.cm.rng.store_state(e, g);
        if (P.cm.u32buf && !RG::kCounter) P.cm.u32buf[e] = u32;
        for (int j = 0; j < P.J; j++) P.X[j * S + e] = LV(s.X, j);
        for (int r = 0; r < P.RL; r++) P.U[r * S + e] = LV(s.U, r);
        for (int k = 0; k < P.E; k++) P.Y[k * S + e] = LV(s.Y, k);
        if (!TU) P.cm.period[e] = t;
        if (fault) atomicOr(P.cm.status, 1u);
    }
}

__global__ void __launch_bounds__(256)
net_reset_kernel(NetParams P, const uint8_t *__restrict__ mask, float *__restrict__ obs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    if (mask && !mask[e]) return;
    const int64_t S = P.cm.Npad;
    for (int j = 0; j < P.J; j++) P.X[j * S + e] = P.I0[j];
    for (int r = 0; r < P.RL; r++) P.U[r * S + e] = 0.0;
    for (int k = 0; k < P.E; k++) P.Y[k * S + e] = 0.0;
    P.cm.period[e] = 0;
    if (obs) {
        float *orow = obs + e * (P.RL + P.J + P.sumL);
        int o = 0;
        for (int r = 0; r < P.RL; r++) orow[o++] = 0.f;
        for (int j = 0; j < P.J; j++) orow[o++] = (float)P.I0[j];
        for (int q = 0; q < P.sumL; q++) orow[o++] = 0.f;
    }
}

#undef LV

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

size_t net_lds_bytes(const NetParams &p) {
    const size_t tile = (size_t)EPW * (p.RL + p.J + p.sumL) * sizeof(float);
    return (size_t)scratch_rows(p.J, p.E, p.RL) * WAVE * sizeof(double) + (tile + 15) / 16 * 16;
}

hipError_t net_run_launch(const NetParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                          hipStream_t s) {
    if (p.cm.N == 0 || io.K <= 0) return hipSuccess;
    const size_t lds = net_lds_bytes(p);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const dim3 grid(grid_for(p.cm.N, EPW)), block(WAVE);
    PolicyIO none{};
    const PolicyIO &pv = pol ? *pol : none;
    if (pol && pol->kind != POL_CONSTANT) return hipErrorInvalidValue;
#define K_(TU, POL)                                                                                    \
    do {                                                                                               \
        if (p.cm.philox) hipLaunchKernelGGL((net_run_kernel<TU, POL, PhiloxGen>), grid, block, lds, s, p, t_u, io, pv); \
        else hipLaunchKernelGGL((net_run_kernel<TU, POL, Pcg>), grid, block, lds, s, p, t_u, io, pv);         \
    } while (0)
    if (t_u >= 0) {
        if (pol) K_(true, true);
        else K_(true, false);
    } else {
        if (pol) K_(false, true);
        else K_(false, false);
    }
#undef K_
    return hipGetLastError();
}

hipError_t net_reset_launch(const NetParams &p, const uint8_t *mask, float *obs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(net_reset_kernel, dim3(grid_for(p.cm.N, 256)), dim3(256), 0, s, p, mask, obs);
    return hipGetLastError();
}

INVSIM_PTRS_STATS_TU(net)

}  // namespace invsim
