// NetInvMgmtMasterEnv.step / reset (network_management.py:301-635) as a
// topology-interpreting HIP kernel for gfx950: one thread per env, the graph
// compiled by the host into index tables that every lane walks in lock-step
// (all indices are wave-uniform, so table reads are scalar loads and the
// per-env node/link scratch lives in LDS at [row][lane] — bank-conflict free).
//
// Per-env HBM state (SoA rows of Npad, f64 like the reference DataFrames):
//   X[J] on-hand inventory, U[RL] unfulfilled market demand, Y[E] pipeline,
//   Rring[sum L] fulfilled orders per link (slot t mod L_e = R[t-L_e], the
//   delivery arriving this period; the same ring is the obs window), period, PCG64.
#include "kernels.hpp"

namespace invsim {
namespace {

constexpr int NET_BS = 64;  // one wave per workgroup; LDS scratch per lane

__device__ __forceinline__ double max0(double x) { return (x > 0) ? x : 0.0; }  // max(0, x)

// reset (:301-332): X = I0, U = Y = 0, period 0; obs = [0(RL), I0(J), 0(sumL)]
__device__ __forceinline__ void net_reset_one(const NetParams &P, int64_t e, float *orow) {
    const int64_t S = P.cm.Npad;
    for (int j = 0; j < P.J; j++) P.X[j * S + e] = P.I0[j];
    for (int r = 0; r < P.RL; r++) P.U[r * S + e] = 0.0;
    for (int k = 0; k < P.E; k++) P.Y[k * S + e] = 0.0;
    P.cm.period[e] = 0;
    if (orow) {
        int o = 0;
        for (int r = 0; r < P.RL; r++) orow[o++] = 0.f;
        for (int j = 0; j < P.J; j++) orow[o++] = (float)P.I0[j];
        for (int q = 0; q < P.sumL; q++) orow[o++] = 0.f;
    }
}

// One step (:436-635) for env e at period t < T.  lds = this lane's scratch base.
__device__ bool net_step_one(const NetParams &P, int64_t e, Pcg &g, const float *__restrict__ arow,
                             float *orow, double &reward, int64_t *dem, double *lds) {
    const int64_t S = P.cm.Npad;
    const int J = P.J, E = P.E, RL = P.RL;
    const int t = P.cm.period[e];
    // LDS rows: Xs[J] cons[J] arr[J] Rn[E] arrv[E] Yn[E] Sr[RL] Un[RL]
    double *Xs = lds, *cons = Xs + J * NET_BS, *arr = cons + J * NET_BS, *Rn = arr + J * NET_BS;
    double *arrv = Rn + E * NET_BS, *Yn = arrv + E * NET_BS, *Sr = Yn + E * NET_BS,
           *Un = Sr + RL * NET_BS;
#define LV(a, i) a[(i) * NET_BS]
    for (int j = 0; j < J; j++) {
        LV(Xs, j) = P.X[j * S + e];
        LV(cons, j) = 0.0;
        LV(arr, j) = 0.0;
    }
    // 0) orders over sorted reorder links (:448-490)
    for (int k = 0; k < E; k++) {
        const double rq = rint((double)arow[k]);          // round() half-to-even
        const double request = (rq > 0) ? rq : 0.0;        // max(0, .)
        const int s = P.sup[k];
        double f;
        if (s < 0) {
            f = request;                                   // raw material: unlimited
        } else {
            const double oav = max0(LV(Xs, s) - LV(cons, s));
            double avail = oav;
            if (P.sup_is_factory[k]) {
                const double mpi = P.v[s] * oav;
                const double mp = (mpi < P.C[s]) ? mpi : P.C[s];   // min(C, v*avail)
                avail = (mp < avail) ? mp : avail;
            }
            f = (avail < request) ? avail : request;       // min(request, avail)
            LV(cons, s) += f / P.v[s];
        }
        LV(Rn, k) = f;
    }
    // 1) pipeline Y[t+1] = Y[t] - R[t-L] + R[t] (:494-511); ring slot t mod L <- R[t]
    for (int k = 0; k < E; k++) {
        const int L = P.L[k];
        double a = 0.0;
        if (L == 0) {
            a = LV(Rn, k);
        } else {
            const int64_t row = P.ring_off[k] + (int)((uint32_t)t % (uint32_t)L);
            if (t >= L) a = P.Rring[row * S + e];
            P.Rring[row * S + e] = LV(Rn, k);
        }
        LV(arrv, k) = a;
        const double y = P.Y[k * S + e] - a + LV(Rn, k);
        LV(Yn, k) = y;
        P.Y[k * S + e] = y;
    }
    // arrivals in predecessor adjacency order (:516-523); X[t+1] (:528)
    for (int j = 0; j < J; j++) {
        double acc = 0.0;
        for (int q = P.pred_ptr[j]; q < P.pred_ptr[j + 1]; q++) acc += LV(arrv, P.pred_idx[q]);
        LV(Xs, j) = (LV(Xs, j) + acc) - LV(cons, j);
    }
    // 2&3) market demand and fulfilment in retail-link edge order (:536-566)
    for (int r = 0; r < RL; r++) {
        double dd;
        if (P.rl_user[r]) {
            const int idx = t < P.T - 1 ? t : P.T - 1;
            dd = rint(P.user_D[(int64_t)r * P.T + idx]);
            if (!(dd > 0)) dd = 0.0;
        } else {
            const int64_t pd = np_poisson(g, P.rl_pc[r]);
            dd = (double)(pd > 0 ? pd : 0);
        }
        if (dem) dem[e * RL + r] = (int64_t)dd;
        const double fill = dd + P.U[r * S + e];
        const int node = P.rl_node[r];
        const double inv = max0(LV(Xs, node));
        const double sale = (inv < fill) ? inv : fill;     // min(fill, inv)
        LV(Xs, node) -= sale;
        LV(Sr, r) = sale;
        const double un = P.backlog ? fill - sale : 0.0;
        LV(Un, r) = un;
        P.U[r * S + e] = un;
    }
    // 5) profit per main node (:578-613)
    double total = 0.0;
    for (int j = 0; j < J; j++) {
        double SR = 0.0, sold = 0.0;
        for (int q = P.succ_ptr[j]; q < P.succ_ptr[j + 1]; q++) {
            const int idx = P.succ_idx[q];
            const bool re = P.succ_kind[q] == 0;
            const double sv = re ? LV(Rn, idx) : LV(Sr, idx);
            SR += (re ? P.lp[idx] : P.rl_p[idx]) * sv;
            sold += sv;
        }
        double PC = 0.0, HCp = 0.0;
        for (int q = P.pred_ptr[j]; q < P.pred_ptr[j + 1]; q++) PC += P.lp[P.pred_idx[q]] * LV(Rn, P.pred_idx[q]);
        const double xj = LV(Xs, j);
        const double HC_on = P.h[j] * max0(xj);
        for (int q = P.pred_ptr[j]; q < P.pred_ptr[j + 1]; q++) HCp += P.lg[P.pred_idx[q]] * max0(LV(Yn, P.pred_idx[q]));
        const double HC = HC_on + HCp;
        double OC = 0.0;
        if (P.is_factory[j]) OC = (P.v[j] > 0) ? P.o[j] * (sold / P.v[j]) : 0.0;
        double UP = 0.0;
        if (P.is_retail[j])
            for (int q = P.succ_ptr[j]; q < P.succ_ptr[j + 1]; q++)
                if (P.succ_kind[q] == 1) UP += P.rl_b[P.succ_idx[q]] * LV(Un, P.succ_idx[q]);
        total += SR - PC - OC - HC - UP;
        P.X[j * S + e] = xj;
    }
    reward = P.alpha_pow[t] * total;                        // :619
    const int t1 = t + 1;
    P.cm.period[e] = t1;
    // obs (:334-413): U[t+1] (RL), X[t+1] (J), for each link with L>0 in sorted
    // order the fulfilled orders R[t+1-L .. t] right-aligned, zeros before t=0
    if (orow) {
        int o = 0;
        for (int r = 0; r < RL; r++) orow[o++] = (float)LV(Un, r);
        for (int j = 0; j < J; j++) orow[o++] = (float)LV(Xs, j);
        for (int k = 0; k < E; k++) {
            const int L = P.L[k];
            if (L == 0) continue;
            for (int p = 0; p < L - 1; p++) {
                const int age = L - 1 - p;                  // R[t - age]
                double v = 0.0;
                if (t - age >= 0) {
                    const int64_t row = P.ring_off[k] + (int)((uint32_t)(t - age) % (uint32_t)L);
                    v = P.Rring[row * S + e];
                }
                orow[o++] = (float)v;
            }
            orow[o++] = (float)LV(Rn, k);
        }
    }
#undef LV
    return t1 >= P.T;
}

__device__ __forceinline__ double *lane_scratch() {
    extern __shared__ __attribute__((aligned(16))) double net_lds[];
    return net_lds + threadIdx.x;
}

__global__ void __launch_bounds__(NET_BS)
net_step_kernel(NetParams P, const float *__restrict__ act, float *__restrict__ obs,
                double *__restrict__ rew, uint8_t *__restrict__ term, uint8_t *__restrict__ trunc,
                float *__restrict__ fobs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int O = P.RL + P.J + P.sumL;
    float *orow = obs + e * O;
    const int t = P.cm.period[e];
    if (t >= P.T) {
        if (P.cm.autoreset == AR_NEXT_STEP) {
            net_reset_one(P, e, orow);
            rew[e] = 0.0;
            term[e] = 0;
            trunc[e] = 0;
        } else {
            atomicOr(P.cm.status, 1u);
        }
        return;
    }
    Pcg g = P.cm.rng.load(e);
    double r;
    const bool tr = net_step_one(P, e, g, act + e * P.E, orow, r, P.cm.info_demand, lane_scratch());
    rew[e] = r;
    term[e] = 0;
    trunc[e] = tr ? 1 : 0;
    if (tr && P.cm.autoreset == AR_SAME_STEP) {
        if (fobs)
            for (int j = 0; j < O; j++) fobs[e * O + j] = orow[j];
        net_reset_one(P, e, orow);
    }
    P.cm.rng.store_state(e, g);
}

__global__ void __launch_bounds__(NET_BS)
net_rollout_kernel(NetParams P, int K, const float *__restrict__ act, float *__restrict__ obs,
                   double *__restrict__ rew, uint8_t *__restrict__ term,
                   uint8_t *__restrict__ trunc) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int64_t N = P.cm.N;
    const int O = P.RL + P.J + P.sumL;
    Pcg g = P.cm.rng.load(e);
    for (int k = 0; k < K; k++) {
        const int64_t oi = (int64_t)k * N + e;
        float *orow = obs + oi * O;
        const int t = P.cm.period[e];
        if (t >= P.T) {
            if (P.cm.autoreset == AR_NEXT_STEP) {
                net_reset_one(P, e, orow);
                rew[oi] = 0.0;
                term[oi] = 0;
                trunc[oi] = 0;
                continue;
            }
            atomicOr(P.cm.status, 1u);
            break;
        }
        double r;
        const bool tr = net_step_one(P, e, g, act + oi * P.E, orow, r,
                                     k == K - 1 ? P.cm.info_demand : nullptr, lane_scratch());
        rew[oi] = r;
        term[oi] = 0;
        trunc[oi] = tr ? 1 : 0;
        if (tr && P.cm.autoreset == AR_SAME_STEP) net_reset_one(P, e, orow);
    }
    P.cm.rng.store_state(e, g);
}

__global__ void __launch_bounds__(256)
net_reset_kernel(NetParams P, const uint8_t *__restrict__ mask, float *__restrict__ obs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    if (mask && !mask[e]) return;
    net_reset_one(P, e, obs ? obs + e * (P.RL + P.J + P.sumL) : nullptr);
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }
inline size_t lds_bytes(const NetParams &p) {
    return (size_t)(3 * p.J + 3 * p.E + 2 * p.RL) * NET_BS * sizeof(double);
}

}  // namespace

hipError_t net_step_launch(const NetParams &p, const float *act, float *obs, double *rew,
                           uint8_t *term, uint8_t *trunc, float *fobs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(net_step_kernel, dim3(grid_for(p.cm.N, NET_BS)), dim3(NET_BS), lds_bytes(p),
                       s, p, act, obs, rew, term, trunc, fobs);
    return hipGetLastError();
}

hipError_t net_rollout_launch(const NetParams &p, int K, const float *act, float *obs,
                              double *rew, uint8_t *term, uint8_t *trunc, hipStream_t s) {
    if (p.cm.N == 0 || K <= 0) return hipSuccess;
    hipLaunchKernelGGL(net_rollout_kernel, dim3(grid_for(p.cm.N, NET_BS)), dim3(NET_BS),
                       lds_bytes(p), s, p, K, act, obs, rew, term, trunc);
    return hipGetLastError();
}

hipError_t net_reset_launch(const NetParams &p, const uint8_t *mask, float *obs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(net_reset_kernel, dim3(grid_for(p.cm.N, 256)), dim3(256), 0, s, p, mask, obs);
    return hipGetLastError();
}

}  // namespace invsim
