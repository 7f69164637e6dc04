// NewsvendorEnv.step / reset (newsvendor.py:100-204) as one-thread-per-env HIP
// kernels for gfx950.
//
// Per-env state (SoA rows of Npad): params price,cost,h,k,mu (f64, they are
// Python floats in the reference), the order pipeline as a ring of L f32 slots
// (slot = (order step) mod L, so a step writes ONE slot instead of shifting L),
// the step counter, and PCG64.
//
// The reward follows NumPy 2 / NEP 50 promotion exactly: every intermediate
// carries a kind tag {Python scalar, np.float32, np.float64} and each binary op
// is evaluated in the dtype numpy would pick.
#include "kernels.hpp"

namespace invsim {
namespace {

enum { K_PY = 0, K_F32 = 1, K_F64 = 2 };
struct Tv {
    double v;
    int k;
};
__device__ __forceinline__ Tv tv(double v, int k) { return Tv{v, k}; }

template <char OP>
__device__ __forceinline__ Tv tv_bin(Tv a, Tv b) {
    if ((a.k == K_F32 && b.k != K_F64) || (b.k == K_F32 && a.k != K_F64)) {
        float fa = (float)a.v, fb = (float)b.v, fr;
        if (OP == '+') fr = fa + fb;
        else if (OP == '-') fr = fa - fb;
        else fr = fa * fb;
        return Tv{(double)fr, K_F32};
    }
    double r;
    if (OP == '+') r = a.v + b.v;
    else if (OP == '-') r = a.v - b.v;
    else r = a.v * b.v;
    return Tv{r, (a.k == K_F64 || b.k == K_F64) ? K_F64 : K_PY};
}

// numpy clip on a float64 (_NPY_CLIP: MIN(MAX(x, lo), hi), NaN propagates)
__device__ __forceinline__ double np_clip(double x, double lo, double hi) {
    double y = (x != x) ? x : (x > lo ? x : lo);
    return (y != y) ? y : (y < hi ? y : hi);
}

// newsvendor.py:100-123 for one env: 5 uniforms, params, zero pipeline, obs row
__device__ __forceinline__ void nv_reset_one(const NvParams &P, int64_t e, Pcg &g, float *orow) {
    const int64_t S = P.cm.Npad;
    double price = g.next_double() * P.p_max;
    if (!(price > 1)) price = 1;                       // max(1, x)
    double cost = g.next_double() * price;
    if (!(cost > 1)) cost = 1;
    double mn = (P.h_max < cost) ? P.h_max : cost;     // min(cost, h_max)
    double hh = g.next_double() * mn;
    double kk = g.next_double() * P.k_max;
    double mu = g.next_double() * P.mu_max;
    P.par[0 * S + e] = price;
    P.par[1 * S + e] = cost;
    P.par[2 * S + e] = hh;
    P.par[3 * S + e] = kk;
    P.par[4 * S + e] = mu;
    P.cm.period[e] = 0;
    if (orow) {
        orow[0] = (float)price;
        orow[1] = (float)cost;
        orow[2] = (float)hh;
        orow[3] = (float)kk;
        orow[4] = (float)mu;
        for (int j = 0; j < P.L; j++) orow[5 + j] = 0.f;
    }
}

// One newsvendor.py:125-204 step.  LT = compile-time lead time (>= 0) or -1
// (runtime lead time, pipeline read from HBM on demand).  Returns truncated.
template <int LT>
__device__ __forceinline__ bool nv_step_one(const NvParams &P, int64_t e, Pcg &g, float action,
                                            float *orow, double &reward, int64_t *dem) {
    const int64_t S = P.cm.Npad;
    const int L = (LT >= 0) ? LT : P.L;
    const int32_t sc = P.cm.period[e];                 // steps already taken
    // pipeline position p (0 = arriving now) lives in slot (sc + 1 + p) mod L,
    // and is empty while p < L - sc (episode younger than the lead time)
    const int base = (L > 0) ? (int)((uint32_t)(sc + 1) % (uint32_t)L) : 0;
    auto slot_of = [&](int p) {
        int s = base + p;
        return s >= L ? s - L : s;
    };
    float pv[(LT > 0) ? LT : 1];
    if (LT > 0) {
#pragma unroll
        for (int p = 0; p < (LT > 0 ? LT : 1); p++)
            pv[p] = (p >= L - sc) ? P.pipe[(int64_t)slot_of(p) * S + e] : 0.f;
    }
    auto pos = [&](int p) -> float {
        if (LT > 0) return pv[p];
        return (p >= L - sc) ? P.pipe[(int64_t)slot_of(p) * S + e] : 0.f;
    };
    const double price = P.par[0 * S + e], cost = P.par[1 * S + e], hh = P.par[2 * S + e],
                 kk = P.par[3 * S + e], mu = P.par[4 * S + e];
    const Tv ZERO = tv(0.0, K_PY);
    Tv oq = tv(np_clip((double)action, 0.0, P.max_order), K_F64);          // :131-132
    float S5 = np_sum<float>(L, pos);                                       // :135
    Tv inv = (L > 0) ? tv((double)pos(0), K_F32) : oq;                      // :136-141
    Tv cap = tv_bin<'-'>(tv(P.max_inventory, K_PY), tv((double)S5, K_F32));
    Tv m1 = (cap.v < oq.v) ? cap : oq;                                      // min(oq, cap)
    Tv q = (m1.v > 0) ? m1 : ZERO;                                          // :143
    int64_t d = np_poisson_dyn(g, mu);                                      // :146
    Tv dv = tv((double)d, K_PY);
    Tv sales = (dv.v < inv.v) ? dv : inv;                                   // :149
    Tv revenue = tv_bin<'*'>(sales, tv(price, K_PY));                       // :150
    Tv ex = tv_bin<'-'>(inv, dv);
    Tv excess = (ex.v > 0) ? ex : ZERO;                                     // :152
    Tv sh = tv_bin<'-'>(dv, inv);
    Tv shortage = (sh.v > 0) ? sh : ZERO;                                   // :153
    Tv purchase = tv_bin<'*'>(q, tv(cost, K_PY));                           // :162
    Tv holding = tv_bin<'*'>(excess, tv(hh, K_PY));                         // :166
    Tv penalty = tv_bin<'*'>(shortage, tv(kk, K_PY));                       // :167
    Tv r = tv_bin<'-'>(tv_bin<'-'>(tv_bin<'-'>(revenue, purchase), holding), penalty); // :170
    const float qf = (float)q.v;
    if (orow) {                                                             // obs after :183
        orow[0] = (float)price;
        orow[1] = (float)cost;
        orow[2] = (float)hh;
        orow[3] = (float)kk;
        orow[4] = (float)mu;
        for (int p = 0; p + 1 < L; p++) orow[5 + p] = pos(p + 1);
        if (L > 0) orow[5 + L - 1] = qf;
    }
    if (L > 0) P.pipe[(int64_t)base * S + e] = qf;                         // new order replaces the arrived slot
    const int32_t sc1 = sc + 1;
    P.cm.period[e] = sc1;
    reward = r.v;
    if (dem) dem[e] = d;
    return sc1 >= P.step_limit;                                             // :190
}

template <int LT>
__global__ void __launch_bounds__(256)
nv_step_kernel(NvParams P, const float *__restrict__ act, float *__restrict__ obs,
               double *__restrict__ rew, uint8_t *__restrict__ term, uint8_t *__restrict__ trunc,
               float *__restrict__ fobs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int O = P.L + 5;
    Pcg g = P.cm.rng.load(e);
    float *orow = obs + e * O;
    const int32_t sc = P.cm.period[e];
    if (P.cm.autoreset == AR_NEXT_STEP && sc >= P.step_limit) {
        nv_reset_one(P, e, g, orow);
        rew[e] = 0.0;
        term[e] = 0;
        trunc[e] = 0;
    } else {
        double r;
        bool tr = nv_step_one<LT>(P, e, g, act[e], orow, r, P.cm.info_demand);
        rew[e] = r;
        term[e] = 0;
        trunc[e] = tr ? 1 : 0;
        if (tr && P.cm.autoreset == AR_SAME_STEP) {
            if (fobs)
                for (int j = 0; j < O; j++) fobs[e * O + j] = orow[j];
            nv_reset_one(P, e, g, orow);
        }
    }
    P.cm.rng.store_state(e, g);
}

// K steps per launch; PCG64 state held in registers across steps.
template <int LT>
__global__ void __launch_bounds__(256)
nv_rollout_kernel(NvParams P, int K, const float *__restrict__ act, float *__restrict__ obs,
                  double *__restrict__ rew, uint8_t *__restrict__ term,
                  uint8_t *__restrict__ trunc) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int64_t N = P.cm.N;
    const int O = P.L + 5;
    Pcg g = P.cm.rng.load(e);
    for (int k = 0; k < K; k++) {
        float *orow = obs + ((int64_t)k * N + e) * O;
        const int32_t sc = P.cm.period[e];
        const int64_t oi = (int64_t)k * N + e;
        if (P.cm.autoreset == AR_NEXT_STEP && sc >= P.step_limit) {
            nv_reset_one(P, e, g, orow);
            rew[oi] = 0.0;
            term[oi] = 0;
            trunc[oi] = 0;
        } else {
            double r;
            bool tr = nv_step_one<LT>(P, e, g, act[oi], orow, r,
                                      k == K - 1 ? P.cm.info_demand : nullptr);
            rew[oi] = r;
            term[oi] = 0;
            trunc[oi] = tr ? 1 : 0;
            if (tr && P.cm.autoreset == AR_SAME_STEP) nv_reset_one(P, e, g, orow);
        }
    }
    P.cm.rng.store_state(e, g);
}

__global__ void __launch_bounds__(256)
nv_reset_kernel(NvParams P, const uint8_t *__restrict__ mask, float *__restrict__ obs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    if (mask && !mask[e]) return;
    Pcg g = P.cm.rng.load(e);
    nv_reset_one(P, e, g, obs ? obs + e * (P.L + 5) : nullptr);
    P.cm.rng.store_state(e, g);
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

#define NV_DISPATCH(LTV, LAUNCH)             \
    switch (LTV) {                           \
        case 0: LAUNCH(0); break;            \
        case 1: LAUNCH(1); break;            \
        case 2: LAUNCH(2); break;            \
        case 3: LAUNCH(3); break;            \
        case 4: LAUNCH(4); break;            \
        case 5: LAUNCH(5); break;            \
        case 6: LAUNCH(6); break;            \
        case 7: LAUNCH(7); break;            \
        case 8: LAUNCH(8); break;            \
        case 9: LAUNCH(9); break;            \
        case 10: LAUNCH(10); break;          \
        case 12: LAUNCH(12); break;          \
        case 16: LAUNCH(16); break;          \
        default: LAUNCH(-1); break;          \
    }

hipError_t nv_step_launch(const NvParams &p, const float *act, float *obs, double *rew,
                          uint8_t *term, uint8_t *trunc, float *fobs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    const dim3 grid(grid_for(p.cm.N, 256)), block(256);
#define L_(X) hipLaunchKernelGGL(nv_step_kernel<X>, grid, block, 0, s, p, act, obs, rew, term, trunc, fobs)
    NV_DISPATCH(p.L, L_)
#undef L_
    return hipGetLastError();
}

hipError_t nv_rollout_launch(const NvParams &p, int K, const float *act, float *obs, double *rew,
                             uint8_t *term, uint8_t *trunc, hipStream_t s) {
    if (p.cm.N == 0 || K <= 0) return hipSuccess;
    const dim3 grid(grid_for(p.cm.N, 256)), block(256);
#define L_(X) hipLaunchKernelGGL(nv_rollout_kernel<X>, grid, block, 0, s, p, K, act, obs, rew, term, trunc)
    NV_DISPATCH(p.L, L_)
#undef L_
    return hipGetLastError();
}

hipError_t nv_reset_launch(const NvParams &p, const uint8_t *mask, float *obs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(nv_reset_kernel, dim3(grid_for(p.cm.N, 256)), dim3(256), 0, s, p, mask, obs);
    return hipGetLastError();
}

}  // namespace invsim
