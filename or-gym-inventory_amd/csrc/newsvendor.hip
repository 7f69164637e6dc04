// NewsvendorEnv.step / reset (newsvendor.py:100-204) as HIP kernels for
// gfx950: one wave of 64 envs (one per lane) per workgroup, K steps per launch.
//
// Per-env HBM state (SoA rows of Npad): params price,cost,h,k,mu (f64: they
// are Python floats in the reference), the order pipeline as a ring of L f32
// slots (slot = order step index mod L: a step writes ONE slot instead of
// shifting L values), the step counter (only when not lock-step), PCG64.
// Inside a launch the pipeline is a positional register shift-register
// (compile-time lead time LT <= 16; LT = -1 reads the ring on demand).
//
// The reward follows NumPy 2 / NEP 50 promotion exactly: every intermediate
// carries a kind tag {Python scalar, np.float32, np.float64} and each binary
// op is evaluated in the dtype numpy would pick.
#include "kernels.hpp"

namespace invsim {
namespace {

#ifdef INVSIM_TIMING
__device__ uint64_t g_tbuf[TB_WAVES * TB_PROBES];
#endif

// NumPy-2 scalar kinds: Python float, np.float32, np.float64, Python int (poisson()
// draws and the int operands of max(1, .) / max(0, .), newsvendor.py:105-106,143-153)
enum { K_PY = 0, K_F32 = 1, K_F64 = 2, K_INT = 3 };
struct Tv {
    double v;
    int k;
};
__device__ __forceinline__ Tv tv(double v, int k) { return Tv{v, k}; }

template <char OP>
__device__ __forceinline__ Tv tv_bin(Tv a, Tv b) {
    if ((a.k == K_F32 && b.k != K_F64) || (b.k == K_F32 && a.k != K_F64)) {
        const float fa = (float)a.v, fb = (float)b.v;
        float fr;
        if (OP == '+') fr = fa + fb;
        else if (OP == '-') fr = fa - fb;
        else fr = fa * fb;
        return Tv{(double)fr, K_F32};
    }
    double r;
    if (OP == '+') r = a.v + b.v;
    else if (OP == '-') r = a.v - b.v;
    else r = a.v * b.v;
    // Python int op Python int stays int (exact here: small integers); any float makes a float
    return Tv{r, (a.k == K_F64 || b.k == K_F64) ? K_F64 : (a.k == K_INT && b.k == K_INT) ? K_INT : K_PY};
}

// numpy clip of a float64: NaN propagates, a bound is taken only when strictly
// exceeded (np.clip(-0.0, 0, hi) is -0.0)
__device__ __forceinline__ double np_clip(double x, double lo, double hi) {
    const double y = (x < lo) ? lo : x;
    return (y > hi) ? hi : y;
}

template <int LT, class G = Pcg>
struct NvState {
    G g;
    double par[5];                 // price, cost, h, k, mu
    float pv[(LT > 0) ? LT : 1];   // pipeline positions 0 (arriving) .. L-1 (newest)
};

__device__ __forceinline__ void obs_params(const double *par, float *orow) {
#pragma unroll
    for (int j = 0; j < 5; j++) orow[j] = (float)par[j];
}

// newsvendor.py:100-123: 5 uniforms, params, empty pipeline, obs row
template <int LT, class G = Pcg>
__device__ __forceinline__ void nv_reset_regs(const NvParams &P, int64_t e, NvState<LT, G> &s, float *orow,
                                              bool leader) {
    s.g.sub(PhiloxGen::RESET);                          // fast stream: the reset's own counter block
    double price = s.g.next_double() * P.p_max;
    if (!(price > 1)) price = 1;                        // max(1, x)
    double cost = s.g.next_double() * price;
    if (!(cost > 1)) cost = 1;
    const double mn = (P.h_max < cost) ? P.h_max : cost; // min(cost, h_max)
    const double hh = s.g.next_double() * mn;
    const double kk = s.g.next_double() * P.k_max;
    const double mu = s.g.next_double() * P.mu_max;
    s.par[0] = price; s.par[1] = cost; s.par[2] = hh; s.par[3] = kk; s.par[4] = mu;
    const int64_t S = P.cm.Npad;
    if (leader)
        for (int j = 0; j < 5; j++) P.par[j * S + e] = s.par[j];
    if (LT > 0) {
#pragma unroll
        for (int p = 0; p < (LT > 0 ? LT : 1); p++) s.pv[p] = 0.f;
    }
    if (orow) {
        obs_params(s.par, orow);
        for (int j = 0; j < P.L; j++) orow[5 + j] = 0.f;
    }
}

// Sum of the pipeline as the observation holds it (float32, numpy pairwise
// order): observation[5:].sum()
template <int LT, class G = Pcg>
__device__ __forceinline__ float nv_pipe_sum(const NvParams &P, int64_t e, int sc, const NvState<LT, G> &s) {
    const int64_t S = P.cm.Npad;
    const int L = (LT >= 0) ? LT : P.L;
    const int base = (L > 0) ? (int)((uint32_t)(sc + 1) % (uint32_t)L) : 0;
    return np_sum<float>(L, [&](int p) -> float {
        if (LT > 0) return s.pv[p];
        int sl = base + p;
        sl = sl >= L ? sl - L : sl;
        return (p >= L - sc) ? P.pipe[(int64_t)sl * S + e] : 0.f;
    });
}

// OrderUpToHeuristicAgent.get_action (benchmark_newsvendor.py:103-111), float32
// as numpy evaluates it: target = mu * (L + 1) * sf, order max(0, target -
// pipeline.sum()) clipped to the action space [0, max_order_quantity]
template <int LT, class G = Pcg>
__device__ __forceinline__ float nv_order_up_to(const NvParams &P, const PolicyIO &pol, int64_t e, int sc,
                                                const NvState<LT, G> &s) {
    const int L = (LT >= 0) ? LT : P.L;
    const float mu = (float)s.par[4];                                  // observation[4]
    const float target = (mu * (float)(L + 1)) * (float)pol.sf;
    const float q = target - nv_pipe_sum<LT>(P, e, sc, s);
    float o = (q > 0.f) ? q : 0.f;                                      // builtin max(0, q)
    const float hi = (float)P.max_order;
    o = (o < 0.f) ? 0.f : o;                                            // np.clip(., low[0], high[0])
    return (o > hi) ? hi : o;
}

// ---- scipy.stats.poisson.ppf for the critical-ratio agents --------------------
// Third-party (scipy 1.15.3, not in the reference): rv_discrete.ppf gives -1 at
// q == 0, inf at q == 1, NaN outside [0, 1]; otherwise poisson_gen._ppf:
//     vals = ceil(pdtrik(q, mu)); vals1 = max(vals - 1, 0)
//     return pdtr(vals1, mu) >= q ? vals1 : vals
// The agents pass q and mu as np.float32, so scipy.special's float32 loops run:
// pdtrik's root x* of the continuous CDF C(s) = Q(s + 1, mu) and pdtr are
// rounded to float32.  Restated by exact arithmetic: j* = the smallest integer
// with CDF(j) >= q; f32(x*) == j* - 1 exactly when x* < j* - 1 + ulp/2, i.e. when
// C(j* - 1 + ulp/2) > q; then the pdtr test on the f32-rounded CDF.
// (Residual: cdflib stops its root search at ~1e-11 relative, which decides
// when x* lies that close to the rounding midpoint.)

// R's dpois_raw (Loader's saddle point) for integer x > 35
__device__ double ppf_dpois_raw(double x, double lam) {
    const double nn = x * x;
    const double S0 = 1.0 / 12, S1 = 1.0 / 360, S2 = 1.0 / 1260, S3 = 1.0 / 1680;
    double st;
    if (x > 500) st = (S0 - S1 / nn) / x;
    else if (x > 80) st = (S0 - (S1 - S2 / nn) / nn) / x;
    else st = (S0 - (S1 - (S2 - S3 / nn) / nn) / nn) / x;
    const double d = x - lam;
    double bd;
    if (fabs(d) < 0.1 * (x + lam)) {
        double v = d / (x + lam);
        double s = d * v;
        double ej = 2 * x * v;
        v = v * v;
        for (int j = 1; j < 1000; j++) {
            ej *= v;
            const double s1 = s + ej / (2 * j + 1);
            if (s1 == s) break;
            s = s1;
        }
        bd = s;
    } else {
        bd = x * log(x / lam) + lam - x;
    }
    return exp(-st - bd) / sqrt(2 * M_PI * x);
}

// regularised upper incomplete gamma Q(a, x), real a > 0, x > 0: series for
// P below a + 1, modified Lentz continued fraction above
__device__ double ppf_igamc(double a, double x) {
    const double lpre = -x + a * log(x) - lgamma(a);
    if (x < a + 1) {
        double s = 1.0 / a, d = s;
        for (int n = 1; n < 100000; n++) {
            d *= x / (a + n);
            s += d;
            if (fabs(d) < fabs(s) * 1e-17) break;
        }
        return 1.0 - s * exp(lpre);
    }
    const double tiny = 1e-300;
    double b = x + 1 - a, c = 1 / tiny, d = 1 / b, h = d;
    for (int i = 1; i < 100000; i++) {
        const double an = -i * (i - a);
        b += 2;
        d = an * d + b;
        if (fabs(d) < tiny) d = tiny;
        c = b + an / c;
        if (fabs(c) < tiny) c = tiny;
        d = 1 / d;
        const double de = d * c;
        h *= de;
        if (fabs(de - 1) < 1e-16) break;
    }
    return exp(lpre) * h;
}

// poisson.ppf(q, mu); single: q and mu reach scipy as np.float32 (else float64)
__device__ double nv_poisson_ppf(double q, double lam, bool single) {
    if (q != q) return NAN;
    if (q == 0) return -1.0;
    if (q == 1) return INFINITY;
    if (!(q > 0 && q < 1)) return NAN;
    // bounded work per lane: the host refuses a policy whose mean can exceed 1e6;
    // params injected past 1e7 by set_state give NaN (order 0)
    if (!(lam <= 1e7)) return NAN;
    // CDF by the pmf recurrence from i0, below which the mass is < 1e-80
    const double sd = sqrt(lam);
    double i0 = lam > 700 ? floor(lam - 20 * sd) : 0;
    double p = (i0 > 0) ? ppf_dpois_raw(i0, lam) : exp(-lam);
    double P = p, Pm1 = 0, Pm2 = 0;                                     // CDF(j), CDF(j-1), CDF(j-2)
    double j = i0 > 0 ? i0 : 0;
    const double jmax = lam + 40 * sd + 64;
    while (P < q && j < jmax) {
        j += 1;
        p = p * lam / j;
        Pm2 = Pm1;
        Pm1 = P;
        P += p;
    }
    if (!single) return j;                                              // float64 loops: exact j*
    double vals = j;
    if (j >= 2) {
        int ex;
        frexp(j - 1, &ex);                                              // j-1 in [2^(ex-1), 2^ex)
        const double half = ldexp(1.0, ex - 1 - 24);                    // half an f32 ulp there
        if (ppf_igamc(j + half, lam) > q) vals = j - 1;                 // f32(x*) == j - 1
    }
    const double vals1 = vals > 1 ? vals - 1 : 0;
    const double c = (vals1 == j) ? P : (vals1 == j - 1) ? Pm1 : (vals1 == j - 2) ? Pm2 : 0.0;
    return ((float)c >= (float)q) ? vals1 : vals;
}

// ClassicNewsvendorAgent.get_action (benchmark_newsvendor.py:121-161).  The
// observation's params are float32 and every expression keeps numpy's dtypes:
// the critical ratio and the effective mean are float32, poisson.ppf returns
// float64, and the order is clipped in float64 and cast to float32.  The ppf
// level depends only on the episode's params: computed once per episode (lvl).
template <int LT, class G = Pcg>
__device__ __forceinline__ float nv_classic(const NvParams &P, const PolicyIO &pol, int64_t e, int sc,
                                            const NvState<LT, G> &s, double &lvl, bool &have) {
    const int L = (LT >= 0) ? LT : P.L;
    const float price = (float)s.par[0], cost = (float)s.par[1], h = (float)s.par[2], k = (float)s.par[3],
                mu = (float)s.par[4];
    const float eps = 1e-6f;                                            // Python 1e-6 against float32 (NEP 50)
    bool fb;
    float cr = 0.f;
    if (pol.variant == 1) {                                             // 'profit_margin' (:128-134)
        const float under = (price - cost) + k, over = h;
        fb = (under + over <= eps) || (under <= 0.f) || (over <= 0.f);
        if (!fb) cr = under / (under + over);
    } else {                                                            // 'k_vs_h' and default (:135-142)
        fb = (h + k <= eps) || (k < 0.f) || (h < 0.f);
        if (!fb) cr = k / (h + k);
    }
    const float pos = nv_pipe_sum<LT>(P, e, sc, s);                     // pipeline_inventory.sum()
    const float hi = (float)P.max_order;
    if (fb) {                                                           // :144-148, float32
        const float q = mu * (float)(L + 1) - pos;
        float o = (q > 0.f) ? q : 0.f;
        o = (o < 0.f) ? 0.f : o;
        return (o > hi) ? hi : o;
    }
    if (!have) {                                                        // :151-153
        const float eff = (mu * (float)(L + 1)) * (float)pol.sf;
        const bool f = eff > eps;                                       // max(1e-6, effective_mu)
        lvl = nv_poisson_ppf((double)cr, f ? (double)eff : 1e-6, f);
        have = true;
    }
    const double d = lvl - (double)pos;                                 // float64 - float32
    double o = (d > 0) ? d : 0.0;                                       // builtin max(0, .)
    o = (o < 0.0) ? 0.0 : o;                                            // np.clip (:160)
    o = (o > (double)hi) ? (double)hi : o;
    return (float)o;
}

// sSPolicyAgent.get_action (benchmark_newsvendor_sb3_rllib.py:363-371, the
// module's last definition): s = ppf(clip(k / (h + k), 0.001, 0.999), mu (L + 1))
// in float32 inputs, S = s * S_buffer_factor; order up to S when the pipeline is
// below s.  The level s is per episode (lvl).
template <int LT, class G = Pcg>
__device__ __forceinline__ float nv_ss(const NvParams &P, const PolicyIO &pol, int64_t e, int sc,
                                       const NvState<LT, G> &s, double &lvl, bool &have) {
    const int L = (LT >= 0) ? LT : P.L;
    if (!have) {
        const float h = (float)s.par[2], k = (float)s.par[3], mu = (float)s.par[4];
        const float eps = 1e-6f;
        double sl = 0.0;                                                // s_lvl = 0
        if (h + k > eps) {
            float q = k / (h + k);
            q = (q < 0.001f) ? 0.001f : q;                              // np.clip(cr_s, 0.001, 0.999): float32
            q = (q > 0.999f) ? 0.999f : q;
            const float eff = mu * (float)(L + 1);
            const bool f = eff > eps;
            sl = nv_poisson_ppf((double)q, f ? (double)eff : 1e-6, f);
        }
        lvl = (sl > 0) ? sl : 0.0;                                      // s_level = max(0, s_lvl)
        have = true;
    }
    const float pos = nv_pipe_sum<LT>(P, e, sc, s);
    const double S_level = lvl * pol.sf;
    double o = 0.0;
    if ((double)pos < lvl) {
        const double d = S_level - (double)pos;
        o = (d > 0) ? d : 0.0;
    }
    const double hi = (double)(float)P.max_order;
    o = (o < 0.0) ? 0.0 : o;
    o = (o > hi) ? hi : o;
    return (float)o;
}

// One newsvendor.py:125-204 step at step count sc.  Returns truncated.
template <int LT, class G = Pcg>
__device__ __forceinline__ bool nv_step_regs(const NvParams &P, int64_t e, bool valid, int sc, NvState<LT, G> &s,
                                             float action, float *orow, const double *lg_l, TableStage *ts,
                                             double &reward, int64_t *dem, int64_t dpre = -1,
                                             double *irec = nullptr, bool ring_store = true) {
    const int64_t S = P.cm.Npad;
    const int L = (LT >= 0) ? LT : P.L;
    const int base = (L > 0) ? (int)((uint32_t)(sc + 1) % (uint32_t)L) : 0;  // slot of position 0
    auto pos = [&](int p) -> float {
        if (LT > 0) return s.pv[p];
        int sl = base + p;
        sl = sl >= L ? sl - L : sl;
        return (p >= L - sc) ? P.pipe[(int64_t)sl * S + e] : 0.f;
    };
    if (ts) ts->flush((int)threadIdx.x);
    TPROBE(1);
    // :146 (dpre >= 0: drawn by the previous launch's lookahead, nv_step1_kernel)
    if (dpre < 0) s.g.sub(0);
    const int64_t d = dpre >= 0 ? dpre : env_poisson_dyn(s.g, s.par[4], lg_l, RHS_LDS_MAX);
    TPROBE(2);
    const Tv ZERO = tv(0.0, K_INT);                                         // the 0 of max(0, .)
    const Tv oq = tv(np_clip((double)action, 0.0, P.max_order), K_F64);    // :131-132
    const float S5 = np_sum<float>(L, pos);                                 // :135
    const Tv inv = (L > 0) ? tv((double)pos(0), K_F32) : oq;                // :136-141
    const Tv cap = tv_bin<'-'>(tv(P.max_inventory, K_PY), tv((double)S5, K_F32));
    const Tv m1 = (cap.v < oq.v) ? cap : oq;                                // min(oq, cap)
    const Tv q = (m1.v > 0) ? m1 : ZERO;                                    // :143
    const Tv dv = tv((double)d, K_INT);                                     // poisson() -> Python int
    const Tv sales = (dv.v < inv.v) ? dv : inv;                             // :149
    // price / cost are the Python int 1 when max(1, .) took its first operand (:105-106)
    const Tv price = tv(s.par[0], s.par[0] == 1.0 ? K_INT : K_PY), cost = tv(s.par[1], s.par[1] == 1.0 ? K_INT : K_PY);
    const Tv revenue = tv_bin<'*'>(sales, price);                           // :150
    const Tv ex = tv_bin<'-'>(inv, dv);
    const Tv excess = (ex.v > 0) ? ex : ZERO;                               // :152
    const Tv sh = tv_bin<'-'>(dv, inv);
    const Tv shortage = (sh.v > 0) ? sh : ZERO;                             // :153
    const Tv purchase = tv_bin<'*'>(q, cost);                               // :162
    const Tv holding = tv_bin<'*'>(excess, tv(s.par[2], K_PY));             // :166
    const Tv penalty = tv_bin<'*'>(shortage, tv(s.par[3], K_PY));           // :167
    const Tv r = tv_bin<'-'>(tv_bin<'-'>(tv_bin<'-'>(revenue, purchase), holding), penalty); // :170
    const float qf = (float)q.v;
    if (orow) {                                                             // obs after :183
        obs_params(s.par, orow);
        for (int p = 0; p + 1 < L; p++) orow[5 + p] = pos(p + 1);
        if (L > 0) orow[5 + L - 1] = qf;
    }
    if (L > 0 && valid && ring_store) P.pipe[(int64_t)base * S + e] = qf;  // replaces the arrived slot
    if (LT > 0) {
#pragma unroll
        for (int p = 0; p + 1 < (LT > 0 ? LT : 1); p++) s.pv[p] = s.pv[p + 1];
        s.pv[(LT > 0 ? LT : 1) - 1] = qf;
    }
    reward = r.v;
    if (dem) dem[e] = d;
    if (irec) {   // step info (:195-199): the cost components, values and NumPy-2 kinds
        double *rr = irec + e * 5;
        rr[0] = revenue.v;
        rr[1] = purchase.v;
        rr[2] = holding.v;
        rr[3] = penalty.v;
        rr[4] = (double)(revenue.k + 4 * purchase.k + 16 * holding.k + 64 * penalty.k);
    }
    TPROBE(3);
    return sc + 1 >= P.step_limit;                                          // :190
}

template <int LT, bool TU, bool ONE, bool POL, class G>
__global__ void __launch_bounds__(WAVE)
nv_run_kernel(NvParams P, int t_u, StepIO<float, float> io, PolicyIO pol) {
    extern __shared__ __attribute__((aligned(16))) float nv_tile[];
    const int lane = threadIdx.x;
    const bool leader = (lane & (LPE - 1)) == 0;
    const int64_t e0 = (int64_t)blockIdx.x * EPW;
    const int64_t e = e0 + lane / LPE;
    const int64_t N = P.cm.N;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < EPW ? (N - e0) : EPW);
    const int O = P.L + 5;
    const int64_t S = P.cm.Npad;
    float *trow = nv_tile + (int64_t)(lane / LPE) * O;
    TPROBE(0);
    TPROBE_ID();
    // obs tile of at most 64 x (16 + 5) f32 in the compile-time lead-time variants
    constexpr int TILE_IT = (EPW * 21 * 4 + 16 * WAVE - 1) / (16 * WAVE);
    // lanes past N mirror env N-1 (loads only; they store nothing): straight-line
    // loads keep the compiler's waits exact, and a real PCG64 stream / rate keeps
    // the Poisson loop finite
    const int64_t el = valid ? e : N - 1;

    NvState<LT, G> st;
    P.cm.rng.load(el, st.g);
    st.g.set_step(P.cm.ph_step);
    int sc = TU ? t_u : P.cm.period[el];
    if (ONE && TU && sc >= P.step_limit && P.cm.autoreset == AR_NEXT_STEP) {
        // lock-step NEXT_STEP autoreset of the whole batch.  DISABLED keeps stepping
        // the same episode past step_limit with truncated=True (newsvendor.py:190
        // has no horizon check; the oracle does the same, oracle.c nv_step), and
        // SAME_STEP resets in the done step, so neither reaches this branch
        nv_reset_regs<LT>(P, e, st, trow, valid);
        if (valid) {
            out_store(io.rew + e, 0.0);
            out_store(io.term + e, (uint8_t)0);
            out_store(io.trunc + e, (uint8_t)0);
            P.cm.rng.store_state(e, st.g);
        }
        wave_lds_sync();
        store_tile<TILE_IT>(nv_tile, io.obs + e0 * O, (int64_t)nvalid * O, lane);
        return;
    }
    // loggam(k + 1) table -> LDS after the tile (written once the step's loads are in flight)
    TableStage ts;
    ts.dst = reinterpret_cast<double *>(nv_tile + ((EPW * O + 3) / 4) * 4);
    ts.load(P.lgtab, RHS_LDS_MAX, lane);
#pragma unroll
    for (int j = 0; j < 5; j++) st.par[j] = P.par[j * S + el];
    if (LT > 0) {
        const int base = (int)((uint32_t)(sc + 1) % (uint32_t)(LT > 0 ? LT : 1));
#pragma unroll
        for (int p = 0; p < (LT > 0 ? LT : 1); p++) {
            int sl = base + p;
            sl = sl >= LT ? sl - LT : sl;
            st.pv[p] = P.pipe[(int64_t)sl * S + el];
            if (!(p >= LT - sc)) st.pv[p] = 0.f;
        }
    }
    constexpr int MD = 2;                       // metrics: reward sum, steps
    double met[MD];
#pragma unroll
    for (int q = 0; q < MD; q++) met[q] = (POL && pol.metrics) ? pol.metrics[el * MD + q] : 0.0;
    const int K = ONE ? 1 : io.K;
    double lvl = 0.0;     // CLASSIC_NV / SS: the episode's ppf level, once computed
    bool have = false;
    // all lanes write the table: before any divergent step/reset branch (with a
    // lock-step single step there is none, and the write waits inside the step)
    if (!(ONE && TU)) ts.flush(lane);
    for (int k = 0; k < K; k++) {
        const int64_t oi = (int64_t)k * N + e;
        float act;
        st.g.set_step(P.cm.ph_step + (uint64_t)k);
        if (!POL) act = io.act[(int64_t)k * N + el];
        if (!(ONE && TU) && P.cm.autoreset == AR_NEXT_STEP && sc >= P.step_limit) {
            nv_reset_regs<LT>(P, e, st, trow, valid);
            have = false;
            if (valid && (!POL || io.rew)) {
                out_store(io.rew + oi, 0.0);
                out_store(io.term + oi, (uint8_t)0);
                out_store(io.trunc + oi, (uint8_t)0);
            }
            sc = 0;
        } else {
            double r;
            if (POL) {
                if (pol.kind == POL_ORDER_UP_TO) act = nv_order_up_to<LT>(P, pol, e, sc, st);
                else if (pol.kind == POL_CLASSIC_NV) act = nv_classic<LT>(P, pol, e, sc, st, lvl, have);
                else if (pol.kind == POL_SS) act = nv_ss<LT>(P, pol, e, sc, st, lvl, have);
                else act = pol.cf[0];
                if (valid && pol.act_out) out_store((float *)pol.act_out + oi, act);
            }
            const bool tr = nv_step_regs<LT>(P, e, valid, sc, st, act, trow, ts.dst, (ONE && TU) ? &ts : nullptr, r,
                                             (valid && k == K - 1) ? P.cm.info_demand : nullptr, -1,
                                             (valid && k == K - 1) ? (double *)P.cm.info_rec : nullptr);
            if (POL) {
                met[0] += r;                    // episode_reward += reward (benchmark_newsvendor.py:241)
                met[1] += 1.0;
            }
            if (valid && (!POL || io.rew)) {
                out_store(io.rew + oi, r);
                out_store(io.term + oi, (uint8_t)0);
                out_store(io.trunc + oi, (uint8_t)(tr ? 1 : 0));
            }
            sc += 1;
            if (tr && P.cm.autoreset == AR_SAME_STEP) {
                wave_lds_sync();
                if (io.fobs && valid)
                    for (int j = 0; j < O; j++) io.fobs[e * O + j] = trow[j];
                wave_lds_sync();
                nv_reset_regs<LT>(P, e, st, trow, valid);
                have = false;
                sc = 0;
            }
        }
        wave_lds_sync();
        if (!POL || io.obs) store_tile<TILE_IT>(nv_tile, io.obs + ((int64_t)k * N + e0) * O, (int64_t)nvalid * O, lane);
        TPROBE(4);
        wave_lds_sync();
    }
    if (valid) {
        P.cm.rng.store_state(e, st.g);
        if (!TU) P.cm.period[e] = sc;
        if (POL && pol.metrics) {
#pragma unroll
            for (int q = 0; q < MD; q++) pol.metrics[e * MD + q] = met[q];
        }
    }
    TWAIT();
    TPROBE(5);
}

// numpy random_poisson's constants of a per-env rate, computed once per episode
// (np_poisson_dyn recomputes them per draw)
__device__ __forceinline__ PtrsConst nv_rate_const(double lam) {
    PtrsConst c;
    c.lam = lam;
    c.slam = sqrt(lam);
    c.loglam = log(lam);
    c.b = 0.931 + 2.53 * c.slam;
    c.a = -0.059 + 0.02483 * c.b;
    c.invalpha = 1.1239 + 1.1328 / (c.b - 3.4);
    c.vr = 0.9277 - 3.6224 / (c.b - 2);
    c.log_invalpha = log(c.invalpha);
    c.a2 = 2 * c.a;
    c.enlam = exp(-lam);
    c.k0 = 0;
    c.nk = 0;
    return c;
}

// np_poisson_dyn with the episode's constants (same draws, same arithmetic)
template <class G>
__device__ __forceinline__ int64_t nv_poisson_c(G &g, const PtrsConst &c, const double *lgtab) {
    if (c.lam >= 10) return np_poisson_ptrs_lg(g, c, lgtab, RHS_LDS_MAX);
    if (c.lam == 0) return 0;
    return np_poisson_mult(g, c.enlam);
}

// Single lock-step step (invsim_step: K = 1, t_u < step_limit, no policy, not a
// SAME_STEP done step) with the demand lookahead.  The demand of a step is
// Poisson(mu) of the env's own stream, and mu is fixed for the episode, so the
// launch of step t can already draw step t+1's demand (PRODUCE, i.e. t+1 <
// step_limit: the step after the last one is a reset, which draws uniforms).
// P.ahead: two slots of rows [state hi, state lo, demand] x Npad, alternating.
//   HIT (slot cur holds each env's state one draw past the committed one and
//        that draw): the step workgroups load d; `gla` workgroups at the front
//        of the grid draw the next demand from slot cur's state into slot cur^1
//        (PRODUCE) -- the per-env-rate Poisson chain runs beside the step -- or
//        copy slot cur's state to cm.rng (!PRODUCE: the cache ends here).
//   !HIT && PRODUCE: the step draws d inline from cm.rng, leaves the state in
//        slot cur, then draws the lookahead into slot cur^1.
// After a PRODUCE launch the committed state (after this step's draw) is slot
// cur, the host flips the slots, and cm.rng is brought up to date from it
// (nv_commit_kernel) only before something reads it.  Streams are consumed in
// the reference's order; arithmetic as nv_step_regs (newsvendor.py:125-204).
// RG = PhiloxGen (the fast stream, newsvendor_ph.hip): the same lookahead, but a
// draw is a function of (key, launch step, mu) only, so a slot holds just the
// next step's demand (row 2) and no generator state is read or written; with
// !PRODUCE the host launches no lookahead workgroups (there is nothing to commit).
template <int LT, bool HIT, bool PRODUCE, class RG = Pcg>
__global__ void __launch_bounds__(WAVE)
nv_step1_kernel(NvParams P, int sc, StepIO<float, float> io, int cur, int gla, int xcdpair) {
    extern __shared__ __attribute__((aligned(16))) float nv_tile[];
    const int lane = threadIdx.x;
    const int64_t N = P.cm.N;
    const int64_t S = P.cm.Npad;
    const int O = P.L + 5;
    double *lg_l = reinterpret_cast<double *>(nv_tile + ((EPW * O + 3) / 4) * 4);
    const uint64_t *Acur = P.ahead + (int64_t)cur * 3 * S;
    uint64_t *Anxt = P.ahead + (int64_t)(cur ^ 1) * 3 * S;
    const int bid = (int)blockIdx.x;
    TPROBE(0);
    TPROBE_ID();
    if (HIT && bid < gla) {   // ---- lookahead workgroups
        // PRODUCE: two workgroups per 64 envs, one per branch of numpy's sampler
        // (bid even: PTRS for lam >= 10 and lam == 0; odd: the multiplication
        // method for 0 < lam < 10), so a wave runs one branch, not both one
        // after the other; a lane works only on the workgroup of its env's branch
        // PRODUCE: which 64 envs and which branch.  xcdpair: the two workgroups of
        // a group are 8 apart (blocks of 16 = 8 groups x 2 branches), so both --
        // and the group's step workgroup, when gla % 8 == 0 -- run on the same XCD
        // (dispatch is round-robin over the 8) and share its L2 for the rows both
        // read (state, increment, mu); else adjacent (bid >> 1, bid & 1)
        int grp = PRODUCE ? bid >> 1 : bid, brn = bid & 1;
        if (PRODUCE && xcdpair && (bid | 15) < gla) {
            grp = ((bid >> 4) << 3) + (bid & 7);
            brn = (bid >> 3) & 1;
        }
        const int64_t e = (int64_t)grp * WAVE + lane;
        const bool valid = e < N;
        const int64_t el = valid ? e : N - 1;
        if constexpr (RG::kCounter) {   // the fast stream: the draw of launch step ph_step + 1
            if (!PRODUCE) return;
            RG g;
            P.cm.rng.load(el, g);
            g.set_step(P.cm.ph_step + 1);
            g.sub(0);
            const double mu = P.par[4 * S + el];
            const bool mult_wg = brn;
            if (!mult_wg) {
                TableStage ts;
                ts.dst = lg_l;
                ts.load(P.lgtab, RHS_LDS_MAX, lane);
                ts.flush(lane);
            }
            const bool mine = mult_wg == (mu < 10 && mu != 0);
            if (!mine) return;
            PtrsConst c;   // the sampler branch's own constants only (PTRS: rows 0-4, else exp(-mu))
            c.lam = mu;
            c.a = c.b = c.vr = c.loglam = c.log_invalpha = c.enlam = 0.0;
            if (mu >= 10) {
                c.a = P.pcon[el];
                c.b = P.pcon[S + el];
                c.vr = P.pcon[2 * S + el];
                c.loglam = P.pcon[3 * S + el];
                c.log_invalpha = P.pcon[4 * S + el];
            } else {
                c.enlam = P.pcon[5 * S + el];
            }
            c.a2 = 2 * c.a;
            c.k0 = 0;
            c.nk = 0;
            const int64_t dn = nv_poisson_c(g, c, lg_l);
            if (valid) st_store(Anxt + 2 * S + e, (uint64_t)dn);
            return;
        } else {
        Pcg g;
        g.hi = Acur[el];
        g.lo = Acur[S + el];
        if (PRODUCE) {
            g.inc_hi = P.cm.rng.inc_hi[el];
            g.inc_lo = P.cm.rng.inc_lo[el];
            const double mu = P.par[4 * S + el];
            const bool mult_wg = brn;
            // the chain's constants (nv_rate_const(mu), stored by its first launch),
            // only the sampler branch's: the PTRS workgroup reads rows 0-4 for every
            // lane, issued with the state and table loads instead of after mu has
            // arrived (its lanes are ~95 % PTRS envs, so the rows' lines are read
            // anyway); exp(-mu) only by the lanes that draw by multiplication
            PtrsConst c;
            c.lam = mu;
            c.a = c.b = c.vr = c.loglam = c.log_invalpha = c.enlam = 0.0;
            if (!mult_wg) {
                c.a = P.pcon[el];
                c.b = P.pcon[S + el];
                c.vr = P.pcon[2 * S + el];
                c.loglam = P.pcon[3 * S + el];
                c.log_invalpha = P.pcon[4 * S + el];
            }
            TableStage ts;
            if (!mult_wg) {
                ts.dst = lg_l;
                ts.load(P.lgtab, RHS_LDS_MAX, lane);
                ts.flush(lane);
            }
            const bool mine = mult_wg == (mu < 10 && mu != 0);
            if (mine && !(mu >= 10)) c.enlam = P.pcon[5 * S + el];
            c.a2 = 2 * c.a;
            c.k0 = 0;
            c.nk = 0;
            TPROBE(1);
            int64_t dn = 0;
            if (!mult_wg) {   // PTRS (lam >= 10) with a compacted second round (group_rng.hpp)
                PtrsJumpLane jt;
                jt.load(lane);
                const bool live = mine && c.lam >= 10;
                dn = np_poisson_ptrs_compact(
                    g, c, LgTab{lg_l},   // as np_poisson_ptrs_lg
                    live, jt,
                    [](const PtrsConst &cc, int src) {
                        PtrsConst r = cc;
                        r.lam = __shfl(cc.lam, src);
                        r.a2 = __shfl(cc.a2, src);
                        r.b = __shfl(cc.b, src);
                        r.vr = __shfl(cc.vr, src);
                        r.loglam = __shfl(cc.loglam, src);
                        r.log_invalpha = __shfl(cc.log_invalpha, src);
                        r.a = __shfl(cc.a, src);
                        return r;
                    },
                    [&](int i) { TPROBE_AT(i, 0); });
                if (mine && !live) dn = nv_poisson_c(g, c, lg_l);   // lam == 0 or NaN
            } else if (mine) {
                dn = nv_poisson_c(g, c, lg_l);
            }
            TPROBE(2);
            if (mine && valid) {
                st_store(Anxt + e, g.hi);
                st_store(Anxt + S + e, g.lo);
                st_store(Anxt + 2 * S + e, (uint64_t)dn);
            }
        } else if (valid) {
            st_store(P.cm.rng.hi + e, g.hi);
            st_store(P.cm.rng.lo + e, g.lo);
        }
        TWAIT();
        TPROBE(5);
        return;
        }
    }
    const int64_t e0 = (int64_t)(bid - (HIT ? gla : 0)) * EPW;
    const int64_t e = e0 + lane;
    const bool valid = e < N;
    const int nvalid = (int)((N - e0) < EPW ? (N - e0) : EPW);
    const int64_t el = valid ? e : N - 1;
    float *trow = nv_tile + (int64_t)lane * O;
    constexpr int TILE_IT = (EPW * 21 * 4 + 16 * WAVE - 1) / (16 * WAVE);
    NvState<LT, RG> st;
    TableStage ts;
    int64_t dpre = -1;
    if (HIT) {
        dpre = (int64_t)Acur[2 * S + el];
    } else {
        P.cm.rng.load(el, st.g);
        st.g.set_step(P.cm.ph_step);
        st.g.sub(0);
        ts.dst = lg_l;
        ts.load(P.lgtab, RHS_LDS_MAX, lane);
    }
#pragma unroll
    for (int j = 0; j < 5; j++) st.par[j] = P.par[j * S + el];
    if (LT > 0) {
        const int base = (int)((uint32_t)(sc + 1) % (uint32_t)(LT > 0 ? LT : 1));
#pragma unroll
        for (int p = 0; p < (LT > 0 ? LT : 1); p++) {
            int sl = base + p;
            sl = sl >= LT ? sl - LT : sl;
            st.pv[p] = P.pipe[(int64_t)sl * S + el];
            if (!(p >= LT - sc)) st.pv[p] = 0.f;
        }
    }
    const float act = io.act[el];
    PtrsConst c;
    if (!HIT) {   // this launch starts a lookahead chain: the episode's constants, once
        c = nv_rate_const(st.par[4]);
        ts.flush(lane);
        dpre = nv_poisson_c(st.g, c, lg_l);                                // :146
        if (valid) {
            st_store(P.pcon + e, c.a);
            st_store(P.pcon + S + e, c.b);
            st_store(P.pcon + 2 * S + e, c.vr);
            st_store(P.pcon + 3 * S + e, c.loglam);
            st_store(P.pcon + 4 * S + e, c.log_invalpha);
            st_store(P.pcon + 5 * S + e, c.enlam);
        }
    }
    double r;
    const bool tr = nv_step_regs<LT>(P, e, valid, sc, st, act, trow, lg_l, nullptr, r,
                                     valid ? P.cm.info_demand : nullptr, dpre,
                                     valid ? (double *)P.cm.info_rec : nullptr);
    if (valid) {
        out_store(io.rew + e, r);
        out_store(io.term + e, (uint8_t)0);
        out_store(io.trunc + e, (uint8_t)(tr ? 1 : 0));
    }
    wave_lds_sync();
    store_tile<TILE_IT>(nv_tile, io.obs + e0 * O, (int64_t)nvalid * O, lane);
    TPROBE(4);
    if (!HIT) {   // PRODUCE (the host runs nv_run_kernel for !HIT && !PRODUCE)
        if constexpr (RG::kCounter) {
            st.g.set_step(P.cm.ph_step + 1);
            st.g.sub(0);
        } else if (valid) {
            st_store((uint64_t *)Acur + e, st.g.hi);
            st_store((uint64_t *)Acur + S + e, st.g.lo);
        }
        const int64_t dn = nv_poisson_c(st.g, c, lg_l);
        if (valid) {
            if constexpr (!RG::kCounter) {
                st_store(Anxt + e, st.g.hi);
                st_store(Anxt + S + e, st.g.lo);
            }
            st_store(Anxt + 2 * S + e, (uint64_t)dn);
        }
    }
    TWAIT();
    TPROBE(5);
}

__device__ __forceinline__ void nv_wg_sync() {
    TBAR_T0();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    TBAR_ADD();
}

// numpy's sampler branch of a rate: true = the multiplication method (0 < lam < 10;
// like nv_poisson_c, anything not >= 10 and not 0 -- NaN included -- goes there)
__device__ __forceinline__ bool nv_mult_branch(double lam) { return !(lam >= 10) && lam != 0; }

// Launch-step chunks of the rollout: a chunk ends after CH steps, at a reset
// step (NEXT_STEP, period >= step_limit: the chunk's last step), or at the end
// of the launch.  Every wave derives the same chunks from the lock-step period.
__device__ __forceinline__ void nv_chunk(int t, int rem, int step_limit, bool nxt, int ch, int &len, bool &rs) {
    len = 0;
    rs = false;
    while (len < ch && len < rem) {
        len++;
        if (nxt && t >= step_limit) {
            rs = true;
            break;
        }
        t++;
    }
}

// numpy random_poisson_mult draws of one rollout chunk for the multiplication
// wave's envs (0 < lam < 10: ~5 % of envs at the default mu_max, a few per
// workgroup), G lanes per env.  The sequential sampler costs one PCG64 step
// (a 128-bit multiply) per uniform and lam + 1 uniforms per draw on the
// wave's critical path; here the G lanes of an env's group compute the next G
// uniforms of its stream at once by jump-ahead (lane jl: state after jl + 1
// LCG steps = A_{jl+1} s + S_{jl+1} inc, group_rng.hpp), then every lane of
// the group runs the product chain over them in stream order -- the same
// roundings, comparisons and draw boundaries as numpy (a round's uniforms can
// finish one draw and start the next) -- and the group's base state advances
// by the uniforms actually consumed.  Owners (lanes with `own`) hand their
// generator to the group and get it back advanced; the lane holding a
// draw-ending uniform writes that draw into the owner's column of `dcol`
// ([CH][WAVE], as doubles: the rollout's demand handoff rows hold every draw
// as a double, see nv_roll_kernel).
// G = 16 for up to 4 envs, then the even count that fits (12 for 5 envs, ...,
// 4 for 11-16); more than 16 envs (small mu_max) keep the one-lane sequential
// sampler (the caller's fallback): returns false.
__device__ __forceinline__ bool nv_mult_chunk_grp(Pcg &g, double enlam, bool own, int nd, double *dcol,
                                                  double *ubuf, const uint64_t *jt, int lane) {
    const uint64_t mm = (uint64_t)__ballot(own && nd > 0);
    const int nm = __popcll(mm);
    if (nm > 16) return false;
    if (nm == 0) return true;
    // G: 16 lanes per env up to 4 envs, else the even count that fits (12,
    // 10, 8, 8, 6, 6, then 4): the workgroups with 5-10 such envs are the
    // kernel's tail, and their rounds scale with 1 / G
    const int G = nm <= 4 ? 16 : nm == 5 ? 12 : nm == 6 ? 10 : nm <= 8 ? 8 : nm <= 10 ? 6 : 4;
    // lane / G as a multiply and shift (exact for lanes < 64 with these G)
    const int M = G == 16 ? 4096 : G == 12 ? 5462 : G == 10 ? 6554 : G == 8 ? 8192 : G == 6 ? 10923 : 16384;
    const int grp = (lane * M) >> 16, jl = lane - grp * G, gbase = grp * G;
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
    int *slot = reinterpret_cast<int *>(ubuf);
    if (own && nd > 0) slot[rank] = lane;                // owner lane of group `rank`
    wave_lds_sync();
    const bool act = grp < nm;
    const int src = act ? slot[grp] : lane;
    wave_lds_sync();
    Pcg s;
    s.hi = shfl_u64(g.hi, src);
    s.lo = shfl_u64(g.lo, src);
    s.inc_hi = shfl_u64(g.inc_hi, src);
    s.inc_lo = shfl_u64(g.inc_lo, src);
    const double en = __shfl(enlam, src);
    // jt: the jump table (group_rng.hpp) staged in LDS, rows a_hi, a_lo, s_hi, s_lo
    const uint64_t ah = jt[jl + 1], al = jt[(JUMP_MAX + 1) + jl + 1];
    uint64_t sih, sil;
    mul128(jt[2 * (JUMP_MAX + 1) + jl + 1], jt[3 * (JUMP_MAX + 1) + jl + 1], s.inc_hi, s.inc_lo, sih, sil);
    int j = act ? 0 : nd;
    int X = 0;
    double prod = 1.0;
    // the uniforms this lane's chain reads: its group's, or (idle lanes past the
    // last group, need = 0) group 0's, so every read stays inside ubuf[WAVE]
    const int rbase = act ? gbase : 0;
    while (__ballot(j < nd)) {
        TTRIP_ADD(1);
        const bool live = j < nd;
        // state after jl + 1 LCG steps: A s + S inc (mod 2^128)
        const unsigned __int128 nx = ((((unsigned __int128)s.hi) << 64) | s.lo) * ((((unsigned __int128)ah) << 64) | al) +
                                     ((((unsigned __int128)sih) << 64) | sil);
        const uint64_t th = (uint64_t)(nx >> 64), tl = (uint64_t)nx;
        const uint64_t x = th ^ tl;
        const unsigned rot = (unsigned)(th >> 58);
        const uint64_t o = (x >> rot) | (x << ((64u - rot) & 63u));
        ubuf[lane] = (double)(o >> 11) * (1.0 / 9007199254740992.0);
        wave_lds_sync();
        // the product chain over the round's uniforms in stream order (4 loaded
        // at a time, then 2 when G is not a multiple of 4): prod, and a bit per uniform that
        // ends a draw (prod <= enlam); then the draws, in order, from the bits
        uint32_t stops = 0;
        int q0 = 0;
        for (; q0 + 4 <= G; q0 += 4) {
            double u[4];
#pragma unroll
            for (int q = 0; q < 4; q++) u[q] = ubuf[rbase + q0 + q];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const double pq = prod * u[q];
                const bool cont = pq > en;
                prod = cont ? pq : 1.0;
                stops |= cont ? 0u : (1u << (q0 + q));
            }
        }
        if (q0 < G) {           // G = 4 m + 2: the last two
            double u[2];
#pragma unroll
            for (int q = 0; q < 2; q++) u[q] = ubuf[rbase + q0 + q];
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const double pq = prod * u[q];
                const bool cont = pq > en;
                prod = cont ? pq : 1.0;
                stops |= cont ? 0u : (1u << (q0 + q));
            }
        }
        // the draws, all at once: lane jl holds the round's stop at position jl
        // (if there is one), its rank among the round's stops and the stop
        // before it, so it writes that draw itself -- X + jl for the round's
        // first stop, the gap to the previous one otherwise -- while it is
        // among the `need` draws the chunk still wants
        const int need = live ? nd - j : 0;
        const uint32_t below = stops & ((1u << jl) - 1u);
        const int idx = __popc(below);
        const bool stop_here = ((stops >> jl) & 1u) != 0;
        if (stop_here && idx < need) {
            const int prev = below ? 31 - __builtin_clz(below) : -1;
            dcol[(j + idx) * WAVE + src] = (double)(prev < 0 ? X + jl : jl - prev - 1);
        }
        // the group's `need`-th stop, if this round reaches it: the uniforms
        // after it stay in the stream (the next chunk starts at the one after)
        const uint64_t fin = (uint64_t)__ballot(stop_here && idx == need - 1);
        const uint32_t gfin = (uint32_t)(fin >> gbase) & (uint32_t)((1ull << G) - 1ull);
        const int ns = __popc(stops);
        const int used = gfin ? __builtin_ctz(gfin) + 1 : G;
        if (live) {
            if (gfin) {             // the chunk's draws are done: the next starts fresh
                j = nd;
                X = 0;
                prod = 1.0;
            } else {
                j += ns;
                X = ns == 0 ? X + G : G - 1 - (31 - __builtin_clz(stops));
            }
        }
        wave_lds_sync();
        const uint64_t nh = shfl_u64(th, gbase + used - 1);
        const uint64_t nl = shfl_u64(tl, gbase + used - 1);
        if (live) {
            s.hi = nh;
            s.lo = nl;
        }
    }
    // the advanced generator back to its owner (group `rank` -> lane rank * G)
    const int back = (own && nd > 0) ? rank * G : lane;
    const uint64_t bh = shfl_u64(s.hi, back), bl = shfl_u64(s.lo, back);
    if (own && nd > 0) {
        g.hi = bh;
        g.lo = bl;
    }
    return true;
}

// K-step lock-step rollout (invsim_rollout without a policy, NEXT_STEP or
// DISABLED autoreset, compile-time lead time LT > 0), one 192-thread workgroup
// per 64 envs:
//   wave 0 (PTRS stream)  draws the demands (newsvendor.py:146) of the envs whose
//   wave 1 (mult stream)  rate takes numpy's PTRS branch (lam >= 10, or 0) /
//                         multiplication branch (0 < lam < 10) for the next chunk
//                         of launch steps into a three-chunk LDS ring, with
//                         the episode's Poisson constants in registers.  A lane
//                         works through its chunk's draws without waiting for
//                         the other lanes' rejections (one flat loop; a PTRS
//                         lane done early runs ahead into the next chunk).  The
//                         branch owning an env's generator runs its reset draws
//                         (5 uniforms -> price, cost, h, k, mu, :100-123) and
//                         hands params and generator state over in LDS; the
//                         branch of the new rate owns it next.
//   wave 2 (dynamics)     the step (:125-204) with the pipeline in registers;
//                         its action is loaded a step ahead, before the previous
//                         step's stores (vmcnt is in order).
// A chunk carries at most one reset (its last step).  Handoff: the stream waves
// fill buffer c % 3, barrier c, the dynamics wave consumes chunk c after
// barrier c (the reset rows and the dynamics -> obs rows alternate over two
// buffers).  Same draws, same order, same arithmetic as nv_run_kernel.
template <int LT>
#ifndef NV_ROLL_CH
#define NV_ROLL_CH 6
#endif
struct NvRoll {
    static constexpr int CH = NV_ROLL_CH;
    static constexpr int O = LT + 5;
    static constexpr int NP = 7;   // reset handoff: price, cost, h, k, mu, state hi, state lo
    static constexpr size_t tile_bytes() { return (size_t)((EPW * O + 3) / 4) * 4 * sizeof(float); }
    // tile, loggam table, demand chunks, reset handoff, mult uniforms, jump table,
    // fast-stream task table, then the dynamics -> obs handoff: the new order
    // hq [2][CH][WAVE] f32, the reward hr [2][CH][WAVE] f64, a reset's params
    // hp [2][5][WAVE] f32
    static constexpr size_t lds() {
        return tile_bytes() + RHS_LDS_MAX * sizeof(double) + 3 * (size_t)CH * WAVE * sizeof(double) +
               2 * NP * (size_t)WAVE * sizeof(double) + (size_t)WAVE * sizeof(double) +
               4 * (JUMP_MAX + 1) * sizeof(uint64_t) + 2 * 2 * (size_t)WAVE * sizeof(uint64_t) +
               2 * (size_t)CH * WAVE * (sizeof(float) + sizeof(double)) + 2 * 5 * (size_t)WAVE * sizeof(float);
    }
};

// The two stream waves of nv_roll_kernel on the fast stream.  A draw is a
// function of (key, launch step, mu) only -- no generator state, no order
// between draws -- so the waves split the chunk's draws instead of the sampler
// branches: wave `role` draws launch steps j = role, role + 2, ... of its
// lane's env when that env is on numpy's PTRS branch (one Philox block per
// candidate: U and V are its two 53-bit halves, as PhiloxGen hands them out),
// and the chunk's multiplication-branch draws (0 < mu < 10: few envs) are
// spread over both waves' lanes as (env, step) tasks.  The reset (5 uniforms
// of the reset step's own counter block, :100-123) is wave 0's; its params go
// to the other waves through the reset handoff rows of pbuf.  Same draws as
// nv_run_kernel<..., PhiloxGen> (test_fast_stream_newsvendor_fused_kernels_...).
template <int LT>
__device__ __forceinline__ void nv_stream_ph(const NvParams &P, int role, int lane, int64_t e, int64_t el, bool valid,
                                             int t_start, int K, bool nxt, double *lg_l, double *dbuf,
                                             double *pbuf, uint64_t *kb) {
    constexpr int CH = NvRoll<LT>::CH, NP = NvRoll<LT>::NP;
    const int64_t S = P.cm.Npad;
    {   // both waves draw PTRS candidates: each writes the whole (identical) table
        TableStage ts;
        ts.dst = lg_l;
        ts.load(P.lgtab, RHS_LDS_MAX, lane);
        ts.flush(lane);
    }
    NvState<LT, PhiloxGen> st;
    P.cm.rng.load(el, st.g);
    const uint2 key = st.g.key;
    PtrsConst c = nv_rate_const(P.par[4 * S + el]);
    uint64_t *kw = kb + role * 2 * WAVE;   // this wave's task table: keys [WAVE], exp(-mu) bits [WAVE]
    bool reset_any = false;
    int t = t_start, cb = 0, c3 = 0;
    for (int k0 = 0; k0 < K;) {
        int len;
        bool rs;
        nv_chunk(t, K - k0, P.step_limit, nxt, NvRoll<LT>::CH, len, rs);
        const int nd = len - (rs ? 1 : 0);                   // the reset step draws none
        double *dcol = dbuf + c3 * CH * WAVE;
        const uint64_t ph0 = P.cm.ph_step + (uint64_t)k0;    // launch step of the chunk's first step
#if defined(INVSIM_ABL_ROLL_NO_DRAW)
        for (int j = role; j < nd; j += 2) dcol[j * WAVE + lane] = 20;
#else
        if (c.lam >= 10) {   // numpy random_poisson_ptrs, one candidate per iteration, lanes independent
            uint32_t cj = 0;                                  // candidate = counter block of the draw
            for (int j = role; j < nd;) {
                const uint64_t stp = ph0 + (uint64_t)j;
                PhiloxBlock b;
                const uint4 x = b.block(make_uint4(cj, 0u, (uint32_t)stp, (uint32_t)(stp >> 32)), key);
                const double U = (double)((((uint64_t)x.y << 32) | x.x) >> 11) * (1.0 / 9007199254740992.0) - 0.5;
                const double V = (double)((((uint64_t)x.w << 32) | x.z) >> 11) * (1.0 / 9007199254740992.0);
                const double us = 0.5 - fabs(U);
                const int64_t kd = (int64_t)floor((c.a2 / us + c.b) * U + c.lam + 0.43);
                bool acc = (us >= 0.07) && (V <= c.vr);
                if (!acc && !((kd < 0) || ((us < 0.013) && (V > us)))) {
                    const double r = (kd < RHS_LDS_MAX)
                                         ? (-c.lam + (double)kd * c.loglam) - lg_l[kd < RHS_LDS_MAX ? kd : 0]
                                         : -c.lam + (double)kd * c.loglam - np_loggam((double)(kd + 1));
                    acc = ptrs_log_accept(c, V, us, r);
                }
                if (acc) {
                    dcol[j * WAVE + lane] = (double)kd;   // exact: kd is the floor of a double
                    j += 2;
                    cj = 0;
                } else {
                    cj++;
                }
            }
        } else if (c.lam == 0) {
            for (int j = role; j < nd; j += 2) dcol[j * WAVE + lane] = 0;
        }
        {   // numpy random_poisson_mult (0 < mu < 10, or NaN): task q = (env rank q / nd, step q % nd)
            const uint64_t mm = (uint64_t)__ballot(nv_mult_branch(c.lam) && nd > 0);
            const int nm = __popcll(mm);
            if (nm > 0) {
                kw[lane] = ((uint64_t)key.y << 32) | key.x;
                kw[WAVE + lane] = (uint64_t)__double_as_longlong(c.enlam);
                wave_lds_sync();
                // a divergent loop: keys and rates of other lanes come through LDS
                for (int q = lane + role * WAVE; q < nm * nd; q += 2 * WAVE) {
                    const int r = q / nd, j = q - r * nd;
                    uint64_t m = mm;
                    for (int i = 0; i < r; i++) m &= m - 1;   // the r-th mult env's lane
                    const int src = (int)__builtin_ctzll(m);
                    PhiloxGen g;
                    const uint64_t kk = kw[src];
                    g.key = make_uint2((uint32_t)kk, (uint32_t)(kk >> 32));
                    g.set_step(ph0 + (uint64_t)j);
                    g.sub(0);
                    dcol[j * WAVE + src] = (double)np_poisson_mult(g, __longlong_as_double((long long)kw[WAVE + src]));
                }
                wave_lds_sync();
            }
        }
#endif
        double *pb = pbuf + cb * NP * WAVE + lane;
        if (rs && role == 0) {                                // reset() at launch step k0 + len - 1
            st.g.set_step(ph0 + (uint64_t)(len - 1));
            nv_reset_regs<LT>(P, e, st, nullptr, false);
#pragma unroll
            for (int j = 0; j < 5; j++) pb[j * WAVE] = st.par[j];
        }
        nv_wg_sync();   // barrier: chunk ready
        if (rs) {
#pragma unroll
            for (int j = 0; j < 5; j++) st.par[j] = pb[j * WAVE];
            c = nv_rate_const(st.par[4]);
            reset_any = true;
            t = 0;
        } else {
            t += len;
        }
        k0 += len;
        cb ^= 1;
        c3 = c3 == 2 ? 0 : c3 + 1;
    }
    nv_wg_sync();   // barrier nch: the obs wave's last chunk
    if (valid && reset_any && role == 0) {
#pragma unroll
        for (int j = 0; j < 5; j++) P.par[j * S + e] = st.par[j];
    }
}

// POL (invsim_rollout_policy): the dynamics wave asks the agent for each
// step's order (OrderUpTo / ClassicNV / (s, S) / Constant, as nv_run_kernel)
// instead of loading it; every output optional, the per-env sums in registers.
// RG = PhiloxGen (the fast stream, newsvendor_ph.hip): the stream waves run
// nv_stream_ph instead (above); the dynamics and obs waves are the same.
//
// Round 4: four waves per 64 envs.  A wave issues at most about one
// instruction every 9 cycles, and a SIMD about one every 3 with four or more
// waves (tools/valu_rates, profiles/r04/launch/valu_rates.txt), so a step whose
// instructions all sit on one wave runs at that wave's issue rate while the
// SIMD idles.  The step therefore splits over two waves:
//   wave 2 (dynamics) the step's state and reward (:125-170) with the pipeline
//                     in registers; it hands the new order q and the reward to
//                     wave 3 in LDS (hq, hr; a reset's params in hp) and writes
//                     no global memory in its loop (the ring slots once, at the
//                     end), so the action it loads a step ahead waits for
//                     nothing but itself
//   wave 3 (obs)      keeps its own copy of the pipeline from the handed-over
//                     orders, writes the tile row, stores the tile, reward and
//                     flags, one chunk behind the dynamics wave
// Chunk c: the stream waves fill it before barrier c, the dynamics wave
// consumes it between barriers c and c + 1, the obs wave between c + 1 and
// c + 2 (every wave passes nch + 1 barriers).
//
// Measured and not kept in round 4 (profiles/r04/pair_ab, layout_ab): the
// PTRS role on lane PAIRS (a PTRS candidate always consumes two uniforms and
// its acceptance depends only on them and the rate, so the two lanes of a pair
// can evaluate candidates n and n + 1 at once, lane 1 jumping two LCG steps
// ahead, and take the accepted ones in stream order -- numpy's draws, half the
// trips per chunk).  As a fifth wave (commit 05546b1) the grid no longer fits
// at once (<= 96 VGPRs, uneven placement of the fifth wave): 29.0 -> 20.4 G.
// As two pair waves with the multiplication draws moved into the obs wave
// (commit b4c9eaf) the obs wave became the tail: 29.3 -> 26.0 G.  Software-
// pipelining the PTRS wave's trips (the next candidate's uniforms drawn while
// the pending one is tested, commit 3513fd2) measured no faster (28.9 against
// 29.1-29.4 G): the trip is not bound by the generator's multiply chain.
#define NV_ROLL_WAVES 4
#define NV_ROLL_BOUNDS __launch_bounds__(4 * WAVE) __attribute__((amdgpu_waves_per_eu(4)))   // <= 128 VGPRs: the grid resident

template <int LT, bool POL, class RG = Pcg>
__global__ void NV_ROLL_BOUNDS
nv_roll_kernel(NvParams P, int t_start, StepIO<float, float> io, PolicyIO pol) {
    using R = NvRoll<LT>;
    constexpr int O = R::O, CH = R::CH, NP = R::NP;
    constexpr int TILE_IT = (EPW * O * 4 + 16 * WAVE - 1) / (16 * WAVE);
    extern __shared__ __attribute__((aligned(16))) float nr_lds[];
    float *tile = nr_lds;
    double *lg_l = reinterpret_cast<double *>(nr_lds + R::tile_bytes() / sizeof(float));
    // [2][CH][WAVE] demands as doubles: a PTRS draw is the floor value of a
    // double (numpy's k = (int64)kd), so the stream wave stores kd as it is and
    // the dynamics wave converts, off the PTRS wave's per-candidate path
    double *dbuf = lg_l + RHS_LDS_MAX;
    double *pbuf = reinterpret_cast<double *>(dbuf + 3 * CH * WAVE);      // [2][NP][WAVE]
    double *ubuf = pbuf + 2 * NP * WAVE;                                   // [WAVE] mult wave's uniforms
    uint64_t *jt = reinterpret_cast<uint64_t *>(ubuf + WAVE);              // [4][JUMP_MAX + 1] jump table
    uint64_t *kb = jt + 4 * (JUMP_MAX + 1);                                // [2][2][WAVE] fast stream: keys, rates
    double *hr = reinterpret_cast<double *>(kb + 2 * 2 * WAVE);            // [2][CH][WAVE] rewards
    float *hq = reinterpret_cast<float *>(hr + 2 * CH * WAVE);             // [2][CH][WAVE] new orders
    float *hp = hq + 2 * CH * WAVE;                                        // [2][5][WAVE] a reset's params
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
    const bool nxt = P.cm.autoreset == AR_NEXT_STEP;
    if constexpr (RG::kCounter) {
        if (role < 2) {   // ---- the fast stream's two stream waves
            nv_stream_ph<LT>(P, role, lane, e, el, valid, t_start, K, nxt, lg_l, dbuf, pbuf, kb);
            return;
        }
    }
    TPROBE_W(0);
    TPROBE_W_ID();
    if constexpr (!RG::kCounter) if (role < 2) {   // ---- stream waves
        const bool multw = role == 1;
        TableStage ts;
        if (!multw) {
            ts.dst = lg_l;
            ts.load(P.lgtab, RHS_LDS_MAX, lane);
        } else {
            const uint64_t *jsrc = &c_jump.a_hi[0];   // the four rows are contiguous
            for (int q = lane; q < 4 * (JUMP_MAX + 1); q += WAVE) jt[q] = jsrc[q];
        }
        NvState<LT> st;
        st.g = P.cm.rng.load(el);
        PtrsConst c = nv_rate_const(P.par[4 * S + el]);
        bool mine = nv_mult_branch(c.lam) == multw;
        if (!multw) ts.flush(lane);
        bool reset_any = false;
        int t = t_start, cb = 0, c3 = 0;
        int carry = 0;   // PTRS lanes: draws of this chunk already made during the previous one
        int ci = 0;
        (void)ci;
        TPROBE_W(1);
        for (int k0 = 0; k0 < K;) {
            int len;
            bool rs;
            nv_chunk(t, K - k0, P.step_limit, nxt, CH, len, rs);
            const int nd = mine ? len - (rs ? 1 : 0) : 0;    // draws of this env (the reset step draws none)
            const int c3n = c3 == 2 ? 0 : c3 + 1;
            double *db = dbuf + c3 * CH * WAVE + lane;
#if defined(INVSIM_ABL_ROLL_NO_DRAW)
            for (int j = 0; j < nd; j++) db[j * WAVE] = 20;
#else
#if defined(INVSIM_ABL_ROLL_NO_MULT) || defined(INVSIM_ABL_ROLL_NO_PTRS)
#ifdef INVSIM_ABL_ROLL_NO_MULT
            if (multw) {
#else
            if (!multw) {
#endif
                for (int j = 0; j < nd; j++) db[j * WAVE] = 5;
            } else
#endif
            if (!multw) {
                if (c.lam == 0) {
                    for (int j = 0; j < nd; j++) db[j * WAVE] = 0;
                } else {
                    // numpy random_poisson_ptrs, one trial per iteration, lanes
                    // independent.  Run-ahead: a lane done with this chunk goes on
                    // with the next chunk's draws (into its ring buffer, which no
                    // wave reads before barrier c + 1) while the others finish,
                    // unless this chunk ends with a reset or is the launch's last;
                    // the wave then pays the max over lanes of the whole launch's
                    // trips, not the sum over chunks of each chunk's max.
                    int nd2 = 0;
                    if (!rs && k0 + len < K) {
                        int len2;
                        bool rs2;
                        nv_chunk(t + len, K - k0 - len, P.step_limit, nxt, CH, len2, rs2);
                        nd2 = mine ? len2 - (rs2 ? 1 : 0) : 0;
                    }
                    const int lim = nd + nd2;
                    double *db2 = dbuf + c3n * CH * WAVE + lane - nd * WAVE;   // draw j >= nd -> next chunk's j - nd
#ifdef INVSIM_TIMING
                    uint32_t trips = 0;
#endif
                    int j = carry;
                    while (__ballot(j < nd)) {
#ifdef INVSIM_TIMING
                        trips++;
#endif
                        if (j >= lim) continue;
                        const double U = st.g.next_double() - 0.5;
                        const double V = st.g.next_double();
                        double kd;
#if INVSIM_PTRS_DECIDE
                        const LgTab src{lg_l};
                        const bool acc = ptrs_decide_d(
                            c, U, V, [&](double kd, bool &ok) { return src.fastd(kd, c, ok); },
                            [&](int64_t kk) { return src.exact(kk, c); }, kd);
#else
                        const double us = 0.5 - fabs(U);
                        const int64_t ki = (int64_t)floor((c.a2 / us + c.b) * U + c.lam + 0.43);
                        kd = (double)ki;
                        bool acc = (us >= 0.07) && (V <= c.vr);
                        if (!acc && !((ki < 0) || ((us < 0.013) && (V > us)))) {
                            const double r = (ki < RHS_LDS_MAX)
                                                 ? (-c.lam + (double)ki * c.loglam) - lg_l[ki < RHS_LDS_MAX ? ki : 0]
                                                 : -c.lam + (double)ki * c.loglam - np_loggam((double)(ki + 1));
                            acc = ptrs_log_accept(c, V, us, r);
                        }
#endif
                        if (acc) {
                            (j < nd ? db : db2)[j * WAVE] = kd;
                            j++;
                        }
                    }
                    carry = j - nd;
#ifdef INVSIM_TIMING
                    TTRIP_ADD(wave_max_u32(trips));
#endif
                }
            } else if (!nv_mult_chunk_grp(st.g, c.enlam, mine, len - (rs ? 1 : 0), dbuf + c3 * CH * WAVE, ubuf, jt, lane)) {
                // more than 16 envs on this branch: numpy random_poisson_mult, one
                // uniform per iteration, lanes independent
                int64_t X = 0;
                double prod = 1.0;
                for (int j = 0; j < nd;) {
                    prod *= st.g.next_double();
                    if (prod > c.enlam) {
                        X += 1;
                    } else {
                        db[j * WAVE] = (double)X;
                        j++;
                        X = 0;
                        prod = 1.0;
                    }
                }
            }
#endif
            double *pb = pbuf + cb * NP * WAVE + lane;
#ifdef INVSIM_TIMING
            if (ci < 4) TPROBE_W(2 + ci);
            ci++;
#endif
            if (rs && mine) {                      // reset() of the owner: 5 uniforms (:105-111)
                nv_reset_regs<LT>(P, e, st, nullptr, false);
#pragma unroll
                for (int j = 0; j < 5; j++) pb[j * WAVE] = st.par[j];
                pb[5 * WAVE] = __longlong_as_double((long long)st.g.hi);
                pb[6 * WAVE] = __longlong_as_double((long long)st.g.lo);
            }
            nv_wg_sync();   // barrier: chunk ready
            if (rs) {                              // the new episode's branch owns the generator
#pragma unroll
                for (int j = 0; j < 5; j++) st.par[j] = pb[j * WAVE];
                st.g.hi = (uint64_t)__double_as_longlong(pb[5 * WAVE]);
                st.g.lo = (uint64_t)__double_as_longlong(pb[6 * WAVE]);
                c = nv_rate_const(st.par[4]);
                mine = nv_mult_branch(c.lam) == multw;
                reset_any = true;
                t = 0;
            } else {
                t += len;
            }
            k0 += len;
            cb ^= 1;
            c3 = c3n;
        }
        nv_wg_sync();   // barrier nch: the obs wave's last chunk
        if (valid) {
            if (mine) P.cm.rng.store_state(e, st.g);
            if (reset_any && !multw) {
#pragma unroll
                for (int j = 0; j < 5; j++) P.par[j * S + e] = st.par[j];
            }
        }
        TWAIT();
        TPROBE_W(6);
        return;
    }
    if (role == 3) {   // ---- obs wave
        float *trow = tile + lane * O;
        int sc = t_start;
        float pf[5], pv[LT];
#pragma unroll
        for (int j = 0; j < 5; j++) pf[j] = (float)P.par[j * S + el];
        {
            const int base = (int)((uint32_t)(sc + 1) % (uint32_t)LT);
#pragma unroll
            for (int p = 0; p < LT; p++) {
                int sl = base + p;
                sl = sl >= LT ? sl - LT : sl;
                pv[p] = P.pipe[(int64_t)sl * S + el];
                if (!(p >= LT - sc)) pv[p] = 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < 5; j++) trow[j] = pf[j];   // the params part changes only at a reset
        // the observation, reward and flags of launch step k (step kk of the chunk
        // in handoff buffer cb); returns whether it was a reset step
        auto obs_step = [&](int k, int kk, int cb) -> bool {
            const int64_t oi = (int64_t)k * N + e;
            const bool rs = nxt && sc >= P.step_limit;
            double r = 0.0;
            bool tr = false;
            if (rs) {                                              // NEXT_STEP autoreset: the new params, empty pipeline
#pragma unroll
                for (int j = 0; j < 5; j++) {
                    pf[j] = hp[(cb * 5 + j) * WAVE + lane];
                    trow[j] = pf[j];
                }
#pragma unroll
                for (int p = 0; p < LT; p++) pv[p] = 0.f;
                sc = 0;
            } else {
                const float q = hq[(cb * CH + kk) * WAVE + lane];
                r = hr[(cb * CH + kk) * WAVE + lane];
#pragma unroll
                for (int p = 0; p + 1 < LT; p++) pv[p] = pv[p + 1];
                pv[LT - 1] = q;
                tr = sc + 1 >= P.step_limit;                       // :190
                sc += 1;
            }
#pragma unroll
            for (int p = 0; p < LT; p++) trow[5 + p] = pv[p];      // obs after :183
            if (valid && (!POL || io.rew)) {
                out_store(io.rew + oi, r);
                out_store(io.term + oi, (uint8_t)0);
                out_store(io.trunc + oi, (uint8_t)(tr ? 1 : 0));
            }
            wave_lds_sync();
#ifndef INVSIM_ABL_ROLL_NO_STORE
            if (!POL || io.obs) store_tile<TILE_IT>(tile, io.obs + ((int64_t)k * N + e0) * O, (int64_t)nvalid * O, lane);
#endif
            wave_lds_sync();
            return rs;
        };
        int kk = 0, cb = 0;
        nv_wg_sync();   // barrier 0
        nv_wg_sync();   // barrier 1: chunk 0 handed over
        TPROBE_W(1);
        int ci = 0;
        (void)ci;
        for (int k = 0; k < K; k++) {
            const bool rs = obs_step(k, kk, cb);
            if (++kk == CH || rs || k == K - 1) {      // chunk consumed
#ifdef INVSIM_TIMING
                if (ci < 4) TPROBE_W(2 + ci);
                ci++;
#endif
                if (k + 1 < K) nv_wg_sync();             // barrier of the next chunk's handoff
                kk = 0;
                cb ^= 1;
            }
        }
        TWAIT();
        TPROBE_W(6);
        return;
    }
    // ---- dynamics wave
    NvState<LT> st;
    int sc = t_start;
#pragma unroll
    for (int j = 0; j < 5; j++) st.par[j] = P.par[j * S + el];
    {
        const int base = (int)((uint32_t)(sc + 1) % (uint32_t)LT);
#pragma unroll
        for (int p = 0; p < LT; p++) {
            int sl = base + p;
            sl = sl >= LT ? sl - LT : sl;
            st.pv[p] = P.pipe[(int64_t)sl * S + el];
            if (!(p >= LT - sc)) st.pv[p] = 0.f;
        }
    }
    float nact = POL ? 0.f : io.act[el];
    constexpr int MD = 2;                       // metrics: reward sum, steps
    double met[MD];
#pragma unroll
    for (int q = 0; q < MD; q++) met[q] = (POL && pol.metrics) ? pol.metrics[el * MD + q] : 0.0;
    double lvl = 0.0;     // CLASSIC_NV / SS: the episode's ppf level, once computed
    bool have = false;
    int64_t dlast = -1;   // the last step's demand (the info record), -1: a reset step
    int kk = 0, cb = 0, c3 = 0;
    int ci = 0;
    (void)ci;
    nv_wg_sync();   // barrier 0: chunk 0 ready
    TPROBE_W(1);
    for (int k = 0; k < K; k++) {
        const int64_t oi = (int64_t)k * N + e;
        float act = nact;
        if (!POL && k + 1 < K) nact = io.act[(int64_t)(k + 1) * N + el];   // the next step's action
        const bool rs = nxt && sc >= P.step_limit;
        if (rs) {                                                  // NEXT_STEP autoreset
            if (valid) {   // the ending episode's ring slots, as its per-step slot writes leave them
                const int base = (int)((uint32_t)(sc + 1) % (uint32_t)LT);
#pragma unroll
                for (int p = 0; p < LT; p++) {
                    int sl = base + p;
                    sl = sl >= LT ? sl - LT : sl;
                    if (p >= LT - sc) P.pipe[(int64_t)sl * S + e] = st.pv[p];
                }
            }
#pragma unroll
            for (int j = 0; j < 5; j++) {
                st.par[j] = pbuf[(cb * NP + j) * WAVE + lane];
                hp[(cb * 5 + j) * WAVE + lane] = (float)st.par[j];   // -> obs wave
            }
#pragma unroll
            for (int p = 0; p < LT; p++) st.pv[p] = 0.f;
            have = false;
            sc = 0;
            dlast = -1;
        } else {
            if (POL) {
                if (pol.kind == POL_ORDER_UP_TO) act = nv_order_up_to<LT>(P, pol, e, sc, st);
                else if (pol.kind == POL_CLASSIC_NV) act = nv_classic<LT>(P, pol, e, sc, st, lvl, have);
                else if (pol.kind == POL_SS) act = nv_ss<LT>(P, pol, e, sc, st, lvl, have);
                else act = pol.cf[0];
                if (valid && pol.act_out) out_store((float *)pol.act_out + oi, act);
            }
            const int64_t d = (int64_t)dbuf[(c3 * CH + kk) * WAVE + lane];
            double r;
            nv_step_regs<LT>(P, e, valid, sc, st, act, nullptr, lg_l, nullptr, r, nullptr, d,
                             (valid && k == K - 1) ? (double *)P.cm.info_rec : nullptr, false);
            if (POL) {
                met[0] += r;                    // episode_reward += reward (benchmark_newsvendor.py:241)
                met[1] += 1.0;
            }
            hq[(cb * CH + kk) * WAVE + lane] = st.pv[LT - 1];     // the new order -> obs wave
            hr[(cb * CH + kk) * WAVE + lane] = r;
            dlast = d;
            sc += 1;
        }
        if (++kk == CH || rs || k == K - 1) {      // chunk consumed
#ifdef INVSIM_TIMING
            if (ci < 4) TPROBE_W(2 + ci);
            ci++;
#endif
            nv_wg_sync();                            // barrier of the next chunk (after the last: the obs wave's)
            kk = 0;
            cb ^= 1;
            c3 = c3 == 2 ? 0 : c3 + 1;
        }
    }
    if (valid) {
        // the ring slots of the final pipeline: the positions this episode has
        // ordered (p >= LT - sc; the others are masked at load and keep the
        // bytes the per-step slot writes of the other kernels leave there)
        const int base = (int)((uint32_t)(sc + 1) % (uint32_t)LT);
#pragma unroll
        for (int p = 0; p < LT; p++) {
            int sl = base + p;
            sl = sl >= LT ? sl - LT : sl;
            if (p >= LT - sc) P.pipe[(int64_t)sl * S + e] = st.pv[p];
        }
        if (P.cm.info_demand && dlast >= 0) P.cm.info_demand[e] = dlast;
        if (POL && pol.metrics) {
#pragma unroll
            for (int q = 0; q < MD; q++) pol.metrics[e * MD + q] = met[q];
        }
    }
    TWAIT();
    TPROBE_W(6);
}

// cm.rng <- the committed slot of the lookahead cache
__global__ void __launch_bounds__(256) nv_commit_kernel(NvParams P, int slot) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    const int64_t S = P.cm.Npad;
    const uint64_t *A = P.ahead + (int64_t)slot * 3 * S;
    P.cm.rng.hi[e] = A[e];
    P.cm.rng.lo[e] = A[S + e];
}

__global__ void __launch_bounds__(256)
nv_reset_kernel(NvParams P, const uint8_t *__restrict__ mask, float *__restrict__ obs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.cm.N) return;
    if (mask && !mask[e]) return;
    float *orow = obs ? obs + e * (P.L + 5) : nullptr;
    if (P.cm.philox) {
        NvState<-1, PhiloxGen> st;
        P.cm.rng.load(e, st.g);
        st.g.set_step(P.cm.ph_step);
        nv_reset_regs<-1>(P, e, st, orow, true);
    } else {
        NvState<-1> st;
        st.g = P.cm.rng.load(e);
        nv_reset_regs<-1>(P, e, st, orow, true);
        P.cm.rng.store_state(e, st.g);
    }
    P.cm.period[e] = 0;
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

#define NV_LT_SWITCH(L_)              \
    switch (p.L) {                    \
        case 0: L_(0); break;         \
        case 1: L_(1); break;         \
        case 2: L_(2); break;         \
        case 3: L_(3); break;         \
        case 4: L_(4); break;         \
        case 5: L_(5); break;         \
        case 6: L_(6); break;         \
        case 7: L_(7); break;         \
        case 8: L_(8); break;         \
        case 9: L_(9); break;         \
        case 10: L_(10); break;       \
        case 12: L_(12); break;       \
        case 16: L_(16); break;       \
        default: L_(-1); break;       \
    }

// The step / rollout dispatch of one demand stream: RG = Pcg (numpy's PCG64,
// parity) or PhiloxGen (the fast stream; instantiated in newsvendor_ph.hip).
// The fast stream's lookahead cache holds demands only: it is never committed,
// and any other launch leaves it stale (the launch-step counter moves past it).
template <class RG>
hipError_t nv_launch_rg(const NvParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                        bool &ahead, int &slot, hipStream_t s) {
    constexpr bool ph = RG::kCounter;
    const size_t lds = (size_t)((EPW * (p.L + 5) + 3) / 4) * 4 * sizeof(float) + RHS_LDS_MAX * sizeof(double);
    const dim3 grid(grid_for(p.cm.N, EPW)), block(WAVE);
    PolicyIO none{};
    const PolicyIO &pv = pol ? *pol : none;
    const bool la = p.ahead && p.cm.kn.nv_ahead;
    if (la && !pol && io.K == 1 && t_u >= 0 && t_u < p.step_limit && io.obs &&
        !(p.cm.autoreset == AR_SAME_STEP && t_u + 1 >= p.step_limit)) {
        const bool produce = t_u + 1 < p.step_limit;
        if (ahead || produce) {
            const bool hit = ahead;
            // lookahead workgroups: two per 64 envs (one per sampler branch) to
            // draw, one to commit the parity stream's state when the chain ends
            const int gla = hit ? (produce ? 2 : (ph ? 0 : 1)) * (int)grid_for(p.cm.N, WAVE) : 0;
            const dim3 grid2(grid.x + gla);
            const int cur = slot;
            const int xp = p.cm.kn.nv_xcd ? 1 : 0;
#define S_(X)                                                                                                \
    do {                                                                                                     \
        if (hit && produce) hipLaunchKernelGGL((nv_step1_kernel<X, true, true, RG>), grid2, block, lds, s, p, t_u, io, cur, gla, xp);  \
        else if (hit) hipLaunchKernelGGL((nv_step1_kernel<X, true, false, RG>), grid2, block, lds, s, p, t_u, io, cur, gla, xp);       \
        else hipLaunchKernelGGL((nv_step1_kernel<X, false, true, RG>), grid2, block, lds, s, p, t_u, io, cur, gla, xp);                \
    } while (0)
            NV_LT_SWITCH(S_)
#undef S_
            if (produce) {
                ahead = true;
                slot ^= 1;
            } else {
                ahead = false;   // cm.rng committed by the lookahead workgroups
            }
            return hipGetLastError();
        }
    }
    if (ahead) {   // the one-wave kernel reads cm.rng: commit, the cache ends
        const hipError_t ce = ph ? hipSuccess : nv_commit_launch(p, slot, s);
        ahead = false;
        if (ce != hipSuccess) return ce;
    }
    if ((!pol || p.cm.kn.nv_pol_roll) && io.K > 1 && t_u >= 0 && p.L > 0 &&
        p.cm.autoreset != AR_SAME_STEP && p.cm.kn.nv_roll) {
        const dim3 gr(grid_for(p.cm.N, WAVE)), br(NV_ROLL_WAVES * WAVE);
        bool done = true;
#define R_(X)                                                                                              \
    do {                                                                                                   \
        if (X > 0) {                                                                                       \
            if (pol) hipLaunchKernelGGL((nv_roll_kernel<(X > 0 ? X : 1), true, RG>), gr, br, NvRoll<(X > 0 ? X : 1)>::lds(), s, p, t_u, io, pv); \
            else hipLaunchKernelGGL((nv_roll_kernel<(X > 0 ? X : 1), false, RG>), gr, br, NvRoll<(X > 0 ? X : 1)>::lds(), s, p, t_u, io, pv); \
        } else done = false;                                                                               \
    } while (0)
        NV_LT_SWITCH(R_)
#undef R_
        if (done) return hipGetLastError();
    }
#define K_(X, TU, ONE, POL) hipLaunchKernelGGL((nv_run_kernel<X, TU, ONE, POL, RG>), grid, block, lds, s, p, t_u, io, pv)
#define L_(X)                                          \
    do {                                               \
        if (pol) {                                     \
            if (t_u >= 0) K_(X, true, false, true);    \
            else K_(X, false, false, true);            \
        } else if (io.K == 1) {                        \
            if (t_u >= 0) K_(X, true, true, false);    \
            else K_(X, false, true, false);            \
        } else {                                       \
            if (t_u >= 0) K_(X, true, false, false);   \
            else K_(X, false, false, false);           \
        }                                              \
    } while (0)
    NV_LT_SWITCH(L_)
#undef L_
#undef K_
    return hipGetLastError();
}

}  // namespace

#ifdef INVSIM_NV_FAST_TU
// newsvendor_ph.hip: this file compiled a second time for the fast-stream
// kernels (a TU of their own, so the two instantiation sets compile in parallel)
hipError_t nv_run_launch_ph(const NvParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                            bool &ahead, int &slot, hipStream_t s) {
    if (p.cm.N == 0 || io.K <= 0) return hipSuccess;
    return nv_launch_rg<PhiloxGen>(p, t_u, pol, io, ahead, slot, s);
}

INVSIM_PTRS_STATS_TU(nv_ph)
#else
hipError_t nv_commit_launch(const NvParams &p, int slot, hipStream_t s) {
    if (p.cm.N == 0 || !p.ahead) return hipSuccess;
    hipLaunchKernelGGL(nv_commit_kernel, dim3(grid_for(p.cm.N, 256)), dim3(256), 0, s, p, slot ^ 1);
    return hipGetLastError();
}

hipError_t nv_run_launch(const NvParams &p, int t_u, const PolicyIO *pol, const StepIO<float, float> &io,
                         bool &ahead, int &slot, hipStream_t s) {
    if (p.cm.N == 0 || io.K <= 0) return hipSuccess;
    if (p.cm.philox) return nv_run_launch_ph(p, t_u, pol, io, ahead, slot, s);   // newsvendor_ph.hip
    return nv_launch_rg<Pcg>(p, t_u, pol, io, ahead, slot, s);
}

hipError_t nv_reset_launch(const NvParams &p, const uint8_t *mask, float *obs, hipStream_t s) {
    if (p.cm.N == 0) return hipSuccess;
    hipLaunchKernelGGL(nv_reset_kernel, dim3(grid_for(p.cm.N, 256)), dim3(256), 0, s, p, mask, obs);
    return hipGetLastError();
}

INVSIM_PTRS_STATS_TU(nv)
#endif

}  // namespace invsim

#if defined(INVSIM_TIMING) && !defined(INVSIM_NV_FAST_TU)
extern "C" int invsim_debug_timing_nv(void *dst, int64_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(invsim::g_tbuf), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int invsim_debug_timing_bar_nv(void *dst, int64_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(invsim::g_tbar), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int invsim_debug_timing_trip_nv(void *dst, int64_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(invsim::g_ttrip), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
#endif
