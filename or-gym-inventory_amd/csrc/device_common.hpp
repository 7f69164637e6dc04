// Device-side building blocks shared by the three env kernels (gfx950).
//
//  * PCG64 (numpy's XSL-RR 128/64) with the 128-bit LCG step done as 64-bit
//    halves (__umul64hi) — one per env, state SoA in HBM.
//  * numpy SeedSequence(pool 4) -> PCG64 seeding, all 32-bit integer ops.
//  * numpy Generator.poisson (PTRS for lam >= 10, multiplication for lam < 10)
//    and random_loggam, restated from numpy 2.2.6 distributions.c (the
//    third-party code the reference calls: newsvendor.py:146,
//    inventory_management.py:172, network_management.py:125/263/540).
//  * numpy add.reduce pairwise order for small f32/f64 sums.
//
// Built with -ffp-contract=off: the reference never fuses multiply-adds, and
// Poisson acceptance tests must see the same roundings.
#pragma once
#include <hip/hip_runtime.h>
#include <rocrand/rocrand_philox4x32_10.h>
#include <stdint.h>

namespace invsim {

constexpr uint64_t PCG_MULT_HI = 0x2360ED051FC65DA4ULL;
constexpr uint64_t PCG_MULT_LO = 0x4385DF649FCCF645ULL;

struct Pcg {
    uint64_t hi, lo;          // 128-bit state
    uint64_t inc_hi, inc_lo;  // 128-bit increment (odd)

    __device__ __forceinline__ uint64_t next64() {
        // state = state * MULT + inc  (mod 2^128).  As one 128-bit multiply-add
        // the compiler emits six v_mad_u64_u32 + four v_mul_lo_u32 and an
        // add-with-carry chain for the increment: ~25 instructions against ~29
        // for the 64-bit-halves form (__umul64hi).  A lone stream wave issues one
        // instruction per ~9 cycles whatever its dependencies, so
        // the instruction count is the step's cost.
        typedef unsigned __int128 u128;
        u128 st = ((u128)hi << 64) | lo;
        st = st * (((u128)PCG_MULT_HI << 64) | PCG_MULT_LO) + (((u128)inc_hi << 64) | inc_lo);
        hi = (uint64_t)(st >> 64);
        lo = (uint64_t)st;
        uint64_t x = hi ^ lo;
        unsigned rot = (unsigned)(hi >> 58);
        return (x >> rot) | (x << ((64u - rot) & 63u));
    }
    __device__ __forceinline__ double next_double() {
        return (double)(next64() >> 11) * (1.0 / 9007199254740992.0);
    }
    // counter positioning of the fast stream (PhiloxGen): a sequential stream has none
    static constexpr bool kCounter = false;
    __device__ __forceinline__ void set_step(uint64_t) {}
    __device__ __forceinline__ void sub(uint32_t) {}
};

// ---------------------------------------------------------------- fast stream
// Opt-in, NON-parity demand stream (invsim_set_demand_stream):
// rocRAND's Philox4x32-10 block function used counter-based.  An env's key is
// its seeded PCG64 increment (high word: 64 bits of SeedSequence output), and
// the counter of draw block j of stream r (0 = demand / market r, RESET = the
// Newsvendor reset's uniforms) in launch step s of the handle is (j, r, s_lo,
// s_hi).  So a draw depends on (seed, step, r) only: no generator state is read
// or written per step, and no draw waits for the previous one.  The samplers
// (PTRS / multiplication / numpy_dists) are the parity ones, fed with 53-bit
// uniforms from the 128-bit blocks (two per block).
struct PhiloxBlock : rocrand_device::philox4x32_10_engine {
    __device__ __forceinline__ uint4 block(uint4 c, uint2 k) { return this->ten_rounds(c, k); }
};

struct PhiloxGen {
    static constexpr uint32_t RESET = 0xffffffffu;
    static constexpr bool kCounter = true;
    uint2 key;
    uint32_t s0 = 0, s1 = 0, r = 0, j = 0;
    uint64_t hold = 0;
    bool have = false;
    __device__ __forceinline__ void set_step(uint64_t s) {
        s0 = (uint32_t)s;
        s1 = (uint32_t)(s >> 32);
    }
    __device__ __forceinline__ void sub(uint32_t rr) {
        r = rr;
        j = 0;
        have = false;
    }
    __device__ __forceinline__ uint64_t next64() {
        if (have) {
            have = false;
            return hold;
        }
        PhiloxBlock b;
        const uint4 x = b.block(make_uint4(j, r, s0, s1), key);
        j++;
        hold = ((uint64_t)x.w << 32) | x.z;
        have = true;
        return ((uint64_t)x.y << 32) | x.x;
    }
    __device__ __forceinline__ double next_double() {
        return (double)(next64() >> 11) * (1.0 / 9007199254740992.0);
    }
};

// A stream wave's draw position (stream_flat_loop): the fast stream is put at
// draw r of launch step j before each attempt (a PTRS rejection continues the
// same (j, r) block sequence, as the run kernels' set_step + sub); a
// sequential stream simply continues.
template <class G>
struct StreamPos {
    uint64_t base;             // the handle's launch-step counter (Common::ph_step)
    int j = -1, r = -1;
    __device__ __forceinline__ explicit StreamPos(uint64_t b) : base(b) {}
    __device__ __forceinline__ void at(G &g, int jj, int rr) {
        if constexpr (G::kCounter) {
            if (jj != j || rr != r) {
                g.set_step(base + (uint64_t)jj);
                g.sub((uint32_t)rr);
                j = jj;
                r = rr;
            }
        }
    }
};

// ---------------------------------------------------------------- SeedSequence
__device__ __forceinline__ uint32_t ss_hashmix(uint32_t v, uint32_t &hc) {
    v ^= hc;
    hc *= 0x931e8875u;
    v *= hc;
    v ^= v >> 16;
    return v;
}
__device__ __forceinline__ uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
    r ^= r >> 16;
    return r;
}

// numpy SeedSequence(entropy words w[0..nw), nw <= 4).generate_state(4, uint64) -> PCG64 seed
__device__ inline void seed_pcg64(const uint32_t w[4], int nw, Pcg &g) {
    uint32_t pool[4];
    uint32_t hc = 0x43b0d7e5u;
#pragma unroll
    for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < nw ? w[i] : 0u, hc);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
    uint32_t out[8];
    uint32_t hb = 0x8b51f9ddu;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= 0x58f38dedu;
        v *= hb;
        v ^= v >> 16;
        out[i] = v;
    }
    uint64_t s_hi = (uint64_t)out[0] | ((uint64_t)out[1] << 32);
    uint64_t s_lo = (uint64_t)out[2] | ((uint64_t)out[3] << 32);
    uint64_t q_hi = (uint64_t)out[4] | ((uint64_t)out[5] << 32);
    uint64_t q_lo = (uint64_t)out[6] | ((uint64_t)out[7] << 32);
    // pcg_setseq_128_srandom_r: inc = (initseq << 1) | 1; state = 0; step; state += initstate; step
    g.inc_hi = (q_hi << 1) | (q_lo >> 63);
    g.inc_lo = (q_lo << 1) | 1ULL;
    g.hi = 0;
    g.lo = 0;
    (void)g.next64();
    uint64_t lo2 = g.lo + s_lo;
    g.hi = g.hi + s_hi + (lo2 < g.lo ? 1ULL : 0ULL);
    g.lo = lo2;
    (void)g.next64();
}

// ---------------------------------------------------------------- Poisson
// Constants of numpy random_poisson_ptrs that depend only on lam.  For a fixed
// lam they are computed on the HOST with the reference platform's libm
// (bit-identical to what numpy computes); for per-env lam (Newsvendor) on device.
struct PtrsConst {
    double lam, slam, loglam, b, a, invalpha, vr, log_invalpha, enlam;
    double a2;        // 2 * a  (numpy evaluates 2 * a / us as (2 * a) / us)
    int32_t k0, nk;   // host table of the PTRS right-hand side for k in [k0, k0 + nk)
    int32_t toff, pad_;  // that table's offset in the handle's RHS table array
};

__host__ __device__ inline PtrsConst ptrs_const(double lam) {
    PtrsConst c;
    c.lam = lam;
    c.slam = sqrt(lam);
    c.loglam = log(lam);
    c.b = 0.931 + 2.53 * c.slam;
    c.a = -0.059 + 0.02483 * c.b;
    c.invalpha = 1.1239 + 1.1328 / (c.b - 3.4);
    c.vr = 0.9277 - 3.6224 / (c.b - 2);
    c.log_invalpha = log(c.invalpha);
    c.enlam = exp(-lam);
    c.a2 = 2 * c.a;
    c.k0 = 0;
    c.nk = 0;
    return c;
}

__host__ __device__ inline double np_loggam(double x) {
    const double a0 = 8.333333333333333e-02, a1 = -2.777777777777778e-03,
                 a2 = 7.936507936507937e-04, a3 = -5.952380952380952e-04,
                 a4 = 8.417508417508418e-04, a5 = -1.917526917526918e-03,
                 a6 = 6.410256410256410e-03, a7 = -2.955065359477124e-02,
                 a8 = 1.796443723688307e-01, a9 = -1.39243221690590e+00;
    if (x == 1.0 || x == 2.0) return 0.0;
    int64_t n = (x < 7.0) ? (int64_t)(7 - x) : 0;
    double x0 = x + (double)n;
    double x2 = (1.0 / x0) * (1.0 / x0);
    double gl0 = a9;
    gl0 *= x2; gl0 += a8;
    gl0 *= x2; gl0 += a7;
    gl0 *= x2; gl0 += a6;
    gl0 *= x2; gl0 += a5;
    gl0 *= x2; gl0 += a4;
    gl0 *= x2; gl0 += a3;
    gl0 *= x2; gl0 += a2;
    gl0 *= x2; gl0 += a1;
    gl0 *= x2; gl0 += a0;
    const double lg2pi = 1.8378770664093453e+00;
    double gl = gl0 / x0 + 0.5 * lg2pi + (x0 - 0.5) * log(x0) - x0;
    if (x < 7.0) {
        for (int64_t k = 1; k <= n; k++) {
            gl -= log(x0 - 1.0);
            x0 -= 1.0;
        }
    }
    return gl;
}

// PTRS right-hand side  -lam + k*log(lam) - loggam(k+1): host table when k is
// inside it (computed with the host libm, exactly as numpy), else on device.
__device__ __forceinline__ double ptrs_rhs(const PtrsConst &c, const double *rhs, int64_t k) {
    if (rhs && k >= c.k0 && k < (int64_t)c.k0 + c.nk) return rhs[k - c.k0];
    return -c.lam + (double)k * c.loglam - np_loggam((double)(k + 1));
}

// PTRS log-acceptance test  log(V) + log(invalpha) - log(a/us^2 + b) <= r,
// decided with the f32 hardware log2 (v_log_f32) whenever the f32 estimate is
// farther from r than a rigorous bound on its error; only near-ties (and
// overflow) evaluate the f64 logs.  Same decision as the f64 test.
#ifdef INVSIM_PTRS_STATS
// Debug build only (make ptrs_stats): per translation unit, [0] log tests,
// [1] tests ptrs_log_accept's f32 pre-test left to f64, [2] bits of the
// smallest relative margin |lhs - r| / (|log V| + |log(1/alpha)| + |log x| + |r|)
// over all tests (non-negative doubles order like their bit patterns), [3] f32
// decisions that disagree with the f64 test (must stay 0), [4] log tests the
// decide path's f32 test (ptrs_decide_d) left to the exact branch.  Read by
// invsim_debug_ptrs_stats.
static __device__ unsigned long long g_ptrs_stats[5] = {0ull, 0ull, 0x7ff0000000000000ull, 0ull, 0ull};
#define INVSIM_PTRS_STATS_TU(tu)                                                                   \
    hipError_t ptrs_stats_##tu(unsigned long long *out, bool clear) {                              \
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ptrs_stats), sizeof(g_ptrs_stats));   \
        if (e != hipSuccess || !clear) return e;                                                   \
        const unsigned long long init[5] = {0ull, 0ull, 0x7ff0000000000000ull, 0ull, 0ull};        \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_ptrs_stats), init, sizeof(init));                    \
    }

__device__ __forceinline__ bool ptrs_log_accept_f32(const PtrsConst &c, double V, double us, double r, bool &decided);

__device__ __forceinline__ bool ptrs_log_accept(const PtrsConst &c, double V, double us, double r) {
    bool decided;
    const bool fast = ptrs_log_accept_f32(c, V, us, r, decided);
    const double lv = log(V), lx = log(c.a / (us * us) + c.b);
    const double lhs = lv + c.log_invalpha - lx;
    const bool exact = lhs <= r;
    const double margin = fabs(lhs - r) / (fabs(lv) + fabs(c.log_invalpha) + fabs(lx) + fabs(r));
    atomicAdd(&g_ptrs_stats[0], 1ull);
    if (!decided) atomicAdd(&g_ptrs_stats[1], 1ull);
    if (decided && fast != exact) atomicAdd(&g_ptrs_stats[3], 1ull);
    atomicMin(&g_ptrs_stats[2], (unsigned long long)__double_as_longlong(margin));
    return exact;
}

__device__ __forceinline__ bool ptrs_log_accept_f32(const PtrsConst &c, double V, double us, double r, bool &decided) {
    decided = true;
#else
#define INVSIM_PTRS_STATS_TU(tu)
__device__ __forceinline__ bool ptrs_log_accept(const PtrsConst &c, double V, double us, double r) {
#endif
    constexpr double LN2 = 0.69314718055994530942;
    const float us32 = (float)us;
    const float x32 = (float)c.a / (us32 * us32) + (float)c.b;   // rel. error < 8 * 2^-24
    if (x32 < 1e30f) {
        const float l2v = __builtin_amdgcn_logf((float)V);        // log2, |err| <= 1 ulp(f32)
        const float l2x = __builtin_amdgcn_logf(x32);
        const double lhs = ((double)l2v * LN2 + c.log_invalpha) - (double)l2x * LN2;
        // |f32 log2 error| <= 2^-22 |log2| (4 ulp) plus the input roundings
        // (V: 2^-24, x: 2^-21 relative -> <= 2^-20 absolute in log2); f64 slack 2^-40
        const double err = (fabs((double)l2v) + fabs((double)l2x)) * (LN2 * 0x1p-22) +
                           LN2 * 0x1p-19 + (fabs(lhs) + fabs(r)) * 0x1p-40;
        if (lhs + err < r) return true;
        if (lhs - err > r) return false;
    }
#ifdef INVSIM_PTRS_STATS
    decided = false;
#endif
    return (log(V) + c.log_invalpha - log(c.a / (us * us) + c.b)) <= r;
}

// One numpy PTRS candidate (the loop body of random_poisson_ptrs) from its two
// uniforms, with the same decision as the branchy form above, laid out for a
// lone wave: its three chains -- k (the f64 division and floor), the f32 log
// test (us, V only) and the RHS table read (k only) -- are computed for every
// lane without branches between them, so they interleave instead of running
// one after the other; only a near-tie of the f32 test, x/us overflow or k
// outside the table take the exact branch.
//
// The fast test runs in f32 end to end (round 5: 9 f32 instructions where the
// f64 combination took ~17; a stream wave's cost is its instruction count).
// With l2v = log2f(fl(V)), l2x = log2f(x32), x32 = a * rcp(us^2) + b in f32,
// and every f32 rounding counted (d = l2v - l2x, L = fma(d, ln2, log_invalpha),
// the f32 ln2, log_invalpha and r, diff = r - L):
//   |diff - (r - lhs)| <= ln2 (|l2v| + |l2x|) (2^-22 + 4 * 2^-24)   [log2f 4 ulp + roundings]
//                       + ln2 * 2^-19                                 [V, x input roundings]
//                       + 3 * 2^-24 |log_invalpha| + 2 * 2^-24 |r| + 2^-24 |diff|
// which  e = (|l2v| + |l2x|) 2^-20 + |r| 2^-22 + (2^-18 + 2^-22 |log_invalpha|)
// bounds with a factor >= 2 to spare (that slack also covers e's own f32
// roundings): diff > e decides accept, diff < -e reject, as numpy's f64 test.
// tab(kd, ok): -lam + kd log lam - loggam(kd + 1) from an LDS table for the
// candidate's floor value kd (ok = false: kd outside it, value unused);
// rhs(k): the same, exactly, on device.
// ptrs_decide_d hands back the candidate as its floor value kd, a double
// (numpy's k is (int64)kd, and kd is integral, so nothing is lost): a caller
// that keeps the draw as a double skips the int64 conversion per candidate.
template <class Tab, class Rhs>
__device__ __forceinline__ bool ptrs_decide_d(const PtrsConst &c, double U, double V, Tab tab, Rhs rhs, double &kd) {
    const double us = 0.5 - fabs(U);
    kd = floor((c.a2 / us + c.b) * U + c.lam + 0.43);
    const float us32 = (float)us;
    const float x32 = (float)c.a * __builtin_amdgcn_rcpf(us32 * us32) + (float)c.b;
    const float l2v = __builtin_amdgcn_logf((float)V);
    const float l2x = __builtin_amdgcn_logf(x32);
    bool ok;
    const double r = tab(kd, ok);      // kd == (double)k wherever the table is read (0 <= k < 2^53)
    // bitwise, not short-circuit, here and below: no branch per condition
    const bool qacc = (us >= 0.07) & (V <= c.vr);
    const bool qrej = (kd < 0.0) | ((us < 0.013) & (V > us));     // k < 0 (kd is never NaN; -inf: k < 0 too)
    const float lia = (float)c.log_invalpha;
    const float r32 = (float)r;
    const float L = __builtin_fmaf(l2v - l2x, 0.693147180559945309f, lia);
    const float diff = r32 - L;
    const float e = __builtin_fmaf(fabsf(l2v) + fabsf(l2x), 0x1p-20f,
                                   __builtin_fmaf(fabsf(r32), 0x1p-22f, __builtin_fmaf(fabsf(lia), 0x1p-22f, 0x1p-18f)));
    const bool fin = ok & (x32 < 1e30f);
    const bool facc = fin & (diff > e), frej = fin & (diff < -e);
#ifdef INVSIM_PTRS_STATS
    if (!qacc && !qrej && (facc || frej)) {   // f32-decided: count and check against the f64 test
        const double lhs64 = log(V) + c.log_invalpha - log(c.a / (us * us) + c.b);
        const bool exact = lhs64 <= r;
        const double margin = fabs(lhs64 - r) / (fabs(log(V)) + fabs(c.log_invalpha) +
                                                 fabs(log(c.a / (us * us) + c.b)) + fabs(r));
        atomicAdd(&g_ptrs_stats[0], 1ull);
        if (facc != exact) atomicAdd(&g_ptrs_stats[3], 1ull);
        atomicMin(&g_ptrs_stats[2], (unsigned long long)__double_as_longlong(margin));
    }
#endif
    const bool dec = qacc | qrej | facc | frej;
#ifdef INVSIM_PTRS_STATS
    if (!dec) atomicAdd(&g_ptrs_stats[4], 1ull);
#endif
    bool acc = qacc | (!qrej & facc);
    if (!dec) acc = ptrs_log_accept(c, V, us, ok ? r : rhs((int64_t)kd));   // rare: the exact path
    return acc;
}

template <class Tab, class Rhs>
__device__ __forceinline__ bool ptrs_decide(const PtrsConst &c, double U, double V, Tab tab, Rhs rhs, int64_t &k) {
    double kd;
    const bool acc = ptrs_decide_d(c, U, V, tab, rhs, kd);
    k = (int64_t)kd;
    return acc;
}

// numpy random_poisson_ptrs (distributions.c), constants precomputed
template <class G>
__device__ inline int64_t np_poisson_ptrs(G &g, const PtrsConst &c, const double *rhs = nullptr) {
    for (;;) {
        double U = g.next_double() - 0.5;
        double V = g.next_double();
        double us = 0.5 - fabs(U);
        int64_t k = (int64_t)floor((c.a2 / us + c.b) * U + c.lam + 0.43);
        if ((us >= 0.07) && (V <= c.vr)) return k;
        if ((k < 0) || ((us < 0.013) && (V > us))) continue;
        if (ptrs_log_accept(c, V, us, ptrs_rhs(c, rhs, k))) return k;
    }
}

// numpy random_poisson_mult (0 < lam < 10), enlam = exp(-lam)
template <class G>
__device__ inline int64_t np_poisson_mult(G &g, double enlam) {
    int64_t X = 0;
    double prod = 1.0;
    for (;;) {
        prod *= g.next_double();
        if (prod > enlam)
            X += 1;
        else
            return X;
    }
}

// numpy random_poisson with host-precomputed constants (fixed lam)
template <class G>
__device__ __forceinline__ int64_t np_poisson(G &g, const PtrsConst &c, const double *rhs = nullptr) {
    if (c.lam >= 10) return np_poisson_ptrs(g, c, rhs);
    if (c.lam == 0) return 0;
    return np_poisson_mult(g, c.enlam);
}

// numpy random_poisson_ptrs for a per-env lam with a (lam-independent) table of
// loggam(k + 1), k < lgn, computed on the host with numpy's own formula
template <class G>
__device__ inline int64_t np_poisson_ptrs_lg(G &g, const PtrsConst &c, const double *lgtab, int lgn) {
    for (;;) {
        double U = g.next_double() - 0.5;
        double V = g.next_double();
        double us = 0.5 - fabs(U);
        int64_t k = (int64_t)floor((c.a2 / us + c.b) * U + c.lam + 0.43);
        if ((us >= 0.07) && (V <= c.vr)) return k;
        if ((k < 0) || ((us < 0.013) && (V > us))) continue;
        const double r = (k < lgn) ? (-c.lam + (double)k * c.loglam) - lgtab[k < lgn ? k : 0]
                                   : -c.lam + (double)k * c.loglam - np_loggam((double)(k + 1));
        if (ptrs_log_accept(c, V, us, r)) return k;
    }
}

// numpy random_poisson for a per-env lam: only the branch's constants are computed
template <class G>
__device__ inline int64_t np_poisson_dyn(G &g, double lam, const double *lgtab, int lgn) {
    if (lam >= 10) {
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
        c.k0 = 0;
        c.nk = 0;
        return np_poisson_ptrs_lg(g, c, lgtab, lgn);
    }
    if (lam == 0) return 0;
    return np_poisson_mult(g, exp(-lam));
}

// numpy random_poisson for a per-env lam: only the branch's constants are computed
template <class G>
__device__ inline int64_t np_poisson_dyn(G &g, double lam) {
    if (lam >= 10) {
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
        c.k0 = 0;
        c.nk = 0;
        return np_poisson_ptrs(g, c);
    }
    if (lam == 0) return 0;
    return np_poisson_mult(g, exp(-lam));
}

// ---------------------------------------------------------------- numpy sums
// numpy add.reduce over a short contiguous 1-D array: identity 0, then
// pairwise_sum (n < 8 sequential; n <= 128 eight accumulators + tail).
template <typename T, class Get>
__device__ __forceinline__ T np_sum(int n, Get get) {
    T res;
    if (n < 8) {
        res = (T)0;
        for (int i = 0; i < n; i++) res += get(i);
    } else {
        T r0 = get(0), r1 = get(1), r2 = get(2), r3 = get(3), r4 = get(4), r5 = get(5),
          r6 = get(6), r7 = get(7);
        int i = 8;
        for (; i < n - (n % 8); i += 8) {
            r0 += get(i + 0); r1 += get(i + 1); r2 += get(i + 2); r3 += get(i + 3);
            r4 += get(i + 4); r5 += get(i + 5); r6 += get(i + 6); r7 += get(i + 7);
        }
        res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (; i < n; i++) res += get(i);
    }
    return (T)0 + res;
}

// ---------------------------------------------------------------- RNG state I/O
// PCG64 per env as four SoA rows (state_hi, state_lo, inc_hi, inc_lo): a
// wave's load of a row is 512 contiguous bytes (a 32-byte record per env was
// measured 1 % slower on the InvMgmt step: twice the cache lines per load)
struct RngSoA {
    uint64_t *hi, *lo, *inc_hi, *inc_lo;
    __device__ __forceinline__ Pcg load(int64_t e) const {
        Pcg g;
        g.hi = hi[e];
        g.lo = lo[e];
        g.inc_hi = inc_hi[e];
        g.inc_lo = inc_lo[e];
        return g;
    }
    __device__ __forceinline__ void store_state(int64_t e, const Pcg &g) const {
        hi[e] = g.hi;
        lo[e] = g.lo;
    }
    __device__ __forceinline__ void store_all(int64_t e, const Pcg &g) const {
        hi[e] = g.hi;
        lo[e] = g.lo;
        inc_hi[e] = g.inc_hi;
        inc_lo[e] = g.inc_lo;
    }
    // a step kernel's generator: the PCG64 stream (32 B in, 16 B out per env) or
    // the fast stream's key (8 B in, nothing out)
    __device__ __forceinline__ void load(int64_t e, Pcg &g) const { g = load(e); }
    __device__ __forceinline__ void load(int64_t e, PhiloxGen &g) const {
        const uint64_t k = inc_hi[e];
        g.key = make_uint2((uint32_t)k, (uint32_t)(k >> 32));
    }
    __device__ __forceinline__ void store_state(int64_t, const PhiloxGen &) const {}
};

}  // namespace invsim
