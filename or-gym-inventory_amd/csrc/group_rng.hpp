// Lane-group Poisson sampling: G = 4 lanes per env evaluate 4 consecutive
// PTRS candidates (or 16 multiplication-method uniforms) of the SAME numpy
// PCG64 stream at once, then agree on the first accepted one.  The draws,
// the accepted value and the final stream position are exactly those of the
// sequential numpy algorithm; only the evaluation is parallel.
//
// Why: at 65 536 envs a one-thread-per-env step is one wave per SIMD, and
// PTRS's accept/reject loop (about 3 rounds per wave once 64 lanes must all
// accept, each with the log test) is a long dependent f64 chain.  Four lanes
// per env quadruple the waves per SIMD and finish the draw in one round
// (all four candidates rejected: p ~ 2e-4 per env).
//
// Stream positions come from PCG64 jump-ahead: after n steps the LCG state is
// A_n * s + S_n * inc  (mod 2^128) with A_n = M^n, S_n = 1 + M + ... + M^(n-1).
#pragma once
#include "device_common.hpp"

namespace invsim {

constexpr int GRP = 4;          // lanes per env
constexpr int JUMP_MAX = 16;    // jump table covers n = 0..16

struct JumpTable {
    uint64_t a_hi[JUMP_MAX + 1], a_lo[JUMP_MAX + 1], s_hi[JUMP_MAX + 1], s_lo[JUMP_MAX + 1];
};

constexpr JumpTable make_jump_table() {
    JumpTable t{};
    typedef unsigned __int128 u128;
    const u128 M = ((u128)PCG_MULT_HI << 64) | PCG_MULT_LO;
    u128 a = 1, s = 0;
    for (int n = 0; n <= JUMP_MAX; n++) {
        t.a_hi[n] = (uint64_t)(a >> 64);
        t.a_lo[n] = (uint64_t)a;
        t.s_hi[n] = (uint64_t)(s >> 64);
        t.s_lo[n] = (uint64_t)s;
        s = s + a;  // S_{n+1} = S_n + M^n
        a = a * M;
    }
    return t;
}

static __constant__ JumpTable c_jump = make_jump_table();

// low 128 bits of (ahi:alo) * (bhi:blo)
__device__ __forceinline__ void mul128(uint64_t ahi, uint64_t alo, uint64_t bhi, uint64_t blo,
                                       uint64_t &rhi, uint64_t &rlo) {
    rlo = alo * blo;
    rhi = __umul64hi(alo, blo) + alo * bhi + ahi * blo;
}

// advance g by n LCG steps (0 <= n <= JUMP_MAX)
__device__ __forceinline__ void pcg_jump(Pcg &g, int n) {
    uint64_t ah, al, sh, sl;
    mul128(c_jump.a_hi[n], c_jump.a_lo[n], g.hi, g.lo, ah, al);
    mul128(c_jump.s_hi[n], c_jump.s_lo[n], g.inc_hi, g.inc_lo, sh, sl);
    const uint64_t lo = al + sl;
    g.hi = ah + sh + (lo < al ? 1ULL : 0ULL);
    g.lo = lo;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    return (uint64_t)__shfl((long long)v, src);
}

// numpy random_poisson_ptrs, lane-group form.  `rhs` (nullable) holds the
// host-computed right-hand side  -lam + k*log(lam) - loggam(k+1)  for k in
// [c.k0, c.k0 + c.nk); outside it the device computes it.  All GRP lanes of an
// env call this together with identical g and c.
__device__ inline int64_t poisson_ptrs_grp(Pcg &g, const PtrsConst &c, const double *rhs) {
    const int lane = (int)(threadIdx.x & 63);
    const int j = lane & (GRP - 1);
    const int base = lane & ~(GRP - 1);
    for (;;) {
        Pcg s = g;
        pcg_jump(s, 2 * j);                               // candidate j: draws 2j+1, 2j+2
        const double U = s.next_double() - 0.5;
        const double V = s.next_double();
        const double us = 0.5 - fabs(U);
        const int64_t k = (int64_t)floor((c.a2 / us + c.b) * U + c.lam + 0.43);
        bool acc;
        if ((us >= 0.07) && (V <= c.vr)) {
            acc = true;
        } else if ((k < 0) || ((us < 0.013) && (V > us))) {
            acc = false;
        } else {
            acc = ptrs_log_accept(c, V, us, ptrs_rhs(c, rhs, k));
        }
        const uint64_t m = (uint64_t)__ballot(acc);
        const unsigned gm = (unsigned)(m >> base) & ((1u << GRP) - 1u);
        if (gm) {
            const int src = base + __builtin_ctz(gm);
            g.hi = shfl_u64(s.hi, src);
            g.lo = shfl_u64(s.lo, src);
            return (int64_t)shfl_u64((uint64_t)k, src);
        }
        g.hi = shfl_u64(s.hi, base + GRP - 1);            // all rejected: continue after 2*GRP draws
        g.lo = shfl_u64(s.lo, base + GRP - 1);
    }
}

// numpy random_poisson_mult (0 < lam < 10), lane-group form: each lane draws 4
// consecutive uniforms, every lane forms the sequential product in stream order.
__device__ inline int64_t poisson_mult_grp(Pcg &g, double enlam) {
    const int lane = (int)(threadIdx.x & 63);
    const int j = lane & (GRP - 1);
    const int base = lane & ~(GRP - 1);
    constexpr int R = 4;                                   // uniforms per lane per round
    int64_t X = 0;
    double prod = 1.0;
    for (;;) {
        Pcg s = g;
        pcg_jump(s, R * j);
        double u[R];
#pragma unroll
        for (int q = 0; q < R; q++) u[q] = s.next_double();
        int stop = -1;
#pragma unroll
        for (int src = 0; src < GRP; src++) {
#pragma unroll
            for (int q = 0; q < R; q++) {
                const double uq = __shfl(u[q], base + src);
                if (stop < 0) {
                    prod *= uq;
                    if (prod > enlam)
                        X += 1;
                    else
                        stop = src * R + q;
                }
            }
        }
        if (stop >= 0) {
            pcg_jump(g, stop + 1);                          // uniforms consumed: stop + 1
            return X;
        }
        pcg_jump(g, R * GRP);
    }
}

// ---------------------------------------------------------------- PTRS with a compacted second round
// One numpy PTRS draw per lane (one env per lane), for the demand lookahead
// whose chain is the launch's tail.  The sequential loop runs until the
// slowest of 64 lanes accepts (~3.5 candidates per wave against 1.15 per
// lane).  Here every lane evaluates its first candidate; the ~13 % of lanes
// that rejected are then packed into groups of CG = 4 lanes (up to 16 envs
// per wave), lane j of a group evaluating candidate j of the env's stream
// (LCG jump-ahead by 2j, group_rng.hpp), and the group takes the first
// accepted one in stream order -- the same draw, value and final state as
// numpy.  A group needs another round with probability ~0.13^4.  More than 16
// rejecting lanes fall back to the sequential loop.
constexpr int CG = 4;

// this lane's jump constants for its group position (A_n, S_n, n = 2 (lane & 3)),
// loaded early so the second round does not wait for them
struct PtrsJumpLane {
    uint64_t a_hi, a_lo, s_hi, s_lo;
    __device__ __forceinline__ void load(int lane) {
        const int n = 2 * (lane & (CG - 1));
        a_hi = c_jump.a_hi[n];
        a_lo = c_jump.a_lo[n];
        s_hi = c_jump.s_hi[n];
        s_lo = c_jump.s_lo[n];
    }
};

// Sources of the PTRS right-hand side  -lam + k log lam - loggam(k + 1):
// fast(k, c, ok) reads an LDS table (ok = false: k outside it, value unused),
// exact(k, c) computes it on device.
struct RhsTab {   // host table of the whole right-hand side for k in [c.k0, c.k0 + c.nk) (fixed rates)
    const double *t;
    __device__ __forceinline__ double fast(int64_t k, const PtrsConst &c, bool &ok) const {
        ok = k >= c.k0 && k < (int64_t)c.k0 + c.nk;
        return t[ok ? (int)(k - c.k0) : 0];
    }
    // the same for a candidate's floor value kd (ptrs_decide)
    __device__ __forceinline__ double fastd(double kd, const PtrsConst &c, bool &ok) const {
        ok = (kd >= (double)c.k0) & (kd < (double)(c.k0 + c.nk));
        return t[ok ? (int)kd - c.k0 : 0];
    }
    __device__ __forceinline__ double exact(int64_t k, const PtrsConst &c) const { return ptrs_rhs(c, nullptr, k); }
};
// (LgTab, the Newsvendor table source, is in kernels.hpp beside RHS_LDS_MAX)

// one PTRS candidate (numpy random_poisson_ptrs loop body) from two uniforms of
// g; src: RhsTab / LgTab.  INVSIM_PTRS_DECIDE=0 builds the branchy body (A/B).
#ifndef INVSIM_PTRS_DECIDE
#define INVSIM_PTRS_DECIDE 1
#endif
template <class G, class Src>
__device__ __forceinline__ bool ptrs_candidate(G &g, const PtrsConst &c, const Src &src, int64_t &k) {
    const double U = g.next_double() - 0.5;
    const double V = g.next_double();
#if INVSIM_PTRS_DECIDE
    return ptrs_decide(
        c, U, V, [&](double kd, bool &ok) { return src.fastd(kd, c, ok); },
        [&](int64_t kk) { return src.exact(kk, c); }, k);
#else
    const double us = 0.5 - fabs(U);
    k = (int64_t)floor((c.a2 / us + c.b) * U + c.lam + 0.43);
    if ((us >= 0.07) && (V <= c.vr)) return true;
    if ((k < 0) || ((us < 0.013) && (V > us))) return false;
    bool ok;
    const double r = src.fast(k, c, ok);
    return ptrs_log_accept(c, V, us, ok ? r : src.exact(k, c));
#endif
}

// PTRS draw of the lane's env (c.lam >= 10 for every lane that calls it with
// `live`; lanes with !live take part in the wave's shuffles only).  For a
// per-env rate, `shfl_c` moves the constants to the group (identity when they
// are wave-uniform).
struct NoProbe {
    __device__ __forceinline__ void operator()(int) const {}
};

template <class Src, class ShflC, class Probe = NoProbe>
__device__ __forceinline__ int64_t np_poisson_ptrs_compact(Pcg &g, const PtrsConst &c, const Src &rhs, bool live,
                                                           const PtrsJumpLane &jt, ShflC shfl_c,
                                                           Probe probe = Probe()) {
    const int lane = (int)(threadIdx.x & 63);
    int64_t k = 0;
    bool acc = !live || ptrs_candidate(g, c, rhs, k);
    const uint64_t rem = (uint64_t)__ballot(!acc);
    const int nr = __popcll(rem);
    probe(3);    // profiling hook (TIMING build): first candidate evaluated
    if (nr == 0) return k;
    if (nr > 64 / CG) {                                   // sequential fallback
        while (!acc) acc = ptrs_candidate(g, c, rhs, k);
        return k;
    }
    // group r (lanes 4r .. 4r + 3) works for the r-th rejecting lane
    const int grp = lane / CG, jl = lane & (CG - 1), gbase = grp * CG;
    int src = lane;                                       // the grp-th set bit of rem: a wave-uniform
    {                                                     // scalar walk over rem's <= 16 bits
        uint64_t x = rem;
        for (int r = 0; r < nr; r++) {
            const int pos = (int)__builtin_ctzll(x);
            x &= x - 1;
            if (r == grp) src = pos;
        }
    }
    const bool act = grp < nr;
    Pcg s;                                                // the env's state after its first candidate
    s.hi = shfl_u64(g.hi, src);
    s.lo = shfl_u64(g.lo, src);
    s.inc_hi = shfl_u64(g.inc_hi, src);
    s.inc_lo = shfl_u64(g.inc_lo, src);
    const PtrsConst cc = shfl_c(c, src);
    uint64_t sih, sil;                                    // S_n * inc
    mul128(jt.s_hi, jt.s_lo, s.inc_hi, s.inc_lo, sih, sil);
    probe(4);    // profiling hook: groups formed
    bool done = !act;
    int64_t kk = 0;
    while (__ballot(!done)) {
        Pcg t = s;                                        // candidate jl: LCG steps 2 jl + 1, 2 jl + 2
        uint64_t ah, al;
        mul128(jt.a_hi, jt.a_lo, s.hi, s.lo, ah, al);
        t.lo = al + sil;
        t.hi = ah + sih + (t.lo < al ? 1ULL : 0ULL);
        int64_t kj = 0;
        const bool aj = !done && ptrs_candidate(t, cc, rhs, kj);
        const unsigned gm = (unsigned)((uint64_t)__ballot(aj) >> gbase) & ((1u << CG) - 1u);
        const int win = gbase + (gm ? __builtin_ctz(gm) : CG - 1);   // first accepted, or the last candidate
        const uint64_t nh = shfl_u64(t.hi, win), nl = shfl_u64(t.lo, win);
        const int64_t kw = (int64_t)shfl_u64((uint64_t)kj, win);
        if (!done) {
            s.hi = nh;
            s.lo = nl;
            if (gm) {
                kk = kw;
                done = true;
            }
        }
    }
    // the result and the advanced generator back to the rejecting lane (group rank)
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(rem >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rem, 0u));
    const int back = (!acc) ? rank * CG : lane;
    const uint64_t bh = shfl_u64(s.hi, back), bl = shfl_u64(s.lo, back);
    const int64_t bk = (int64_t)shfl_u64((uint64_t)kk, back);
    if (!acc) {
        g.hi = bh;
        g.lo = bl;
        k = bk;
    }
    return k;
}

// numpy random_poisson with fixed-lam constants (host libm) and optional RHS table
__device__ __forceinline__ int64_t np_poisson_grp(Pcg &g, const PtrsConst &c, const double *rhs) {
    if (c.lam >= 10) return poisson_ptrs_grp(g, c, rhs);
    if (c.lam == 0) return 0;
    return poisson_mult_grp(g, c.enlam);
}

// numpy random_poisson for a per-env lam (Newsvendor): constants on device
__device__ inline int64_t np_poisson_dyn_grp(Pcg &g, double lam) {
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
        return poisson_ptrs_grp(g, c, nullptr);
    }
    if (lam == 0) return 0;
    return poisson_mult_grp(g, exp(-lam));
}

}  // namespace invsim
