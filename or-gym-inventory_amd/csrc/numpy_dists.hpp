// numpy 2.2.6 Generator samplers for the InvManagement demand distributions
// other than Poisson (inventory_management.py:173-182):
//   dist 2  np_random.binomial(n, p)            random_binomial (inversion / BTPE)
//   dist 3  np_random.integers(low, high + 1)   random_bounded_uint64_fill (Lemire,
//                                               32-bit draws buffered in the bit generator)
//   dist 4  np_random.geometric(p)              random_geometric (search / inversion
//                                               of the 256-level exponential ziggurat)
// Every per-(n, p) constant is computed on the host with the host libm (numpy's
// bits); per-draw libm calls (BTPE's logs, the ziggurat's rare exp/log1p) use
// the device libm.  The CPU oracle (oracle/oracle.c) restates the same and is
// checked draw-for-draw against numpy itself (tests/test_oracle.py).
#pragma once
#include "device_common.hpp"
#include "numpy_ziggurat.hpp"

namespace invsim {

struct NpDist {
    int32_t kind;        // 2 binomial, 3 integers, 4 geometric
    int32_t flip;        // binomial with p > 0.5: n - X(n, 1 - p)
    int32_t inversion;   // binomial: inversion (else BTPE); geometric: search (else inversion)
    int32_t zero;        // binomial n == 0 or p == 0: always 0
    int64_t n;           // binomial n
    double p;            // binomial: the p the sampler runs with (<= 0.5); geometric p
    // binomial inversion: q, qn, np, bound; BTPE: r, q, fm, m, p1, xm, xl, xr, c, laml, lamr, p2, p3, p4
    double q, qn, np_, r, fm, p1, xm, xl, xr, c, laml, lamr, p2, p3, p4;
    int64_t bound, m;
    // integers: off + [0, rng]
    uint64_t off, rng;
    // geometric inversion: log1p(-p)
    double log1mp;
};

// pcg64_next32: low half first, high half buffered (bit 32 of buf = has_uint32)
template <class G>
__device__ __forceinline__ uint32_t np_next32(G &g, uint64_t &buf) {
    if (buf >> 32) {
        const uint32_t v = (uint32_t)buf;
        buf = 0;
        return v;
    }
    const uint64_t x = g.next64();
    buf = (1ull << 32) | (x >> 32);
    return (uint32_t)x;
}

template <class G>
__device__ inline int64_t np_integers(G &g, uint64_t &buf, const NpDist &d) {
    const uint64_t r = d.rng;
    if (r == 0) return (int64_t)d.off;
    if (r <= 0xFFFFFFFFull) {
        if (r == 0xFFFFFFFFull) return (int64_t)(d.off + np_next32(g, buf));
        const uint32_t rng_excl = (uint32_t)r + 1;
        uint64_t m = (uint64_t)np_next32(g, buf) * rng_excl;
        uint32_t leftover = (uint32_t)m;
        if (leftover < rng_excl) {
            const uint32_t threshold = (uint32_t)((0xFFFFFFFFu - (uint32_t)r) % rng_excl);
            while (leftover < threshold) {
                m = (uint64_t)np_next32(g, buf) * rng_excl;
                leftover = (uint32_t)m;
            }
        }
        return (int64_t)(d.off + (m >> 32));
    }
    if (r == 0xFFFFFFFFFFFFFFFFull) return (int64_t)(d.off + g.next64());
    const uint64_t rng_excl = r + 1;
    uint64_t x = g.next64();
    uint64_t lo = x * rng_excl, hi = __umul64hi(x, rng_excl);
    if (lo < rng_excl) {
        const uint64_t threshold = (0xFFFFFFFFFFFFFFFFull - r) % rng_excl;
        while (lo < threshold) {
            x = g.next64();
            lo = x * rng_excl;
            hi = __umul64hi(x, rng_excl);
        }
    }
    return (int64_t)(d.off + hi);
}

template <class G>
__device__ inline int64_t np_binomial_inversion(G &g, const NpDist &d) {
    const int64_t n = d.n;
    const double p = d.p, q = d.q, qn = d.qn;
    int64_t X = 0;
    double px = qn;
    double U = g.next_double();
    while (U > px) {
        X++;
        if (X > d.bound) {
            X = 0;
            px = qn;
            U = g.next_double();
        } else {
            U -= px;
            px = ((n - X + 1) * p * px) / (X * q);
        }
    }
    return X;
}

template <class G>
__device__ inline int64_t np_binomial_btpe(G &g, const NpDist &d) {
    const int64_t n = d.n, m = d.m;
    const double r = d.r, q = d.q, xm = d.xm, xl = d.xl, xr = d.xr, c = d.c, laml = d.laml, lamr = d.lamr;
    const double p1 = d.p1, p2 = d.p2, p3 = d.p3, p4 = d.p4;
    const double nrq = n * r * q;
    for (;;) {
        const double u = g.next_double() * p4;
        double v = g.next_double();
        int64_t y;
        if (u <= p1) return (int64_t)floor(xm - p1 * v + u);                  // Step10 -> 60
        if (u <= p2) {                                                        // Step20
            const double x = xl + (u - p1) / c;
            v = v * c + 1.0 - fabs(m - x + 0.5) / p1;
            if (v > 1.0) continue;
            y = (int64_t)floor(x);
        } else if (u <= p3) {                                                 // Step30
            y = (int64_t)floor(xl + log(v) / laml);
            if ((y < 0) || (v == 0.0)) continue;
            v = v * (u - p2) * laml;
        } else {                                                              // Step40
            y = (int64_t)floor(xr - log(v) / lamr);
            if ((y > n) || (v == 0.0)) continue;
            v = v * (u - p3) * lamr;
        }
        const int64_t k = y > m ? y - m : m - y;                              // Step50
        if (!((k > 20) && (k < ((nrq) / 2.0 - 1)))) {
            const double s = r / q;
            const double a = s * (n + 1);
            double F = 1.0;
            if (m < y) {
                for (int64_t i = m + 1; i <= y; i++) F *= (a / i - s);
            } else if (m > y) {
                for (int64_t i = y + 1; i <= m; i++) F /= (a / i - s);
            }
            if (v > F) continue;
            return y;
        }
        // Step52
        const double rho = (k / (nrq)) * ((k * (k / 3.0 + 0.625) + 0.16666666666666666) / nrq + 0.5);
        const double t = -k * k / (2 * nrq);
        const double A = log(v);
        if (A < (t - rho)) return y;
        if (A > (t + rho)) continue;
        const double x1 = y + 1, f1 = m + 1, z = n + 1 - m, w = n - y + 1;
        const double x2 = x1 * x1, f2 = f1 * f1, z2 = z * z, w2 = w * w;
        if (A > (xm * log(f1 / x1) + (n - m + 0.5) * log(z / w) + (y - m) * log(w * r / (x1 * q)) +
                 (13680. - (462. - (132. - (99. - 140. / f2) / f2) / f2) / f2) / f1 / 166320. +
                 (13680. - (462. - (132. - (99. - 140. / z2) / z2) / z2) / z2) / z / 166320. +
                 (13680. - (462. - (132. - (99. - 140. / x2) / x2) / x2) / x2) / x1 / 166320. +
                 (13680. - (462. - (132. - (99. - 140. / w2) / w2) / w2) / w2) / w / 166320.))
            continue;
        return y;
    }
}

template <class G>
__device__ inline int64_t np_binomial(G &g, const NpDist &d) {
    if (d.zero) return 0;
    const int64_t X = d.inversion ? np_binomial_inversion(g, d) : np_binomial_btpe(g, d);
    return d.flip ? d.n - X : X;
}

template <class G>
__device__ inline double np_standard_exponential(G &g) {
    for (;;) {
        uint64_t ri = g.next64();
        ri >>= 3;
        const int idx = (int)(ri & 0xFF);
        ri >>= 8;
        const double x = ri * npz_we[idx];
        if (ri < npz_ke[idx]) return x;
        if (idx == 0) return NPZ_EXP_R - log1p(-g.next_double());
        if ((npz_fe[idx - 1] - npz_fe[idx]) * g.next_double() + npz_fe[idx] < exp(-x)) return x;
    }
}

template <class G>
__device__ inline int64_t np_geometric(G &g, const NpDist &d) {
    if (d.inversion) {                                   // search, p >= 1/3
        int64_t X = 1;
        double sum = d.p, prod = d.p;
        const double U = g.next_double();
        while (U > sum) {
            prod *= d.q;
            sum += prod;
            X++;
        }
        return X;
    }
    const double z = ceil(-np_standard_exponential(g) / d.log1mp);
    if (z >= 9.223372036854776e+18) return INT64_MAX;
    return (int64_t)z;
}

template <class G>
__device__ __forceinline__ int64_t np_demand(G &g, uint64_t &buf, const NpDist &d) {
    if (d.kind == 2) return np_binomial(g, d);
    if (d.kind == 3) return np_integers(g, buf, d);
    return np_geometric(g, d);
}

// host: the per-(n, p) constants numpy computes on first use (binomial_t cache)
inline NpDist np_dist_binomial(int64_t n, double p) {
    NpDist d{};
    d.kind = 2;
    d.zero = (n == 0) || (p == 0.0f);
    double pp = p;
    if (p > 0.5) {
        d.flip = 1;
        pp = 1.0 - p;
    }
    d.n = n;
    d.p = pp;
    if (pp * n <= 30.0) {
        d.inversion = 1;
        d.q = 1.0 - pp;
        d.qn = exp(n * log(d.q));
        d.np_ = n * pp;
        d.bound = (int64_t)fmin((double)n, d.np_ + 10.0 * sqrt(d.np_ * d.q + 1));
    } else {
        d.r = fmin(pp, 1.0 - pp);
        d.q = 1.0 - d.r;
        d.fm = n * d.r + d.r;
        d.m = (int64_t)floor(d.fm);
        d.p1 = floor(2.195 * sqrt(n * d.r * d.q) - 4.6 * d.q) + 0.5;
        d.xm = d.m + 0.5;
        d.xl = d.xm - d.p1;
        d.xr = d.xm + d.p1;
        d.c = 0.134 + 20.5 / (15.3 + d.m);
        double a = (d.fm - d.xl) / (d.fm - d.xl * d.r);
        d.laml = a * (1.0 + a / 2.0);
        a = (d.xr - d.fm) / (d.xr * d.q);
        d.lamr = a * (1.0 + a / 2.0);
        d.p2 = d.p1 * (1.0 + 2.0 * d.c);
        d.p3 = d.p2 + d.c / d.laml;
        d.p4 = d.p3 + d.c / d.lamr;
    }
    return d;
}

inline NpDist np_dist_integers(int64_t low, int64_t high_incl) {
    NpDist d{};
    d.kind = 3;
    d.off = (uint64_t)low;
    d.rng = (uint64_t)high_incl - (uint64_t)low;
    return d;
}

inline NpDist np_dist_geometric(double p) {
    NpDist d{};
    d.kind = 4;
    d.p = p;
    d.q = 1.0 - p;
    d.inversion = p >= 0.333333333333333333333333;
    d.log1mp = log1p(-p);
    return d;
}

}  // namespace invsim
