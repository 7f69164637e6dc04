/* invsim ORACLE — test infrastructure only (see oracle.h).
 *
 * CPU restatement of the reference hot path.  Every function cites the
 * reference file:line it restates.  Compile with -ffp-contract=off: the
 * reference's arithmetic (numpy / CPython on x86-64 SSE2) never fuses a
 * multiply-add, and neither may we.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ======================================================================
 * numpy SeedSequence (numpy/random/bit_generator.pyx, numpy 2.2.6):
 * pool_size 4, hashmix/mix constants below, generate_state(4, uint64).
 * Called by gymnasium.utils.seeding.np_random(seed) from Env.reset(seed=)
 * (newsvendor.py:102, inventory_management.py:197, network_management.py:303).
 * ==================================================================== */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t value, uint32_t *hc) {
    value ^= *hc;
    *hc *= SS_MULT_A;
    value *= *hc;
    value ^= value >> 16;
    return value;
}

static uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
    r ^= r >> 16;
    return r;
}

static const u128 PCG_MULT = ((u128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;

void orc_seed_pcg64(const uint32_t *words, int nwords, uint64_t rng[4]) {
    uint32_t pool[4];
    uint32_t hc = SS_INIT_A;
    for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < nwords ? words[i] : 0u, &hc);
    for (int s = 0; s < 4; s++)
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
    for (int s = 4; s < nwords; s++)
        for (int d = 0; d < 4; d++) pool[d] = ss_mix(pool[d], ss_hashmix(words[s], &hc));
    uint32_t out[8];
    uint32_t hb = SS_INIT_B;
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= SS_MULT_B;
        v *= hb;
        v ^= v >> 16;
        out[i] = v;
    }
    uint64_t w64[4];
    for (int k = 0; k < 4; k++) w64[k] = (uint64_t)out[2 * k] | ((uint64_t)out[2 * k + 1] << 32);
    /* PCG64.__init__ -> pcg64_set_seed(seed = w64[0:2], inc = w64[2:4]):
     * pcg_setseq_128_srandom_r: state=0; inc=(initseq<<1)|1; step; state+=initstate; step */
    u128 initstate = ((u128)w64[0] << 64) | w64[1];
    u128 initseq = ((u128)w64[2] << 64) | w64[3];
    u128 inc = (initseq << 1) | 1u;
    u128 st = 0;
    st = st * PCG_MULT + inc;
    st += initstate;
    st = st * PCG_MULT + inc;
    rng[0] = (uint64_t)(st >> 64);
    rng[1] = (uint64_t)st;
    rng[2] = (uint64_t)(inc >> 64);
    rng[3] = (uint64_t)inc;
}

/* PCG64 XSL-RR 128/64 (numpy pcg64.h pcg64_next64) */
uint64_t orc_next64(uint64_t rng[4]) {
    u128 st = ((u128)rng[0] << 64) | rng[1];
    u128 inc = ((u128)rng[2] << 64) | rng[3];
    st = st * PCG_MULT + inc;
    rng[0] = (uint64_t)(st >> 64);
    rng[1] = (uint64_t)st;
    uint64_t x = rng[0] ^ rng[1];
    unsigned rot = (unsigned)(rng[0] >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

/* numpy next_double: (next64 >> 11) * 2^-53 */
double orc_next_double(uint64_t rng[4]) {
    return (double)(orc_next64(rng) >> 11) * (1.0 / 9007199254740992.0);
}

/* numpy distributions.c random_loggam */
double orc_loggam(double x) {
    static const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03,
                                 7.936507936507937e-04, -5.952380952380952e-04,
                                 8.417508417508418e-04, -1.917526917526918e-03,
                                 6.410256410256410e-03, -2.955065359477124e-02,
                                 1.796443723688307e-01, -1.39243221690590e+00};
    int64_t n;
    if (x == 1.0 || x == 2.0) return 0.0;
    if (x < 7.0)
        n = (int64_t)(7 - x);
    else
        n = 0;
    double x0 = x + n;
    double x2 = (1.0 / x0) * (1.0 / x0);
    const double lg2pi = 1.8378770664093453e+00;
    double gl0 = a[9];
    for (int k = 8; k >= 0; k--) {
        gl0 *= x2;
        gl0 += a[k];
    }
    double gl = gl0 / x0 + 0.5 * lg2pi + (x0 - 0.5) * log(x0) - x0;
    if (x < 7.0) {
        for (int64_t k = 1; k <= n; k++) {
            gl -= log(x0 - 1.0);
            x0 -= 1.0;
        }
    }
    return gl;
}

/* numpy distributions.c random_poisson_ptrs (lam >= 10) */
static int64_t poisson_ptrs(uint64_t rng[4], double lam) {
    double slam = sqrt(lam);
    double loglam = log(lam);
    double b = 0.931 + 2.53 * slam;
    double a = -0.059 + 0.02483 * b;
    double invalpha = 1.1239 + 1.1328 / (b - 3.4);
    double vr = 0.9277 - 3.6224 / (b - 2);
    for (;;) {
        double U = orc_next_double(rng) - 0.5;
        double V = orc_next_double(rng);
        double us = 0.5 - fabs(U);
        int64_t k = (int64_t)floor((2 * a / us + b) * U + lam + 0.43);
        if ((us >= 0.07) && (V <= vr)) return k;
        if ((k < 0) || ((us < 0.013) && (V > us))) continue;
        if ((log(V) + log(invalpha) - log(a / (us * us) + b)) <=
            (-lam + k * loglam - orc_loggam(k + 1)))
            return k;
    }
}

/* numpy distributions.c random_poisson_mult (0 < lam < 10) */
static int64_t poisson_mult(uint64_t rng[4], double lam) {
    double enlam = exp(-lam);
    int64_t X = 0;
    double prod = 1.0;
    for (;;) {
        double U = orc_next_double(rng);
        prod *= U;
        if (prod > enlam)
            X += 1;
        else
            return X;
    }
}

int64_t orc_poisson(uint64_t rng[4], double lam) {
    if (lam >= 10) return poisson_ptrs(rng, lam);
    if (lam == 0) return 0;
    return poisson_mult(rng, lam);
}

void orc_poisson_fill(uint64_t rng[4], double lam, int64_t *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = orc_poisson(rng, lam);
}

/* ---- numpy Generator.integers / binomial / geometric (numpy 2.2.6,
 * random/src/distributions/distributions.c + pcg64.h), the demand samplers of
 * inventory_management.py:173-182 (dist 2, 3, 4). */

/* pcg64_next32: the low half of a 64-bit output first, the high half buffered
 * in the bit generator (has_uint32 / uinteger) for the next 32-bit draw */
uint32_t orc_next32(uint64_t rng[4], uint32_t *buf /* [2]: has, value */) {
    if (buf[0]) {
        buf[0] = 0;
        return buf[1];
    }
    uint64_t x = orc_next64(rng);
    buf[0] = 1;
    buf[1] = (uint32_t)(x >> 32);
    return (uint32_t)x;
}

/* random_bounded_uint64_fill(cnt = 1, use_masked = false): off + [0, rng] via
 * Lemire's method (32-bit buffered draws when rng fits in 32 bits) */
uint64_t orc_bounded_uint64(uint64_t rng[4], uint32_t *buf, uint64_t off, uint64_t r) {
    if (r == 0) return off;
    if (r <= 0xFFFFFFFFULL) {
        if (r == 0xFFFFFFFFULL) return off + orc_next32(rng, buf);
        const uint32_t rng_excl = (uint32_t)r + 1;
        uint64_t m = (uint64_t)orc_next32(rng, buf) * rng_excl;
        uint32_t leftover = (uint32_t)m;
        if (leftover < rng_excl) {
            const uint32_t threshold = (uint32_t)((UINT32_MAX - (uint32_t)r) % rng_excl);
            while (leftover < threshold) {
                m = (uint64_t)orc_next32(rng, buf) * rng_excl;
                leftover = (uint32_t)m;
            }
        }
        return off + (m >> 32);
    }
    if (r == 0xFFFFFFFFFFFFFFFFULL) return off + orc_next64(rng);
    const uint64_t rng_excl = r + 1;
    u128 m = (u128)orc_next64(rng) * rng_excl;
    uint64_t leftover = (uint64_t)m;
    if (leftover < rng_excl) {
        const uint64_t threshold = (UINT64_MAX - r) % rng_excl;
        while (leftover < threshold) {
            m = (u128)orc_next64(rng) * rng_excl;
            leftover = (uint64_t)m;
        }
    }
    return off + (uint64_t)(m >> 64);
}

/* Generator.integers(low, high) (high exclusive, int64) */
int64_t orc_integers(uint64_t rng[4], uint32_t *buf, int64_t low, int64_t high) {
    const uint64_t r = (uint64_t)high - (uint64_t)low - 1;
    return (int64_t)orc_bounded_uint64(rng, buf, (uint64_t)low, r);
}

/* random_binomial_inversion (n * p <= 30) */
static int64_t binomial_inversion(uint64_t rng[4], int64_t n, double p) {
    const double q = 1.0 - p;
    const double qn = exp(n * log(q));
    const double np = n * p;
    const int64_t bound = (int64_t)fmin((double)n, np + 10.0 * sqrt(np * q + 1));
    int64_t X = 0;
    double px = qn;
    double U = orc_next_double(rng);
    while (U > px) {
        X++;
        if (X > bound) {
            X = 0;
            px = qn;
            U = orc_next_double(rng);
        } else {
            U -= px;
            px = ((n - X + 1) * p * px) / (X * q);
        }
    }
    return X;
}

/* random_binomial_btpe (n * p > 30, p <= 0.5) */
static int64_t binomial_btpe(uint64_t rng[4], int64_t n, double p) {
    const double r = fmin(p, 1.0 - p);
    const double q = 1.0 - r;
    const double fm = n * r + r;
    const int64_t m = (int64_t)floor(fm);
    const double p1 = floor(2.195 * sqrt(n * r * q) - 4.6 * q) + 0.5;
    const double xm = m + 0.5;
    const double xl = xm - p1;
    const double xr = xm + p1;
    const double c = 0.134 + 20.5 / (15.3 + m);
    double a = (fm - xl) / (fm - xl * r);
    const double laml = a * (1.0 + a / 2.0);
    a = (xr - fm) / (xr * q);
    const double lamr = a * (1.0 + a / 2.0);
    const double p2 = p1 * (1.0 + 2.0 * c);
    const double p3 = p2 + c / laml;
    const double p4 = p3 + c / lamr;
    double u, v, x, s, F, rho, t, A, x1, x2, f1, f2, z, z2, w, w2, nrq;
    int64_t y, k, i;
step10:
    nrq = n * r * q;
    u = orc_next_double(rng) * p4;
    v = orc_next_double(rng);
    if (u > p1) goto step20;
    y = (int64_t)floor(xm - p1 * v + u);
    goto step60;
step20:
    if (u > p2) goto step30;
    x = xl + (u - p1) / c;
    v = v * c + 1.0 - fabs(m - x + 0.5) / p1;
    if (v > 1.0) goto step10;
    y = (int64_t)floor(x);
    goto step50;
step30:
    if (u > p3) goto step40;
    y = (int64_t)floor(xl + log(v) / laml);
    if ((y < 0) || (v == 0.0)) goto step10;
    v = v * (u - p2) * laml;
    goto step50;
step40:
    y = (int64_t)floor(xr - log(v) / lamr);
    if ((y > n) || (v == 0.0)) goto step10;
    v = v * (u - p3) * lamr;
step50:
    k = llabs(y - m);
    if ((k > 20) && (k < ((nrq) / 2.0 - 1))) goto step52;
    s = r / q;
    a = s * (n + 1);
    F = 1.0;
    if (m < y) {
        for (i = m + 1; i <= y; i++) F *= (a / i - s);
    } else if (m > y) {
        for (i = y + 1; i <= m; i++) F /= (a / i - s);
    }
    if (v > F) goto step10;
    goto step60;
step52:
    rho = (k / (nrq)) * ((k * (k / 3.0 + 0.625) + 0.16666666666666666) / nrq + 0.5);
    t = -k * k / (2 * nrq);
    A = log(v);
    if (A < (t - rho)) goto step60;
    if (A > (t + rho)) goto step10;
    x1 = y + 1;
    f1 = m + 1;
    z = n + 1 - m;
    w = n - y + 1;
    x2 = x1 * x1;
    f2 = f1 * f1;
    z2 = z * z;
    w2 = w * w;
    if (A > (xm * log(f1 / x1) + (n - m + 0.5) * log(z / w) + (y - m) * log(w * r / (x1 * q)) +
             (13680. - (462. - (132. - (99. - 140. / f2) / f2) / f2) / f2) / f1 / 166320. +
             (13680. - (462. - (132. - (99. - 140. / z2) / z2) / z2) / z2) / z / 166320. +
             (13680. - (462. - (132. - (99. - 140. / x2) / x2) / x2) / x2) / x1 / 166320. +
             (13680. - (462. - (132. - (99. - 140. / w2) / w2) / w2) / w2) / w / 166320.))
        goto step10;
step60:
    if (p > 0.5) y = n - y;
    return y;
}

/* random_binomial */
int64_t orc_binomial(uint64_t rng[4], int64_t n, double p) {
    if ((n == 0) || (p == 0.0f)) return 0;
    if (p <= 0.5) {
        if (p * n <= 30.0) return binomial_inversion(rng, n, p);
        return binomial_btpe(rng, n, p);
    }
    const double q = 1.0 - p;
    if (q * n <= 30.0) return n - binomial_inversion(rng, n, q);
    return n - binomial_btpe(rng, n, q);
}

#include "numpy_ziggurat.h"
#ifdef _OPENMP
#include <omp.h>
#endif

/* Env-parallel batch loops (each env owns its generator and history, so the
 * results do not depend on the thread count).  Default 1 thread: the tests use
 * the oracle as a checker; bench.py's cpu_baseline sets the host's cores. */
static int orc_threads = 1;
void orc_set_threads(int n) { orc_threads = n > 0 ? n : 1; }
int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_num_procs();
#else
    return 1;
#endif
}

/* random_standard_exponential (256-level ziggurat, tables from numpy) */
double orc_standard_exponential(uint64_t rng[4]) {
    for (;;) {
        uint64_t ri = orc_next64(rng);
        ri >>= 3;
        const uint8_t idx = (uint8_t)(ri & 0xFF);
        ri >>= 8;
        const double x = ri * npz_we[idx];
        if (ri < npz_ke[idx]) return x;
        if (idx == 0) return NPZ_EXP_R - log1p(-orc_next_double(rng));
        if ((npz_fe[idx - 1] - npz_fe[idx]) * orc_next_double(rng) + npz_fe[idx] < exp(-x)) return x;
    }
}

/* random_geometric: search for p >= 1/3, else inversion of the exponential */
int64_t orc_geometric(uint64_t rng[4], double p) {
    if (p >= 0.333333333333333333333333) {
        int64_t X = 1;
        double sum = p, prod = p;
        const double q = 1.0 - p;
        const double U = orc_next_double(rng);
        while (U > sum) {
            prod *= q;
            sum += prod;
            X++;
        }
        return X;
    }
    const double z = ceil(-orc_standard_exponential(rng) / log1p(-p));
    if (z >= 9.223372036854776e+18) return INT64_MAX;
    return (int64_t)z;
}

void orc_dist_fill(uint64_t rng[4], uint32_t *buf, int dist, int64_t n_or_low, int64_t high, double p,
                   int64_t *out, int64_t count) {
    for (int64_t i = 0; i < count; i++) {
        if (dist == 2) out[i] = orc_binomial(rng, n_or_low, p);
        else if (dist == 3) out[i] = orc_integers(rng, buf, n_or_low, high);
        else if (dist == 4) out[i] = orc_geometric(rng, p);
        else out[i] = 0;
    }
}

double orc_exponential_fill(uint64_t rng[4], double *out, int64_t count) {
    for (int64_t i = 0; i < count; i++) out[i] = orc_standard_exponential(rng);
    return 0.0;
}

/* numpy add.reduce for float32/float64 1-D contiguous input: identity 0 then
 * pairwise_sum (loops_utils.h.src): n<8 sequential; n<=128 eight accumulators;
 * else split at n/2 rounded down to a multiple of 8. */
static float pw_f32(const float *a, int64_t n) {
    if (n < 8) {
        float res = 0.f;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        float r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pw_f32(a, n2) + pw_f32(a + n2, n - n2);
    }
}

static double pw_f64(const double *a, int64_t n) {
    if (n < 8) {
        double res = 0.;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pw_f64(a, n2) + pw_f64(a + n2, n - n2);
    }
}

float orc_sum_f32(const float *a, int64_t n) { return 0.f + pw_f32(a, n); }
double orc_sum_f64(const double *a, int64_t n) { return 0. + pw_f64(a, n); }

/* ======================================================================
 * NumPy-2 (NEP 50) scalar type lattice used by NewsvendorEnv.step.
 * PY  = Python int/float ("weak": cast to the other operand's dtype)
 * F32 = np.float32, F64 = np.float64.
 * ==================================================================== */
enum { K_PY = 0, K_F32 = 1, K_F64 = 2 };
typedef struct {
    double v;
    int k;
} tv;

static tv tv_make(double v, int k) {
    tv r;
    r.v = v;
    r.k = k;
    return r;
}

static tv tv_bin(tv a, tv b, char op) {
    tv r;
    if (a.k == K_F64 || b.k == K_F64 || (a.k == K_PY && b.k == K_PY)) {
        r.k = (a.k == K_F64 || b.k == K_F64) ? K_F64 : K_PY;
        switch (op) {
            case '+': r.v = a.v + b.v; break;
            case '-': r.v = a.v - b.v; break;
            default: r.v = a.v * b.v; break;
        }
    } else {
        float fa = (float)a.v, fb = (float)b.v, fr;
        switch (op) {
            case '+': fr = fa + fb; break;
            case '-': fr = fa - fb; break;
            default: fr = fa * fb; break;
        }
        r.k = K_F32;
        r.v = (double)fr;
    }
    return r;
}

/* ======================================================================
 * NewsvendorEnv (newsvendor.py)
 * ==================================================================== */
typedef struct {
    orc_nv_cfg c;
    int64_t n;
    uint64_t *rng;  /* [n][4] */
    double *par;    /* [n][5] price, cost, h, k, mu (Python floats) */
    float *state;   /* [n][L+5] self.state */
    int32_t *step_count;
} nv_t;

void *orc_nv_create(const orc_nv_cfg *cfg, int64_t n) {
    nv_t *h = (nv_t *)calloc(1, sizeof(nv_t));
    h->c = *cfg;
    if (h->c.lead_time < 0) h->c.lead_time = 0; /* newsvendor.py:65 max(0, lead_time) */
    h->n = n;
    h->rng = (uint64_t *)calloc((size_t)n * 4, sizeof(uint64_t));
    h->par = (double *)calloc((size_t)n * 5, sizeof(double));
    h->state = (float *)calloc((size_t)n * (h->c.lead_time + 5), sizeof(float));
    h->step_count = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    return h;
}

void orc_nv_destroy(void *p) {
    nv_t *h = (nv_t *)p;
    free(h->rng);
    free(h->par);
    free(h->state);
    free(h->step_count);
    free(h);
}

void orc_nv_seed(void *p, const uint32_t *words, const int32_t *nwords) {
    nv_t *h = (nv_t *)p;
    for (int64_t i = 0; i < h->n; i++) orc_seed_pcg64(words + 4 * i, nwords[i], h->rng + 4 * i);
}

/* newsvendor.py:100-123 */
void orc_nv_reset(void *p, float *obs) {
    nv_t *h = (nv_t *)p;
    const int O = h->c.lead_time + 5;
#pragma omp parallel for schedule(static) num_threads(orc_threads)
    for (int64_t i = 0; i < h->n; i++) {
        uint64_t *rng = h->rng + 4 * i;
        double *par = h->par + 5 * i;
        double price = orc_next_double(rng) * h->c.p_max;
        if (!(price > 1)) price = 1; /* max(1, x) */
        double cost = orc_next_double(rng) * price;
        if (!(cost > 1)) cost = 1;
        double mn = (h->c.h_max < cost) ? h->c.h_max : cost; /* min(cost, h_max) */
        double hh = orc_next_double(rng) * mn;
        double kk = orc_next_double(rng) * h->c.k_max;
        double mu = orc_next_double(rng) * h->c.mu_max;
        par[0] = price;
        par[1] = cost;
        par[2] = hh;
        par[3] = kk;
        par[4] = mu;
        float *st = h->state + (int64_t)O * i;
        for (int j = 0; j < O; j++) st[j] = 0.f;
        for (int j = 0; j < 5; j++) st[j] = (float)par[j];
        h->step_count[i] = 0;
        if (obs) memcpy(obs + (int64_t)O * i, st, sizeof(float) * O);
    }
}

void orc_nv_get_params(void *p, double *params) {
    nv_t *h = (nv_t *)p;
    memcpy(params, h->par, sizeof(double) * 5 * h->n);
}

/* numpy clip of a float64 (newsvendor.py:132): NaN propagates and a bound is
 * taken only when strictly exceeded, so np.clip(-0.0, 0, hi) stays -0.0
 * (checked against numpy in tests/test_oracle.py) */
static double np_clip(double x, double lo, double hi) {
    double y = (x < lo) ? lo : x;
    return (y > hi) ? hi : y;
}

/* newsvendor.py:125-204 */
void orc_nv_step(void *p, const float *action, float *obs, double *reward, uint8_t *truncated,
                 int64_t *demand) {
    nv_t *h = (nv_t *)p;
    const int L = h->c.lead_time;
    const int O = L + 5;
    const tv ZERO = tv_make(0.0, K_PY);
#pragma omp parallel for schedule(static) num_threads(orc_threads)
    for (int64_t i = 0; i < h->n; i++) {
        uint64_t *rng = h->rng + 4 * i;
        const double *par = h->par + 5 * i;
        float *st = h->state + (int64_t)O * i;
        h->step_count[i] += 1;                                                     /* :127 */
        tv oq = tv_make(np_clip((double)action[i], 0, h->c.max_order_quantity), K_F64); /* :131-132 */
        float S5 = orc_sum_f32(st + 5, L);                                         /* :135 */
        tv inv = (L > 0) ? tv_make((double)st[5], K_F32) : oq;                     /* :136-141 */
        tv cap = tv_bin(tv_make(h->c.max_inventory, K_PY), tv_make((double)S5, K_F32), '-');
        tv m1 = (cap.v < oq.v) ? cap : oq;                                         /* min(oq, cap) */
        tv q = (m1.v > 0) ? m1 : ZERO;                                             /* :143 max(0, .) */
        int64_t d = orc_poisson(rng, par[4]);                                      /* :146 */
        tv dv = tv_make((double)d, K_PY);
        tv sales = (dv.v < inv.v) ? dv : inv;                                      /* :149 min(inv, d) */
        tv price = tv_make(par[0], K_PY), cost = tv_make(par[1], K_PY);
        tv hh = tv_make(par[2], K_PY), kk = tv_make(par[3], K_PY);
        tv revenue = tv_bin(sales, price, '*');                                    /* :150 */
        tv ex = tv_bin(inv, dv, '-');
        tv excess = (ex.v > 0) ? ex : ZERO;                                        /* :152 */
        tv sh = tv_bin(dv, inv, '-');
        tv shortage = (sh.v > 0) ? sh : ZERO;                                      /* :153 */
        tv purchase = tv_bin(q, cost, '*');                                        /* :162 */
        tv holding = tv_bin(excess, hh, '*');                                      /* :166 */
        tv penalty = tv_bin(shortage, kk, '*');                                    /* :167 */
        tv r = tv_bin(tv_bin(tv_bin(revenue, purchase, '-'), holding, '-'), penalty, '-'); /* :170 */
        if (L > 0) {                                                               /* :174-183 */
            for (int j = 0; j < L - 1; j++) st[5 + j] = st[6 + j];
            st[5 + L - 1] = (float)q.v;
        }
        reward[i] = r.v;
        truncated[i] = (uint8_t)(h->step_count[i] >= h->c.step_limit);            /* :190 */
        if (demand) demand[i] = d;
        if (obs) memcpy(obs + (int64_t)O * i, st, sizeof(float) * O);
    }
}

/* ======================================================================
 * InvManagementMasterEnv (inventory_management.py)
 * ==================================================================== */
typedef struct {
    int32_t m, m1, T, lt_max, O, backlog, dist;
    double mu, alpha;
    int64_t dn, dlow, dhigh;
    double dp;
    uint32_t *u32; /* per env [2]: the bit generator's buffered 32-bit half */
    int64_t *I0, *c, *L, *user_D;
    double up[64], uc[64], kc[64], hc[64]; /* f32 coefficients widened exactly */
    int64_t n;
    uint64_t *rng;
    int64_t *I, *R, *B, *alog; /* per env histories */
    int32_t *period;
} im_t;

void *orc_im_create(const orc_im_cfg *cfg, int64_t n) {
    im_t *h = (im_t *)calloc(1, sizeof(im_t));
    h->m = cfg->num_stages;
    h->m1 = h->m - 1;
    h->T = cfg->periods;
    h->backlog = cfg->backlog;
    h->dist = cfg->dist;
    h->mu = cfg->mu;
    h->alpha = cfg->alpha;
    h->dn = cfg->dist_n;
    h->dp = cfg->dist_p;
    h->dlow = cfg->dist_low;
    h->dhigh = cfg->dist_high;
    h->I0 = (int64_t *)malloc(sizeof(int64_t) * h->m1);
    h->c = (int64_t *)malloc(sizeof(int64_t) * h->m1);
    h->L = (int64_t *)malloc(sizeof(int64_t) * h->m1);
    h->user_D = (int64_t *)calloc(h->T, sizeof(int64_t));
    h->lt_max = 0;
    for (int i = 0; i < h->m1; i++) {
        h->I0[i] = cfg->I0[i];
        h->c[i] = cfg->supply_capacity[i];
        h->L[i] = cfg->lead_time[i];
        if (h->L[i] > h->lt_max) h->lt_max = (int32_t)h->L[i]; /* :100 */
    }
    if (cfg->user_D)
        for (int t = 0; t < h->T; t++) h->user_D[t] = cfg->user_D[t];
    for (int j = 0; j < h->m; j++) {
        h->up[j] = (double)cfg->unit_price[j];
        h->uc[j] = (double)cfg->unit_cost[j];
        h->kc[j] = (double)cfg->demand_cost[j];
        h->hc[j] = (double)cfg->holding_cost[j];
    }
    h->O = h->m1 * (h->lt_max + 1); /* :119 */
    h->n = n;
    h->rng = (uint64_t *)calloc((size_t)n * 4, sizeof(uint64_t));
    h->I = (int64_t *)calloc((size_t)n * (h->T + 1) * h->m1, sizeof(int64_t));
    h->R = (int64_t *)calloc((size_t)n * (h->T + 1) * h->m1, sizeof(int64_t));
    h->B = (int64_t *)calloc((size_t)n * (h->T + 1) * h->m, sizeof(int64_t));
    h->alog = (int64_t *)calloc((size_t)n * (h->T + 1) * h->m1, sizeof(int64_t));
    h->period = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    h->u32 = (uint32_t *)calloc((size_t)n * 2, sizeof(uint32_t));
    return h;
}

void orc_im_destroy(void *p) {
    im_t *h = (im_t *)p;
    free(h->u32);
    free(h->I0); free(h->c); free(h->L); free(h->user_D);
    free(h->rng); free(h->I); free(h->R); free(h->B); free(h->alog); free(h->period);
    free(h);
}

void orc_im_seed(void *p, const uint32_t *words, const int32_t *nwords) {
    im_t *h = (im_t *)p;
    for (int64_t i = 0; i < h->n; i++) {
        orc_seed_pcg64(words + 4 * i, nwords[i], h->rng + 4 * i);
        h->u32[2 * i] = 0;   /* a new Generator: has_uint32 = 0 */
    }
}

/* _get_obs :354-391 */
static void im_obs(im_t *h, int64_t i, int64_t *obs) {
    const int m1 = h->m1;
    const int t = h->period[i];
    const int64_t *I = h->I + (int64_t)i * (h->T + 1) * m1;
    const int64_t *alog = h->alog + (int64_t)i * (h->T + 1) * m1;
    int64_t *o = obs + (int64_t)h->O * i;
    for (int j = 0; j < h->O; j++) o[j] = 0;
    for (int j = 0; j < m1; j++) o[j] = I[(int64_t)t * m1 + j];
    if (t > 0) {
        int npast = t < h->lt_max ? t : h->lt_max;
        for (int r = 0; r < npast; r++)
            for (int j = 0; j < m1; j++) o[m1 + r * m1 + j] = alog[(int64_t)(t - npast + r) * m1 + j];
    }
}

/* reset :186-222 (no RNG draws) */
void orc_im_reset(void *p, int64_t *obs) {
    im_t *h = (im_t *)p;
    const int m1 = h->m1, m = h->m;
#pragma omp parallel for schedule(static) num_threads(orc_threads)
    for (int64_t i = 0; i < h->n; i++) {
        int64_t *I = h->I + (int64_t)i * (h->T + 1) * m1;
        memset(I, 0, sizeof(int64_t) * (h->T + 1) * m1);
        memset(h->R + (int64_t)i * (h->T + 1) * m1, 0, sizeof(int64_t) * (h->T + 1) * m1);
        memset(h->B + (int64_t)i * (h->T + 1) * m, 0, sizeof(int64_t) * (h->T + 1) * m);
        memset(h->alog + (int64_t)i * (h->T + 1) * m1, 0, sizeof(int64_t) * (h->T + 1) * m1);
        for (int j = 0; j < m1; j++) I[j] = h->I0[j];
        h->period[i] = 0;
        if (obs) im_obs(h, i, obs);
    }
}

/* numpy int64 array arithmetic wraps around (two's complement) */
static int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

/* numpy float64 -> int64 astype of an in-range value, and np.minimum(int64, f64) */
static int64_t np_min_i64_f64(int64_t a, double b) {
    double x = (double)a;
    double r = (x <= b) ? x : b;
    return (int64_t)r;
}

/* step :224-352 */
void orc_im_step(void *p, const int64_t *action, int64_t *obs, double *reward, uint8_t *truncated,
                 int64_t *demand, int64_t *sales, int64_t *unfulfilled, int64_t *ending_inventory,
                 int64_t *backlog_next) {
    im_t *h = (im_t *)p;
    const int m1 = h->m1, m = h->m;
#pragma omp parallel for schedule(static) num_threads(orc_threads)
    for (int64_t i = 0; i < h->n; i++) {
        uint64_t *rng = h->rng + 4 * i;
        const int t = h->period[i];
        int64_t *I = h->I + (int64_t)i * (h->T + 1) * m1;
        int64_t *R = h->R + (int64_t)i * (h->T + 1) * m1;
        int64_t *B = h->B + (int64_t)i * (h->T + 1) * m;
        int64_t *alog = h->alog + (int64_t)i * (h->T + 1) * m1;
        int64_t req[64], ordreq[64], Rf[64], Icur[64], S[65], U[65];
        for (int j = 0; j < m1; j++) {
            int64_t a = action[(int64_t)i * m1 + j];
            req[j] = a > 0 ? a : 0;                                   /* :250 */
            ordreq[j] = req[j];
            if (t >= 1) ordreq[j] = wadd(ordreq[j], B[(int64_t)t * m + 1 + j]); /* :254-255 */
        }
        for (int j = 0; j < m1; j++) {
            int64_t r = ordreq[j] < h->c[j] ? ordreq[j] : h->c[j];    /* :263 */
            double sup = (j + 1 < m1) ? (double)I[(int64_t)t * m1 + j + 1] : INFINITY; /* :260 */
            Rf[j] = np_min_i64_f64(r, sup);                           /* :265 */
            R[(int64_t)t * m1 + j] = Rf[j];                           /* :267 */
            alog[(int64_t)t * m1 + j] = req[j];                       /* :268 */
        }
        for (int j = 0; j < m1; j++) {                                /* :271-277 */
            Icur[j] = I[(int64_t)t * m1 + j];
            if (t - h->L[j] >= 0) Icur[j] = wadd(Icur[j], R[(int64_t)(t - h->L[j]) * m1 + j]);
        }
        int64_t d;
        if (h->dist == 5)
            d = t < h->T ? h->user_D[t] : 0;                          /* :182 */
        else if (h->dist == 2)
            d = orc_binomial(rng, h->dn, h->dp);                      /* :175 */
        else if (h->dist == 3)
            d = orc_integers(rng, h->u32 + 2 * i, h->dlow, h->dhigh + 1); /* :178 */
        else if (h->dist == 4)
            d = orc_geometric(rng, h->dp);                            /* :181 */
        else
            d = orc_poisson(rng, h->mu);                              /* :172 */
        if (d < 0) d = 0;                                             /* :280 */
        int64_t dfill = d;
        if (t >= 1) dfill = wadd(dfill, B[(int64_t)t * m + 0]);       /* :285-286 */
        int64_t s0 = Icur[0] < dfill ? Icur[0] : dfill;               /* :288 */
        Icur[0] = wsub(Icur[0], s0);
        S[0] = s0;
        for (int j = 0; j < m1; j++) S[j + 1] = Rf[j];                /* :295 */
        for (int j = 1; j < m1; j++) Icur[j] = wsub(Icur[j], Rf[j]);  /* :300 (reference quirk) */
        U[0] = wsub(dfill, s0);                                       /* :303 */
        for (int j = 0; j < m1; j++) U[j + 1] = wsub(ordreq[j], Rf[j]); /* :304 */
        for (int j = 0; j < m; j++) B[(int64_t)(t + 1) * m + j] = h->backlog ? U[j] : 0; /* :307-312 */
        double terms[65];
        for (int j = 0; j < m; j++) {                                 /* :315-321 */
            double Sj = (double)S[j];
            int64_t inv = (j < m1) ? Icur[j] : 0;
            double hold = h->hc[j] * (double)(inv > 0 ? inv : 0);
            terms[j] = ((h->up[j] * Sj - h->uc[j] * Sj) - hold) - h->kc[j] * (double)U[j];
        }
        double profit = orc_sum_f64(terms, m);
        double disc = pow(h->alpha, (double)t) * profit;             /* :322 */
        for (int j = 0; j < m1; j++) I[(int64_t)(t + 1) * m1 + j] = Icur[j]; /* :326 */
        h->period[i] = t + 1;
        reward[i] = disc;
        truncated[i] = (uint8_t)(h->period[i] >= h->T);               /* :350 */
        if (obs) im_obs(h, i, obs);
        if (demand) demand[i] = d;
        if (sales) for (int j = 0; j < m; j++) sales[(int64_t)i * m + j] = S[j];
        if (unfulfilled) for (int j = 0; j < m; j++) unfulfilled[(int64_t)i * m + j] = U[j];
        if (ending_inventory) for (int j = 0; j < m1; j++) ending_inventory[(int64_t)i * m1 + j] = Icur[j];
        if (backlog_next) for (int j = 0; j < m; j++) backlog_next[(int64_t)i * m + j] = B[(int64_t)(t + 1) * m + j];
    }
}

/* ======================================================================
 * NetInvMgmtMasterEnv (network_management.py)
 * ==================================================================== */
typedef struct {
    orc_net_cfg c; /* pointers copied below */
    int32_t J, E, RL, T, O, backlog;
    double alpha;
    double *I0, *h, *C, *o, *v;
    int32_t *is_factory, *is_retail, *sup, *pur, *L, *sup_is_factory, *rl_node, *rl_user;
    double *lp, *lg, *rl_p, *rl_b, *rl_lam, *user_D;
    int32_t *succ_n, *succ_kind, *succ_idx, *pred_n, *pred_idx;
    int32_t *rl_dist;
    int64_t *rl_n, *rl_high;
    double *rl_dp;
    int64_t n;
    uint64_t *rng;
    uint32_t *u32; /* per env [2]: the bit generator's buffered 32-bit half (integers markets) */
    double *X, *Y, *R, *S, *U, *D;
    int32_t *period;
} net_t;

#define DUP(dst, src, cnt, ty)                                  \
    do {                                                        \
        dst = (ty *)calloc((size_t)((cnt) > 0 ? (cnt) : 1), sizeof(ty)); \
        if (src) memcpy(dst, src, sizeof(ty) * (size_t)(cnt));  \
    } while (0)

void *orc_net_create(const orc_net_cfg *cfg, int64_t n) {
    net_t *h = (net_t *)calloc(1, sizeof(net_t));
    h->J = cfg->J;
    h->E = cfg->E;
    h->RL = cfg->RL;
    h->T = cfg->num_periods;
    h->backlog = cfg->backlog;
    h->alpha = cfg->alpha;
    DUP(h->I0, cfg->I0, h->J, double);
    DUP(h->h, cfg->h, h->J, double);
    DUP(h->C, cfg->C, h->J, double);
    DUP(h->o, cfg->o, h->J, double);
    DUP(h->v, cfg->v, h->J, double);
    DUP(h->is_factory, cfg->is_factory, h->J, int32_t);
    DUP(h->is_retail, cfg->is_retail, h->J, int32_t);
    DUP(h->sup, cfg->sup, h->E, int32_t);
    DUP(h->pur, cfg->pur, h->E, int32_t);
    DUP(h->L, cfg->L, h->E, int32_t);
    DUP(h->sup_is_factory, cfg->sup_is_factory, h->E, int32_t);
    DUP(h->lp, cfg->lp, h->E, double);
    DUP(h->lg, cfg->lg, h->E, double);
    DUP(h->rl_node, cfg->rl_node, h->RL, int32_t);
    DUP(h->rl_p, cfg->rl_p, h->RL, double);
    DUP(h->rl_b, cfg->rl_b, h->RL, double);
    DUP(h->rl_lam, cfg->rl_lam, h->RL, double);
    DUP(h->rl_user, cfg->rl_user, h->RL, int32_t);
    DUP(h->user_D, cfg->user_D, h->RL * h->T, double);
    DUP(h->succ_n, cfg->succ_n, h->J, int32_t);
    DUP(h->succ_kind, cfg->succ_kind, h->J * ORC_NET_MAXADJ, int32_t);
    DUP(h->succ_idx, cfg->succ_idx, h->J * ORC_NET_MAXADJ, int32_t);
    DUP(h->pred_n, cfg->pred_n, h->J, int32_t);
    DUP(h->pred_idx, cfg->pred_idx, h->J * ORC_NET_MAXADJ, int32_t);
    DUP(h->rl_dist, cfg->rl_dist, h->RL, int32_t);
    if (!cfg->rl_dist)
        for (int r = 0; r < h->RL; r++) h->rl_dist[r] = 1;
    DUP(h->rl_n, cfg->rl_n, h->RL, int64_t);
    DUP(h->rl_high, cfg->rl_high, h->RL, int64_t);
    DUP(h->rl_dp, cfg->rl_dp, h->RL, double);
    int sumL = 0;
    for (int e = 0; e < h->E; e++) sumL += h->L[e];
    h->O = h->RL + h->J + sumL; /* :188-190 */
    h->n = n;
    h->rng = (uint64_t *)calloc((size_t)n * 4, sizeof(uint64_t));
    h->u32 = (uint32_t *)calloc((size_t)n * 2, sizeof(uint32_t));
    h->X = (double *)calloc((size_t)n * (h->T + 2) * h->J, sizeof(double));
    h->Y = (double *)calloc((size_t)n * (h->T + 2) * (h->E ? h->E : 1), sizeof(double));
    h->R = (double *)calloc((size_t)n * (h->T + 2) * (h->E ? h->E : 1), sizeof(double));
    h->S = (double *)calloc((size_t)n * (h->T + 2) * (h->E + h->RL + 1), sizeof(double));
    h->U = (double *)calloc((size_t)n * (h->T + 2) * (h->RL ? h->RL : 1), sizeof(double));
    h->D = (double *)calloc((size_t)n * (h->T + 2) * (h->RL ? h->RL : 1), sizeof(double));
    h->period = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    return h;
}

void orc_net_destroy(void *p) {
    net_t *h = (net_t *)p;
    free(h->I0); free(h->h); free(h->C); free(h->o); free(h->v);
    free(h->is_factory); free(h->is_retail); free(h->sup); free(h->pur); free(h->L);
    free(h->sup_is_factory); free(h->lp); free(h->lg); free(h->rl_node); free(h->rl_p);
    free(h->rl_b); free(h->rl_lam); free(h->rl_user); free(h->user_D); free(h->succ_n);
    free(h->succ_kind); free(h->succ_idx); free(h->pred_n); free(h->pred_idx);
    free(h->rl_dist); free(h->rl_n); free(h->rl_high); free(h->rl_dp); free(h->u32);
    free(h->rng); free(h->X); free(h->Y); free(h->R); free(h->S); free(h->U); free(h->D);
    free(h->period);
    free(h);
}

int32_t orc_net_obs_dim(void *p) { return ((net_t *)p)->O; }

void orc_net_seed(void *p, const uint32_t *words, const int32_t *nwords) {
    net_t *h = (net_t *)p;
    for (int64_t i = 0; i < h->n; i++) {
        orc_seed_pcg64(words + 4 * i, nwords[i], h->rng + 4 * i);
        h->u32[2 * i] = 0;   /* a new Generator: has_uint32 = 0 */
    }
}

#define NX(h, i) ((h)->X + (int64_t)(i) * ((h)->T + 2) * (h)->J)
#define NY(h, i) ((h)->Y + (int64_t)(i) * ((h)->T + 2) * ((h)->E ? (h)->E : 1))
#define NR(h, i) ((h)->R + (int64_t)(i) * ((h)->T + 2) * ((h)->E ? (h)->E : 1))
#define NS(h, i) ((h)->S + (int64_t)(i) * ((h)->T + 2) * ((h)->E + (h)->RL + 1))
#define NU(h, i) ((h)->U + (int64_t)(i) * ((h)->T + 2) * ((h)->RL ? (h)->RL : 1))
#define ND(h, i) ((h)->D + (int64_t)(i) * ((h)->T + 2) * ((h)->RL ? (h)->RL : 1))

/* _get_obs :334-413 */
static void net_obs(net_t *h, int64_t i, float *obs) {
    const int t = h->period[i];
    const int E = h->E ? h->E : 1, RLs = h->RL ? h->RL : 1;
    float *o = obs + (int64_t)h->O * i;
    int k = 0;
    for (int r = 0; r < h->RL; r++) o[k++] = (float)NU(h, i)[(int64_t)t * RLs + r];
    for (int j = 0; j < h->J; j++) o[k++] = (float)NX(h, i)[(int64_t)t * h->J + j];
    for (int e = 0; e < h->E; e++) {
        int L = h->L[e];
        if (L == 0) continue;
        int start = t - L > 0 ? t - L : 0;
        if (start > h->T - 1) start = h->T - 1;
        int end = t < h->T ? t : h->T;
        float *pad = o + k;
        for (int q = 0; q < L; q++) pad[q] = 0.f;
        int cnt = end - start;
        if (cnt > 0)
            for (int q = 0; q < cnt; q++) pad[L - cnt + q] = (float)NR(h, i)[(int64_t)(start + q) * E + e];
        k += L;
    }
}

/* reset :301-332 (no RNG draws) */
void orc_net_reset(void *p, float *obs) {
    net_t *h = (net_t *)p;
    const int E = h->E ? h->E : 1, RLs = h->RL ? h->RL : 1;
#pragma omp parallel for schedule(static) num_threads(orc_threads)
    for (int64_t i = 0; i < h->n; i++) {
        memset(NX(h, i), 0, sizeof(double) * (h->T + 2) * h->J);
        memset(NY(h, i), 0, sizeof(double) * (h->T + 2) * E);
        memset(NR(h, i), 0, sizeof(double) * (h->T + 2) * E);
        memset(NS(h, i), 0, sizeof(double) * (h->T + 2) * (h->E + h->RL + 1));
        memset(NU(h, i), 0, sizeof(double) * (h->T + 2) * RLs);
        memset(ND(h, i), 0, sizeof(double) * (h->T + 2) * RLs);
        for (int j = 0; j < h->J; j++) NX(h, i)[j] = h->I0[j];
        h->period[i] = 0;
        if (obs) net_obs(h, i, obs);
    }
}

static double py_max0(double x) { return (x > 0) ? x : 0.0; } /* max(0, x) */

/* step :436-635 */
void orc_net_step(void *p, const float *action, float *obs, double *reward, uint8_t *truncated,
                  double *Xo, double *Uo, double *Do, double *Ro, double *Yo, double *Po, double *So) {
    net_t *h = (net_t *)p;
    const int J = h->J, EE = h->E, RL = h->RL;
    const int E = EE ? EE : 1, RLs = RL ? RL : 1, SL = h->E + h->RL + 1;
    double cons[64], arr[64], xb[64], prof[64];
#pragma omp parallel for schedule(static) num_threads(orc_threads) private(cons, arr, xb, prof)
    for (int64_t i = 0; i < h->n; i++) {
        uint64_t *rng = h->rng + 4 * i;
        const int t = h->period[i];
        double *X = NX(h, i), *Y = NY(h, i), *R = NR(h, i), *S = NS(h, i), *U = NU(h, i), *D = ND(h, i);
        for (int j = 0; j < J; j++) cons[j] = 0.0, arr[j] = 0.0;
        /* 0) orders, sorted reorder links :448-490 */
        for (int e = 0; e < EE; e++) {
            double raw = (double)action[(int64_t)i * EE + e];
            double rq = nearbyint(raw);                   /* round() half-to-even */
            double request = (rq > 0) ? rq : 0.0;         /* max(0, .) */
            double f;
            int s = h->sup[e];
            if (s < 0) {
                f = request;                              /* raw material: unlimited */
            } else {
                double avail = X[(int64_t)t * J + s] - cons[s];
                double oav = py_max0(avail);
                double order_available = oav;
                if (h->sup_is_factory[e]) {
                    double mpi = h->v[s] * oav;
                    double mp = (mpi < h->C[s]) ? mpi : h->C[s]; /* min(C, mpi) */
                    order_available = (mp < order_available) ? mp : order_available;
                }
                f = (order_available < request) ? order_available : request; /* min(request, avail) */
                cons[s] += f / h->v[s];                  /* v = node.get('v', 1.0) */
            }
            R[(int64_t)t * E + e] = f;
            S[(int64_t)t * SL + e] = f;
        }
        /* 1) pipeline :494-511 */
        for (int e = 0; e < EE; e++) {
            int L = h->L[e];
            double arrv = 0.0;
            if (t - L >= 0 && t - L < h->T) arrv = R[(int64_t)(t - L) * E + e];
            Y[(int64_t)(t + 1) * E + e] = Y[(int64_t)t * E + e] - arrv + R[(int64_t)t * E + e];
        }
        /* arrivals :516-523 */
        for (int j = 0; j < J; j++) {
            for (int q = 0; q < h->pred_n[j]; q++) {
                int e = h->pred_idx[j * ORC_NET_MAXADJ + q];
                int L = h->L[e];
                if (t - L >= 0 && t - L < h->T) arr[j] += R[(int64_t)(t - L) * E + e];
            }
        }
        for (int j = 0; j < J; j++) X[(int64_t)(t + 1) * J + j] = X[(int64_t)t * J + j] + arr[j] - cons[j]; /* :528 */
        /* 2&3) market :536-566 */
        for (int j = 0; j < J; j++) xb[j] = X[(int64_t)(t + 1) * J + j];
        for (int r = 0; r < RL; r++) {
            double dd;
            if (h->rl_user[r]) {
                int idx = t < h->T - 1 ? t : h->T - 1;
                dd = h->user_D[(int64_t)r * h->T + idx];
                dd = nearbyint(dd);                        /* max(0, int(round(x))) */
                if (!(dd > 0)) dd = 0.0;
            } else {                                       /* max(0, int(round(f(**p)))) :263 */
                int64_t pd;
                switch (h->rl_dist[r]) {
                    case 2: pd = orc_binomial(rng, h->rl_n[r], h->rl_dp[r]); break;
                    case 3: pd = orc_integers(rng, h->u32 + 2 * i, h->rl_n[r], h->rl_high[r]); break;
                    case 4: pd = orc_geometric(rng, h->rl_dp[r]); break;
                    default: pd = orc_poisson(rng, h->rl_lam[r]);
                }
                dd = (double)(pd > 0 ? pd : 0);
            }
            D[(int64_t)t * RLs + r] = dd;
            double fill = dd + U[(int64_t)t * RLs + r];
            int node = h->rl_node[r];
            double inv = py_max0(xb[node]);
            double sale = (inv < fill) ? inv : fill;       /* min(fill, inv) */
            S[(int64_t)t * SL + EE + r] = sale;
            if (So) So[i * RLs + r] = sale;
            xb[node] -= sale;
            double unf = fill - sale;
            U[(int64_t)(t + 1) * RLs + r] = h->backlog ? unf : 0.0;
        }
        for (int j = 0; j < J; j++) X[(int64_t)(t + 1) * J + j] = xb[j]; /* :571 */
        /* 5) profit :578-613 */
        double total = 0.0;
        for (int j = 0; j < J; j++) {
            double SR = 0.0, PC = 0.0, HCp = 0.0, OC = 0.0, UP = 0.0, sold = 0.0;
            for (int q = 0; q < h->succ_n[j]; q++) {
                int kind = h->succ_kind[j * ORC_NET_MAXADJ + q], idx = h->succ_idx[j * ORC_NET_MAXADJ + q];
                double pr = kind == 0 ? h->lp[idx] : h->rl_p[idx];
                double sv = kind == 0 ? S[(int64_t)t * SL + idx] : S[(int64_t)t * SL + EE + idx];
                SR += pr * sv;
            }
            for (int q = 0; q < h->pred_n[j]; q++) {
                int e = h->pred_idx[j * ORC_NET_MAXADJ + q];
                PC += h->lp[e] * R[(int64_t)t * E + e];
            }
            double HC_on = h->h[j] * py_max0(X[(int64_t)(t + 1) * J + j]);
            for (int q = 0; q < h->pred_n[j]; q++) {
                int e = h->pred_idx[j * ORC_NET_MAXADJ + q];
                HCp += h->lg[e] * py_max0(Y[(int64_t)(t + 1) * E + e]);
            }
            double HC = HC_on + HCp;
            if (h->is_factory[j]) {
                for (int q = 0; q < h->succ_n[j]; q++) {
                    int kind = h->succ_kind[j * ORC_NET_MAXADJ + q], idx = h->succ_idx[j * ORC_NET_MAXADJ + q];
                    sold += kind == 0 ? S[(int64_t)t * SL + idx] : S[(int64_t)t * SL + EE + idx];
                }
                OC = (h->v[j] > 0) ? h->o[j] * (sold / h->v[j]) : 0.0;
            }
            if (h->is_retail[j]) {
                for (int q = 0; q < h->succ_n[j]; q++) {
                    if (h->succ_kind[j * ORC_NET_MAXADJ + q] != 1) continue;
                    int r = h->succ_idx[j * ORC_NET_MAXADJ + q];
                    UP += h->rl_b[r] * U[(int64_t)(t + 1) * RLs + r];
                }
            }
            double np_ = SR - PC - OC - HC - UP;
            prof[j] = np_;
            total += np_;
        }
        double disc = pow(h->alpha, (double)t) * total; /* :619 */
        h->period[i] = t + 1;
        reward[i] = disc;
        truncated[i] = (uint8_t)(h->period[i] >= h->T);
        if (obs) net_obs(h, i, obs);
        if (Xo) for (int j = 0; j < J; j++) Xo[(int64_t)i * J + j] = X[(int64_t)(t + 1) * J + j];
        if (Uo) for (int r = 0; r < RL; r++) Uo[(int64_t)i * RL + r] = U[(int64_t)(t + 1) * RLs + r];
        if (Do) for (int r = 0; r < RL; r++) Do[(int64_t)i * RL + r] = D[(int64_t)t * RLs + r];
        if (Ro) for (int e = 0; e < EE; e++) Ro[(int64_t)i * EE + e] = R[(int64_t)t * E + e];
        if (Yo) for (int e = 0; e < EE; e++) Yo[(int64_t)i * EE + e] = Y[(int64_t)(t + 1) * E + e];
        if (Po) for (int j = 0; j < J; j++) Po[(int64_t)i * J + j] = prof[j];
    }
}

/* ======================================================================
 * Generator states (test access: the final PCG64 state of every stream is
 * compared with the device's after long runs)
 * ==================================================================== */
void orc_nv_rng(void *p, uint64_t *out /*[n][4]*/) {
    nv_t *h = (nv_t *)p;
    memcpy(out, h->rng, sizeof(uint64_t) * 4 * (size_t)h->n);
}

void orc_im_rng(void *p, uint64_t *out) {
    im_t *h = (im_t *)p;
    memcpy(out, h->rng, sizeof(uint64_t) * 4 * (size_t)h->n);
}

void orc_net_rng(void *p, uint64_t *out) {
    net_t *h = (net_t *)p;
    memcpy(out, h->rng, sizeof(uint64_t) * 4 * (size_t)h->n);
}
