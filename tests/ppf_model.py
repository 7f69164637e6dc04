"""Python model of the device poisson.ppf (newsvendor.hip nv_poisson_ppf), the
spec the HIP code follows step for step.  TEST INFRASTRUCTURE: checked against
the third-party scipy.stats.poisson.ppf (scipy 1.15.3, as the reference's
ClassicNewsvendorAgent / sSPolicyAgent call it) in tests/test_policies.py.
"""
import math

import numpy as np

f32 = np.float32


def dpois_raw(x, lam):
    # exp(-stirlerr(x) - bd0(x, lam)) / sqrt(2 pi x), x > 35
    nn = x * x
    S0, S1, S2, S3 = 1 / 12, 1 / 360, 1 / 1260, 1 / 1680
    if x > 500:
        st = (S0 - S1 / nn) / x
    elif x > 80:
        st = (S0 - (S1 - S2 / nn) / nn) / x
    else:
        st = (S0 - (S1 - (S2 - S3 / nn) / nn) / nn) / x
    d = x - lam
    if abs(d) < 0.1 * (x + lam):
        v = d / (x + lam)
        s = d * v
        ej = 2 * x * v
        v = v * v
        j = 1
        while True:
            ej *= v
            s1 = s + ej / (2 * j + 1)
            if s1 == s:
                break
            s = s1
            j += 1
        bd = s1
    else:
        bd = x * math.log(x / lam) + lam - x
    return math.exp(-st - bd) / math.sqrt(2 * math.pi * x)


def igamc(a, x):
    """Q(a, x), a > 0 real, x > 0 (series / Lentz continued fraction)."""
    lpre = -x + a * math.log(x) - math.lgamma(a)
    if x < a + 1:
        s = 1.0 / a
        d = s
        n = 1
        while n < 100000:
            d *= x / (a + n)
            s += d
            if abs(d) < abs(s) * 1e-17:
                break
            n += 1
        return 1.0 - s * math.exp(lpre)
    tiny = 1e-300
    b = x + 1 - a
    c = 1 / tiny
    d = 1 / b
    h = d
    i = 1
    while i < 100000:
        an = -i * (i - a)
        b += 2
        d = an * d + b
        if abs(d) < tiny:
            d = tiny
        c = b + an / c
        if abs(c) < tiny:
            c = tiny
        d = 1 / d
        de = d * c
        h *= de
        if abs(de - 1) < 1e-16:
            break
        i += 1
    return math.exp(lpre) * h


def ppf(q, lam, single):
    """scipy.stats.poisson.ppf(q, lam); single: q and lam are float32 (the
    f32 ufunc loops of pdtrik / pdtr)."""
    if math.isnan(q):
        return math.nan
    if q == 0:
        return -1.0
    if q == 1:
        return math.inf
    if not (0 < q < 1):
        return math.nan
    if not (lam <= 1e7):
        return math.nan
    sd = math.sqrt(lam)
    i0 = math.floor(lam - 20 * sd) if lam > 700 else 0
    i0 = max(i0, 0)
    p = math.exp(-lam) if i0 == 0 else dpois_raw(i0, lam)
    P = p
    j = i0
    Pm1 = Pm2 = 0.0   # CDF(j-1), CDF(j-2)
    jmax = lam + 40 * sd + 64
    while P < q and j < jmax:
        j += 1
        p = p * lam / j
        Pm2, Pm1 = Pm1, P
        P += p
    if not single:
        return float(j)                 # float64 loops: exact j*
    vals = j
    if j >= 2:
        e = math.floor(math.log2(j - 1))
        half = 2.0 ** (e - 24)          # half an f32 ulp at j - 1
        if igamc(j + half, lam) > q:    # x* < j - 1 + half: f32(x*) == j - 1
            vals = j - 1
    vals1 = vals - 1 if vals > 1 else 0
    c = P if vals1 == j else Pm1 if vals1 == j - 1 else Pm2 if vals1 == j - 2 else 0.0
    return float(vals1) if f32(c) >= f32(q) else float(vals)
