"""The error bound behind closest-hit pruning (csrc/trace.h, struct Prune).

A sphere hit that hit.c:19-39 records at t lies, as the exact point o + t d,
within 2^-9.3 max(|o - c|, r) <= 2^-9.3 (t|d| + r + ...) of the sphere's
surface (analysis in trace.h); the kernel grows boxes by 2^-8 (best |d| +
r_max), or before any hit by 2^-7 (|o|_inf + c_max). This sweeps the reference's
float32 arithmetic (numpy float32 is IEEE with no contraction, the same
operation order as hit.c:19-39 with hit.c:28 in double) over random and
grazing configurations, including unnormalised directions, and checks the
observed distance stays well inside the bound.
"""
import numpy as np

F = np.float32


def _dot(a, b):
    return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]


def _sweep(rng, n, grazing, unnormalised, radii):
    c = rng.uniform(-60, 60, (n, 3)).astype(F)
    r = radii(n).astype(F)
    o = rng.uniform(-60, 60, (n, 3)).astype(F)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    k = rng.uniform(0.95, 1.05, n) if grazing else rng.uniform(0.0, 1.2, n)
    d = c.astype(np.float64) + u * (k * r)[:, None] - o
    d /= np.linalg.norm(d, axis=1)[:, None]
    if unnormalised:
        d *= rng.uniform(0.1, 10.0, n)[:, None]
    d = d.astype(F)
    oc = o - c
    a = _dot(d, d)
    b = F(2) * _dot(oc, d)
    cc = _dot(oc, oc) - r * r
    disc = b * b - (F(4) * a) * cc
    ok = disc > 0
    with np.errstate(invalid="ignore"):
        num = (-b).astype(np.float64) - np.sqrt(disc.astype(np.float64))
    t = (num / (F(2) * a).astype(np.float64)).astype(F)
    ok &= t > F(1e-6)
    p = o.astype(np.float64) + t.astype(np.float64)[:, None] * d.astype(np.float64)
    dist = np.abs(np.linalg.norm(p - c.astype(np.float64), axis=1) - r.astype(np.float64))
    scale = t.astype(np.float64) * np.sqrt(a.astype(np.float64)) + r.astype(np.float64)
    m_geo = np.maximum(np.linalg.norm(oc.astype(np.float64), axis=1), r.astype(np.float64))
    return (dist / scale)[ok], (dist / m_geo)[ok]


def test_hit_point_error_inside_prune_margin():
    rng = np.random.default_rng(1)
    worst = worst_m = 0.0
    for grazing in (True, False):
        for unnorm in (False, True):
            for radii in (lambda n: rng.uniform(0.5, 5.0, n), lambda n: 10 ** rng.uniform(-3, 3, n)):
                ratio, ratio_m = _sweep(rng, 400_000, grazing, unnorm, radii)
                assert ratio.size > 1000
                worst = max(worst, float(ratio.max()))
                worst_m = max(worst_m, float(ratio_m.max()))
    # analysis: D < 2^-9.3 M with M = max(|o - c|, r) <= t|d| + r + D; the
    # kernel grows boxes by 2^-8 (best |d| + r_max), or by 2^-7 (|o| + c_max)
    # >= 2^-8 M before any hit (prune_m0)
    assert worst < 2.0 ** -9.3, worst
    assert worst_m < 2.0 ** -9.3, worst_m
