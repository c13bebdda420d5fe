"""Tree statistics of a render scene's BVH (CPU only): node kinds, the
one-sided chains the reference's SAH fallback builds, and the surface-area
cost of the reference tree, of the chain-collapsed tree the walks use, and of
a fresh binned-SAH tree over the same live leaves -- how much a different
walk topology could save (the closest-hit rule is topology-free).

  python scripts/tree_stats.py [--n 10000] [--bench] [--bins 32]
"""
import argparse
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def area(lo, hi):
    d = np.maximum(hi - lo, 0)
    return 2 * (d[..., 0] * d[..., 1] + d[..., 1] * d[..., 2] + d[..., 2] * d[..., 0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--bench", action="store_true", help="benchmark.c scene (S_bench) instead of main.c's")
    ap.add_argument("--bins", type=int, default=32)
    a = ap.parse_args()
    m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
    s = m.create_benchmark_spheres(a.n, 1) if a.bench else m.create_random_spheres(a.n, 1)
    nd = m.build_bvh(s).nodes
    nn = len(nd)
    sph = nd["sphere"]
    skip = nd["skip"] & 0x7FFFFFFF
    empty = (nd["skip"] & 0x80000000) != 0
    lo = nd["bmin"].astype(np.float64)
    hi = nd["bmax"].astype(np.float64)
    leaf = sph >= 0
    dead = leaf & (empty | (sph >= a.n))
    inner = ~leaf
    left = np.arange(nn) + 1
    right = np.zeros(nn, np.int64)
    right[inner] = skip[left[inner]]
    chain = np.zeros(nn, bool)
    chain[inner] = dead[left[inner]] ^ dead[right[inner]]
    A = area(lo, hi)
    root = A[0]
    ref_cost = (A[inner].sum() + A[leaf & ~dead].sum()) / root
    live_inner = inner & ~chain
    col_cost = (A[live_inner].sum() + A[leaf & ~dead].sum()) / root
    depth = np.zeros(nn, np.int64)
    for i in range(nn):
        if inner[i]:
            depth[left[i]] = depth[right[i]] = depth[i] + 1
    print(f"nodes {nn}  inner {inner.sum()}  leaves {leaf.sum()} (dead {dead.sum()})  chain nodes {chain.sum()}  "
          f"max depth {depth.max()}  mean live-leaf depth {depth[leaf & ~dead].mean():.1f}")
    # fresh binned SAH over the live leaves' boxes (centroid bins, leaf = 1)
    L = np.nonzero(leaf & ~dead)[0]
    blo, bhi = lo[L], hi[L]
    cen = 0.5 * (blo + bhi)
    tot = [0.0]

    def build(idx):
        bl, bh = blo[idx].min(0), bhi[idx].max(0)
        if len(idx) == 1:
            tot[0] += area(bl, bh)
            return
        tot[0] += area(bl, bh)
        c = cen[idx]
        cl, ch = c.min(0), c.max(0)
        best = (np.inf, None)
        for ax in range(3):
            ext = ch[ax] - cl[ax]
            if ext <= 0:
                continue
            b = np.minimum(((c[:, ax] - cl[ax]) / ext * a.bins).astype(np.int64), a.bins - 1)
            cnt = np.bincount(b, minlength=a.bins)
            blo_b = np.full((a.bins, 3), np.inf)
            bhi_b = np.full((a.bins, 3), -np.inf)
            np.minimum.at(blo_b, b, blo[idx])
            np.maximum.at(bhi_b, b, bhi[idx])
            llo = np.minimum.accumulate(blo_b, 0)
            lhi = np.maximum.accumulate(bhi_b, 0)
            rlo = np.minimum.accumulate(blo_b[::-1], 0)[::-1]
            rhi = np.maximum.accumulate(bhi_b[::-1], 0)[::-1]
            nl = np.cumsum(cnt)
            for k in range(a.bins - 1):
                if nl[k] == 0 or nl[k] == len(idx):
                    continue
                cost = nl[k] * area(llo[k], lhi[k]) + (len(idx) - nl[k]) * area(rlo[k + 1], rhi[k + 1])
                if cost < best[0]:
                    best = (cost, (ax, b <= k))
        if best[1] is None:
            h = len(idx) // 2
            build(idx[:h])
            build(idx[h:])
            return
        msk = best[1][1]
        build(idx[msk])
        build(idx[~msk])

    sys.setrecursionlimit(100000)
    build(np.arange(len(L)))
    print(f"SAH cost (node + leaf areas / root area): reference {ref_cost:.1f}  collapsed {col_cost:.1f}  "
          f"fresh binned ({a.bins} bins) {tot[0] / root:.1f}")


if __name__ == "__main__":
    main()
