"""Generate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Runs only in the build container, where /root/reference exists: it builds
oracle/_ref/libref_<W>x<H>.so (the unmodified reference hot-path sources +
oracle/ref_harness.c, see oracle/Makefile) and records what the reference
computes. Nothing here uses the oracle restatement or the product; the tests
then check both of those against these vectors.

    python tests/golden/make_golden.py          # ~3-4 min on one core

Outputs (data only: inputs and the reference's outputs):
  golden.json     rand() streams, contract draws, tree stats and SHA-256 of
                  large scenes / trees / framebuffers, camera-ray bit patterns
  small.npz       scenes (pre/post build), flattened trees, per-ray hit
                  records, small framebuffers
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.lib import Reference, abi, build  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def tree_stats(flat, leaf_counts, n_spheres):
    """node / leaf / empty-leaf / multi-sphere-leaf counts and max depth."""
    n = len(flat)
    leaf = flat["sphere"] >= 0
    empty = (flat["skip"] & abi.NODE_EMPTY) != 0
    depth = np.zeros(n, np.int32)
    skip = flat["skip"] & abi.SKIP_MASK
    # pre-order: children of inner node i are i+1 and the node at the end of
    # the left subtree (skip of i+1)
    for i in range(n):
        if not leaf[i]:
            depth[i + 1] = depth[i] + 1
            depth[skip[i + 1]] = depth[i] + 1
    return {"nodes": int(n), "leaves": int(leaf.sum()), "empty_leaves": int(empty.sum()),
            "multi_leaves": int((leaf_counts > 1).sum()), "max_depth": int(depth.max()),
            "sentinel_leaves": int((flat["sphere"] == n_spheres).sum())}


def random_rays(rng, n, lo, hi):
    rays = np.zeros(n, abi.RAY)
    rays["origin"] = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    rays["direction"] = d
    return rays


def edge_rays(spheres, rng):
    """Zero / negative-zero direction components, origins inside spheres,
    rays through sphere centres, tangent (grazing) rays, zero direction."""
    out = []

    def add(o, d):
        r = np.zeros(1, abi.RAY)
        r["origin"] = np.asarray(o, np.float32)
        r["direction"] = np.asarray(d, np.float32)
        out.append(r)

    cam = (0.0, 4.0, 50.0)
    for d in [(0, 0, -1), (1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0.6, 0, -0.8),
              (0, 0.6, -0.8), (-0.0, 0.0, -1.0), (0.0, -0.0, -1.0), (0, 0, 0), (1e-30, 0, -1)]:
        add(cam, d)
        add((0, 0, 0), d)
    for s in spheres[:48]:
        c = s["center"].astype(np.float32)
        r = np.float32(s["radius"])
        add(c, (0, 0, -1))                                    # origin at a centre
        add(c + np.float32([0, 0, r * 0.5]), (0.0, 0.0, 1.0))  # origin inside
        o = np.float32([0, 4, 50])
        d = (c - o)
        add(o, d / np.float32(np.linalg.norm(d)))            # aimed at the centre
        add(c + np.float32([r, 0, 20]), (0, 0, -1))          # tangent in x
        add(c + np.float32([0, r, -20]), (0, 0, 1))          # tangent in y
        add(c + np.float32([np.nextafter(r, np.float32(0)), 0, 20]), (0, 0, -1))
        add(c + np.float32([-r, 0, 0]) - np.float32([5, 0, 0]), (1, 0, 0))  # hits box face
    rays = np.concatenate(out)
    return rays


def main():
    t0 = time.time()
    build(ref=True)
    G = {"generated_by": "tests/golden/make_golden.py from oracle/_ref (unmodified reference sources)"}
    S = {}
    r160 = Reference(160, 90)
    L = r160.L
    G["sizeof"] = {"Sphere": L.h_sizeof_sphere(), "BVHNode": L.h_sizeof_node(),
                   "HitRecord": L.h_sizeof_hit(), "Camera": L.h_sizeof_camera()}

    # glibc rand() streams (the reference's only RNG, vec3.c:64-69, sphere.c:14-16)
    G["rand"] = {}
    for seed in [0, 1, 2, 12345, 2**31 + 5, 4294967295]:
        L.h_srand(seed)
        G["rand"][str(seed)] = [L.h_rand() for _ in range(400)]

    # per-pixel contract draws: what the interposed rand() returns
    import ctypes as C
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle.lib import Oracle  # the contract lives in oracle/rng_contract.h (shared by harness and oracle)
    o = Oracle()
    G["contract"] = [[seed, px, smp, k, o.contract_draw(seed, px, smp, k)]
                     for seed in [1, 7, 2**40 + 3] for px in [0, 1, 2073599, 123457]
                     for smp in [0, 1, 3] for k in [0, 1, 2, 9, 31]]

    # scenes and trees (sphere.c:52-59 via main.c:218-221; bvh.c:117-209)
    G["scenes"] = {}
    for seed in [1, 2]:
        for n in [20, 100, 1000]:
            s = r160.render_scene(seed, n)
            S[f"render_{n}_{seed}_pre"] = s.copy()
            t = r160.build(s)
            S[f"render_{n}_{seed}_post"] = s.copy()
            S[f"render_{n}_{seed}_tree"] = r160.flatten(t, s)
            r160.free(t)
    s = r160.bench_scene(1, 1000)
    S["bench_1000_1_pre"] = s.copy()
    t = r160.build(s, 0, 999, 20)                 # benchmark.c:317
    S["bench_1000_1_post"] = s.copy()
    S["bench_1000_1_tree"] = r160.flatten(t, s)
    r160.free(t)

    for kind, n, start_end_depth in [("render", 10000, None), ("render", 100000, None),
                                     ("bench", 1000000, None), ("render", 1000000, None)]:
        t1 = time.time()
        s = r160.render_scene(1, n) if kind == "render" else r160.bench_scene(1, n)
        pre = sha(s)
        t = r160.build(s)
        flat = r160.flatten(t, s)
        st = tree_stats(flat, r160.leaf_counts(t), n)
        st.update({"scene_sha": pre, "post_sha": sha(s), "tree_sha": sha(flat), "build_s": round(time.time() - t1, 2)})
        G["scenes"][f"{kind}_{n}_1"] = st
        r160.free(t)
        print(kind, n, st, flush=True)

    # per-ray closest hits (hit.c:91-109), sphere and slab primitives (hit.c:19-82)
    rng = np.random.default_rng(2024)
    # the reference tree points INTO the array it was built on: keep that
    # array alive and use it as the sphere base
    s = S["render_1000_1_pre"].copy()
    t = r160.build(s)
    assert s.tobytes() == S["render_1000_1_post"].tobytes()
    rays = np.concatenate([random_rays(rng, 4000, [-45, -25, -15], [45, 25, 55]), edge_rays(s, rng)])
    S["hits_rays"] = rays
    S["hits_render_1000"] = r160.intersect(t, s, rays)
    # trace_ray on explicit rays: depth 1 with the glibc stream, depth 5 under the contract
    S["trace_d1_mode0"] = r160.trace_rays(rays, s, t, depth=1, mode=0, seed=3)
    S["trace_d5_mode1"] = r160.trace_rays(rays, s, t, depth=5, mode=1, seed=3)
    S["trace_d5_mode1_brute"] = r160.trace_rays(rays[:1500], s, None, depth=5, use_bvh=False, mode=1, seed=3)
    r160.free(t)
    sb = S["bench_1000_1_pre"].copy()
    tb = r160.build(sb, 0, 999, 20)
    brays = random_rays(rng, 3000, [-10, -10, -10], [10, 10, 10])
    S["hits_bench_rays"] = brays
    S["hits_bench_1000"] = r160.intersect(tb, sb, brays)
    r160.free(tb)
    # element-wise primitives on random pairs + the edge rays
    m = len(rays)
    pair_s = s[rng.integers(0, len(s), m)]
    S["pairs_spheres"] = pair_s
    S["pairs_sphere_hits"] = r160.sphere_pairs(rays, pair_s)
    boxes = np.zeros(m, abi.AABB)
    lo = rng.uniform(-45, 40, (m, 3)).astype(np.float32)
    boxes["min"] = lo
    boxes["max"] = lo + rng.uniform(0, 10, (m, 3)).astype(np.float32)
    boxes[:64]["min"] = np.float32(np.inf)          # empty boxes (bvh.c:19-24)
    boxes[:64]["max"] = np.float32(-np.inf)
    S["pairs_boxes"] = boxes
    S["pairs_box_hits"] = r160.aabb_pairs(rays, boxes)

    # camera rays (ray.c:17-32 with main.c:356-366), default camera and a turned one
    cams = [abi.default_camera()]
    c2 = abi.default_camera()
    c2.yaw = np.float32(-np.pi + 0.37)
    c2.pitch = np.float32(-0.21)
    c2.position = abi.Vec3(3.5, 7.25, 41.0)
    L.h_camera_update(C.byref(c2))
    cams.append(c2)
    S["cameras"] = np.array([c.to_numpy() for c in cams], dtype=abi.CAMERA)
    G["camera_rays"] = {}
    for (W, H) in [(160, 90), (1920, 1080)]:
        R = Reference(W, H)
        for ci, cam in enumerate(cams):
            rows = [0, 1, H // 2, H - 1]
            cr = R.camera_rays(cam, rows=rows)
            key = f"{W}x{H}_cam{ci}"
            S[f"camrays_{key}"] = cr
            G["camera_rays"][key] = {"rows": rows, "sha": sha(cr)}

    # framebuffers (main.c:358-374 fresh frame)
    G["frames"] = {}

    def frame(W, H, kind, n, depth, mode, use_bvh=True, seed=1, cam_i=0, store=False, step=1, threads=8):
        R = Reference(W, H)
        sp = R.render_scene(1, n) if kind == "render" else R.bench_scene(1, n)
        tr = R.build(sp)
        t1 = time.time()
        img = R.render(cams[cam_i], sp, tr, depth=depth, use_bvh=use_bvh, mode=mode, seed=seed, step=step,
                       threads=threads)
        R.free(tr)
        key = f"{W}x{H}_{kind}{n}_d{depth}_m{mode}_b{int(use_bvh)}_s{seed}_c{cam_i}_step{step}"
        G["frames"][key] = {"sha": sha(img), "seconds": round(time.time() - t1, 2), "rows": img.shape[0]}
        if store:
            S["frame_" + key] = img
        print(key, G["frames"][key], flush=True)

    for n in [100, 10000]:
        for depth, mode in [(1, 0), (5, 0), (5, 1)]:
            for cam_i in [0, 1]:
                frame(160, 90, "render", n, depth, mode, cam_i=cam_i, store=True)
            frame(320, 180, "render", n, depth, mode)
    frame(160, 90, "render", 100, 5, 1, use_bvh=False, store=True)
    frame(160, 90, "render", 100, 1, 0, use_bvh=False, store=True)
    frame(160, 90, "render", 1000, 5, 1, seed=9, store=True)
    frame(640, 480, "render", 100, 1, 0)
    frame(640, 480, "render", 100, 5, 1)
    frame(800, 600, "render", 20, 5, 1)
    frame(1920, 1080, "render", 10000, 1, 0)                 # the unmodified reference, full frame
    frame(1920, 1080, "render", 10000, 5, 1)                 # headline config under the contract
    frame(1920, 1080, "render", 100000, 1, 0, step=64)       # every 64th row
    frame(1920, 1080, "bench", 1000000, 5, 1, step=64)

    np.savez_compressed(os.path.join(OUT, "small.npz"), **S)
    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(G, f, indent=1)
    print("done in", round(time.time() - t0, 1), "s")


if __name__ == "__main__":
    main()
