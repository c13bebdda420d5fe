"""Headline benchmark: Mrays/s of the primary-ray render path at 1920x1080 with
10,000 random spheres (BASELINE.json configs[1]): camera rays -> BVH
traversal + ray/sphere tests -> diffuse shading (depth 5, the reference's
MAX_DEPTH, main.c:19/366) -> RGBA8 framebuffer.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (N > 1)

One step at N GPUs = N successive frames of the reference's accumulating
display loop (main.c:379-408: the camera holds still, frame j adds RNG sample
j), each 1920x1080 at 1 primary ray per pixel: every rank renders its
interleaved 8-row blocks of all N frames in ONE launch into its HBM slabs
(scene resident, uploaded once), folds them into its accumulation buffer on
the device, and for N > 1 the displayed slabs are gathered to rank 0 over
RCCL and de-interleaved there. Per-GPU work is one frame's worth of rays
whatever N is ("scaling": "weak"); `--scaling strong` instead splits ONE
frame over the N ranks (its per-GPU launch shrinks with N until the bounce
pass's longest chains set the time). value = W*H primary rays per frame *
frames per step * K / (max over ranks of the timed region). Rank 0 prints
one JSON line.

Successive steps are triple-buffered (`--pipeline 3`, default): three device
contexts with the scene resident in each take turns on their own streams, so
step k + 1's launches fill the CU slots that step k's bounce pass frees while
its last chains drain (measured: 1.73 ms per frame serial, 1.38 / 1.33 /
1.30 ms with 2 / 3 / 4 contexts). Each frame is still rendered whole and
its bytes do not change; only the gap between frames closes. The timed
region still brackets all K steps (barrier + synchronize on both sides).
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
shard = importlib.import_module("cs201_sah-bvh_ray_tracer_amd.shard")

W, H, NSPH, DEPTH, SEED, ROW_BLOCK = 1920, 1080, 10000, 5, 1, 8
KIND, SPP, JITTER = "render", 1, False
# --workload: BASELINE.json configs (the default is configs[1], the metric's
# own configuration; the others are measured on request, one GPU or more)
WORKLOADS = {
    "1080p_10k": dict(W=1920, H=1080, KIND="render", NSPH=10000, SPP=1, JITTER=False,
                      desc="1920x1080, 10000 random spheres, 1 primary ray/pixel, diffuse shading depth 5 "
                           "(BASELINE configs[1])"),
    "1080p_100k": dict(W=1920, H=1080, KIND="render", NSPH=100000, SPP=1, JITTER=False,
                       desc="1920x1080, 100000 random spheres (deep BVH, LDS-stack stress), depth 5 "
                            "(BASELINE configs[2])"),
    "4k_10k": dict(W=3840, H=2160, KIND="render", NSPH=10000, SPP=1, JITTER=False,
                   desc="3840x2160, 10000 random spheres, depth 5 (BASELINE configs[3])"),
    "4k_1m_4spp": dict(W=3840, H=2160, KIND="bench", NSPH=1000000, SPP=4, JITTER=True,
                       desc="3840x2160, 1000000 benchmark spheres (benchmark.c:307-314, built over [0, N)), "
                            "4 spp jittered, depth 5 (BASELINE configs[4])"),
}
PEAK_HBM_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
NODE_B, SPHERE_B, COLOR_B, PIXEL_B = 32, 16, 4, 4
KERNEL = "bounce_kernel<true, 2, false>"   # dominant kernel of the default (wavefront, four-wide) schedule


def algorithmic_bytes(c, pixels):
    """per frame, sum over traced rays of 32 B per reference-DFS
    node test + 16 B per sphere test, 4 B per hit colour, 4 B per pixel written."""
    return NODE_B * c["nodes"] + SPHERE_B * c["spheres"] + COLOR_B * c["hits"] + PIXEL_B * pixels


def bounce_bytes(c):
    """The same per-unit figures restricted to the bounce kernel's work: the
    node/sphere tests and hit colours of depth levels >= 1, plus one pixel
    write per bounce chain (one chain per camera ray that hit)."""
    return (NODE_B * (c["nodes"] - c["nodes_primary"]) + SPHERE_B * (c["spheres"] - c["spheres_primary"])
            + COLOR_B * (c["hits"] - c["hits_primary"]) + PIXEL_B * c["hits_primary"])


def cpu_baseline(target_s=12.0):
    """The reference render path on this host's cores: oracle/_ref (the
    unmodified reference sources compiled in-tree) if present, else the
    oracle restatement. Bounded sample: evenly spaced rows of the same
    frame, stride chosen so the run takes ~target_s."""
    from oracle.lib import Oracle, Reference
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    try:
        ref = Reference(W, H)
        kind = "reference"
    except (FileNotFoundError, OSError):
        ref, kind = None, "port"
    o = Oracle()
    # same scene (bit-identical generator), same tree ([0, N), depth 0)
    s = o.render_scene(SEED, NSPH) if KIND == "render" else o.bench_scene(SEED, NSPH)
    cam = mirt.default_camera()
    if ref is not None:
        s_ref = s.copy()
        tree = ref.build(s_ref)

        def run(step, nthreads):
            t0 = time.perf_counter()
            img = ref.render(cam, s_ref, tree, depth=DEPTH, mode=1, seed=SEED, row0=0, step=step,
                             threads=nthreads, jitter=JITTER)
            return time.perf_counter() - t0, img.shape[0]
    else:
        tree = o.build(s)

        def run(step, nthreads):
            rows = np.arange(0, H, step, dtype=np.int32)
            t0 = time.perf_counter()
            o.render(cam, W, H, s, tree, depth=DEPTH, mode=1, seed=SEED, rows=rows, threads=nthreads, jitter=JITTER)
            return time.perf_counter() - t0, len(rows)

    def sample(step, nthreads, budget):
        # repeat the strided frame until the budget is spent (a fast host
        # renders the whole frame in a few seconds)
        t = rows = reps = 0
        while t < budget or reps == 0:
            dt, n = run(step, nthreads)
            t, rows, reps = t + dt, rows + n, reps + 1
        return t, rows, reps

    probe_t, probe_rows = run(max(1, H // (2 * threads)), threads)   # ~2 rows per thread
    per_row = probe_t / max(probe_rows, 1)
    step = max(1, int(np.ceil(H * per_row / target_s)))
    t, rows, reps = sample(step, threads, 0.8 * target_s)
    value = rows * W / t / 1e6
    step1 = max(step * threads, 1)                 # single core, same row density / threads
    t1, rows1, reps1 = sample(step1, 1, 0.8 * target_s)
    value1 = rows1 * W / t1 / 1e6
    if ref is not None:
        ref.free(tree)
    else:
        o.free(tree)
    return {"value": round(value, 5), "unit": "Mrays/s", "cores": threads, "kind": kind,
            "sample": f"every {step}th row of the {W}x{H} frame (sample 0{', jittered' if JITTER else ''}) x {reps} "
                      f"({rows} rows, {rows * W} primary rays, depth {DEPTH}, {threads} OpenMP threads, "
                      f"row-dynamic schedule) in {t:.1f} s",
            "single_core_value": round(value1, 5),
            "single_core_sample": f"every {step1}th row x {reps1} ({rows1} rows) in {t1:.1f} s"}


def load_traffic(kernel):
    """Per-launch HBM bytes of the render kernel from the committed PMC
    profile (profiles/pmc_render.json, written by scripts/collect_profiles.py
    from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this bench), if
    it was taken on this workload and kernel."""
    p = os.path.join(ROOT, "profiles", "pmc_render.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    if d.get("workload") != [W, H, NSPH, DEPTH] or d.get("kernel") != kernel:
        return None
    return d.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (D2H) leg")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="1080p_10k")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="device contexts alternating successive steps on their own streams (1 = serial)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: N frames in flight per step at N GPUs (default); strong: one frame split N ways")
    args = ap.parse_args()
    global W, H, NSPH, KIND, SPP, JITTER
    wl = WORKLOADS[args.workload]
    W, H, NSPH, KIND, SPP, JITTER = wl["W"], wl["H"], wl["NSPH"], wl["KIND"], wl["SPP"], wl["JITTER"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"

    spheres = (mirt.create_random_spheres(NSPH, SEED) if KIND == "render"
               else mirt.create_benchmark_spheres(NSPH, SEED))
    t0 = time.perf_counter()
    bvh = mirt.build_bvh(spheres)
    build_s = time.perf_counter() - t0
    dev = local if world > 1 else 0
    rs = [mirt.Renderer(dev) for _ in range(max(1, args.pipeline))]
    for x in rs:
        x.upload(spheres, bvh)
    r = rs[0]
    cam = mirt.default_camera()
    # frames (accumulated samples) in flight per step: SPP per frame x N at N GPUs (weak scaling)
    frames = SPP * (world if args.scaling == "weak" else 1)
    sf = shard.ShardedFrame(r, W, H, ROW_BLOCK, samples=frames, renderers=rs)
    fd = sf.desc(depth=DEPTH, seed=SEED, jitter=JITTER)
    my_rows = shard.shard_row_count(H, ROW_BLOCK, world, rank)

    # algorithmic work of this rank's launch (instrumented build, untimed):
    # the walk as configured (pruned), and the reference's exhaustive DFS
    counts = r.count_frame(cam, W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, shard=rank, num_shards=world,
                           samples=frames, jitter=JITTER)
    r.set_option(mirt.abi.OPT_PRUNE, 0)
    ref_counts = r.count_frame(cam, W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, shard=rank,
                               num_shards=world, samples=frames, jitter=JITTER)
    r.set_option(mirt.abi.OPT_PRUNE, 1)
    alg_bytes = algorithmic_bytes(counts, my_rows * W * frames)

    # a non-default stream for the serial measurement loop below (the timed
    # loop runs on the ShardedFrame's own streams when double-buffered)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    for _ in range(args.warmup):
        sf.render_local(cam, fd)
        if world > 1:
            sf.gather()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        sf.render_local(cam, fd)
        if world > 1:
            sf.gather()          # N = 1: the slab is the frame
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # depth 1 alongside (camera rays and their shading only),
    # same pipeline, same step
    fd1 = sf.desc(depth=1, seed=SEED, jitter=JITTER)
    for _ in range(2):
        sf.render_local(cam, fd1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    for k in range(args.steps):
        sf.render_local(cam, fd1)
        if world > 1:
            sf.gather()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed_d1 = time.perf_counter() - t1

    # per-kernel split of the same launch, one context, serial (untimed loop:
    # each launch waits for its events): torch events around the launch and
    # the HIP events the library records around the primary and bounce passes
    slabs = torch.zeros((frames, sf.rows, W), dtype=torch.int32, device="cuda")
    acc = torch.zeros((sf.rows, W, 3), dtype=torch.float32, device="cuda") if frames > 1 else None
    phases, launch = [], []
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r.render_frame_device(cam, fd, slabs.data_ptr(), acc.data_ptr() if acc is not None else None,
                              stream.cuda_stream)
        e1.record(stream)
        phases.append(r.last_phase_ms())
        e1.synchronize()
        launch.append(e0.elapsed_time(e1))
    primary_ms, bounce_ms = (float(v) for v in np.mean(np.array(phases), axis=0))
    kernel_ms = float(np.mean(launch))

    t = torch.tensor([elapsed, kernel_ms, elapsed_d1], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms_max, elapsed_d1 = float(t[0]), float(t[1]), float(t[2])

    if rank == 0:
        value = W * H * frames * args.steps / elapsed / 1e6   # primary rays: W*H per sample
        frame_gbs = alg_bytes / (kernel_ms / 1e3) / 1e9
        b_bytes = bounce_bytes(counts)
        achieved = b_bytes / (bounce_ms / 1e3) / 1e9
        traffic = load_traffic(KERNEL) if world == 1 else None
        # the same frame through the blocking host API (kernel + D2H over PCIe)
        host = None
        if world == 1 and not args.no_host:
            img = r.render_frame(cam, W, H, depth=DEPTH, seed=SEED, samples=SPP, jitter=JITTER)
            dts = []
            for _ in range(11):   # median call: pageable-buffer page faults make single calls noisy
                t1 = time.perf_counter()
                img = r.render_frame(cam, W, H, depth=DEPTH, seed=SEED, samples=SPP, jitter=JITTER)
                dts.append(time.perf_counter() - t1)
            host = W * H * SPP / sorted(dts)[len(dts) // 2] / 1e6
        line = {
            "metric": "Mrays/s at 1080p, 10k spheres; 1/2/4/8 GPU + CPU baseline",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (create_random_sphere scene, srand(1); default camera main.c:203-211)",
            "config": {"workload": wl["desc"], "name": args.workload,
                       "width": W, "height": H, "spheres": NSPH, "scene": KIND, "max_depth": DEPTH, "spp": SPP,
                       "jitter": JITTER,
                       "frames_per_step": frames, "pipeline": len(rs), "bvh_nodes": len(bvh),
                       "row_block": ROW_BLOCK,
                       "parallelism": f"row-block shard x{world}" + (" + RCCL gather" if world > 1 else "")
                                      + (f", {frames} accumulated frames in flight" if frames > 1 else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                         "kernel": KERNEL, "kernel_ms": round(bounce_ms, 4),
                         "algorithmic_bytes_per_launch": int(b_bytes),
                         "primary_kernel_ms": round(primary_ms, 4),
                         "primary_algorithmic_bytes": int(alg_bytes - b_bytes),
                         "frame_ms": round(kernel_ms, 4), "frame_algorithmic_bytes": int(alg_bytes),
                         "frame_achieved": round(frame_gbs, 1),
                         "frame_achieved_pipelined": round(alg_bytes / (elapsed / args.steps) / 1e9, 1),
                         "note": "bytes of the node/sphere reads the (pruned) walk performs, per SURVEY 8(d) "
                                 "unit costs; the tree is L2/MALL-resident, so frac measures the achieved "
                                 "cache-fed rate against the HBM peak. kernel_ms / frame_ms: one launch alone "
                                 "(serial loop); the timed loop overlaps successive launches (pipeline)"},
            "work": {k: int(v) for k, v in counts.items()},
            "work_reference_dfs": {k: int(v) for k, v in ref_counts.items() if k != "lane_steps"},
            "traced_rays_per_s_M": round(counts["rays"] * world / (kernel_ms_max / 1e3) / 1e6, 3),
            "depth1_mrays_s": round(W * H * frames * args.steps / elapsed_d1 / 1e6, 3),
            "host_inclusive_mrays_s": None if host is None else round(host, 3),
            "bvh_build_s": round(build_s, 4),
        }
        if world == 1 and not args.no_cpu:
            cb = cpu_baseline()
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu"] = round(value / cb["value"], 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    for x in rs:
        x.close()


if __name__ == "__main__":
    main()
