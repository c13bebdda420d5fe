"""Headline benchmark: Mrays/s of the primary-ray render path at 1920x1080 with
10,000 random spheres (BASELINE.json configs[1]): camera rays -> BVH
traversal + ray/sphere tests -> diffuse shading (depth 5, the reference's
MAX_DEPTH, main.c:19/366) -> RGBA8 framebuffer.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (N > 1)

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment
starts the N rank processes itself (one per GPU, MASTER_ADDR 127.0.0.1); the
parent never touches the GPU and exits with the worst rank's status.

One step at N GPUs = N successive frames of the reference's accumulating
display loop (main.c:379-408: the camera holds still, frame j adds RNG sample
j), each 1920x1080 at 1 primary ray per pixel: every rank renders its
interleaved 8-row blocks of all N frames in ONE launch into its HBM slabs
(scene resident, uploaded once), folds them into its accumulation buffer on
the device, and for N > 1 the displayed slabs are gathered to rank 0 over
RCCL and de-interleaved there. Per-GPU work is one frame's worth of rays
whatever N is ("scaling": "weak"). At N > 1 the line also carries
`value_strong`: ONE frame split N ways per step, timed the same way (its
per-GPU launch shrinks with N until the bounce pass's longest chains set the
time); `--scaling strong` makes that the headline. value = W*H primary rays
per frame * frames per step * K / (max over ranks of the timed region).

Successive steps are quadruple-buffered (`--pipeline 4`, default): four device
contexts with the scene resident in each take turns on their own streams (one
per hardware queue), so step k + 1's launches fill the CU slots that step k's
bounce pass frees while its last chains drain. With frames in flight each
context's persistent bounce pass runs 1.5 workgroups per CU
(`--bounce-blocks`, MIRT_OPT_BOUNCE_BLOCKS; a launch alone keeps the full
occupancy x CUs): the four frames' passes then share the chip instead of the
first holding every slot. Each frame is still rendered whole and its bytes do
not change; only the gap between frames closes. The timed region brackets all
K steps (barrier + synchronize on both sides).

Also in the line (N = 1): `host_inclusive_mrays_s`, SURVEY §8(d)'s t_frame
(call -> RGBA8 frame in host memory): the same four contexts, each frame's
D2H copy into page-locked memory enqueued behind its kernels
(mirt_render_frame_async) so it overlaps the next frame; the blocking
single-call rate into pageable memory beside it. `roofline`: the dominant
kernel (the bounce pass) priced per §8(d) plus the bound the PMC counters
measured (profiles/r02_pmc_bound.json). `cpu_baseline`: the unmodified
reference sources (oracle/_ref) on this host's cores.

`--dry` (CPU only, gloo): the same launcher, shard geometry, gather and
max-over-ranks timing with a synthetic slab in place of the GPU frame --
a plumbing check for CPU tests; its line says "dry": true and is no measurement.
"""
import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
shard = importlib.import_module("cs201_sah-bvh_ray_tracer_amd.shard")

METRIC = "Mrays/s at 1080p, 10k spheres; 1/2/4/8 GPU + CPU baseline"
W, H, NSPH, DEPTH, SEED, ROW_BLOCK = 1920, 1080, 10000, 5, 1, 8
KIND, SPP, JITTER = "render", 1, False
WORKLOAD = "1080p_10k"
# --workload: BASELINE.json configs (the default is configs[1], the metric's
# own configuration; the others are measured on request, one GPU or more)
WORKLOADS = {
    "1080p_10k": dict(W=1920, H=1080, KIND="render", NSPH=10000, SPP=1, JITTER=False,
                      desc="1920x1080, 10000 random spheres, 1 primary ray/pixel, diffuse shading depth 5 "
                           "(BASELINE configs[1])"),
    # BB_PER_CU: persistent bounce workgroups per CU with frames in flight (1.5 unless stated): the
    # 100k tree's walks are twice as long, and 2 per CU measured +4.5% there (1,019 / 1,044 -> 1,091 /
    # 1,058 Mrays/s) while 1080p/10k and 4K lose with it (profiles/r04i/, r04k/)
    "1080p_100k": dict(W=1920, H=1080, KIND="render", NSPH=100000, SPP=1, JITTER=False, BB_PER_CU=2.0,
                       desc="1920x1080, 100000 random spheres (deep BVH, LDS-stack stress), depth 5 "
                            "(BASELINE configs[2])"),
    "4k_10k": dict(W=3840, H=2160, KIND="render", NSPH=10000, SPP=1, JITTER=False,
                   desc="3840x2160, 10000 random spheres, depth 5 (BASELINE configs[3])"),
    "4k_1m_4spp": dict(W=3840, H=2160, KIND="bench", NSPH=1000000, SPP=4, JITTER=True,
                       desc="3840x2160, 1000000 benchmark spheres (benchmark.c:307-314, built over [0, N)), "
                            "4 spp jittered, depth 5 (BASELINE configs[4])"),
}
PEAK_HBM_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
PEAK_L2_GBS = 34500.0   # aggregate L2 (MI355X_MICROARCH.md §L2)
NODE_B, SPHERE_B, COLOR_B, PIXEL_B = 32, 16, 4, 4
# frames per launch by GPU count, measured at the driver's --steps 20: one
# frame per launch is fastest at N = 1 (bench.py itself, profiles/r03c/:
# 1 / 2 / 4 frames 2,358-2,408 / 2,142-2,206 / 2,062-2,064 Mrays/s); the
# one-frame split at N ranks emulated shard by shard on one GPU
# (scripts/shard_times.py --pipeline 4 --batch B, profiles/r03d/k20_*):
# N = 2: 4,634 / 4,517 / 4,372, N = 4: 7,286 / 7,393 / 7,966, N = 8:
# 9,460 / 11,243 / 13,735 Mrays/s before the gather
DEFAULT_BATCH = {1: 1, 2: 1, 4: 4, 8: 4}
# at N > 1: contexts in flight per rank and the hardware queues that gives
# them (emulated at N = 8, K = 20, 4 frames per launch: 4 ctxs / 4 queues with
# a gather-sized copy on a fifth stream 11.9 Grays/s, 8 queues 13.2; 8 ctxs on
# 8 queues without the copy 15.2; profiles/r03f/)
PIPELINE_MULTI, HW_QUEUES_MULTI = 8, 16
# at N = 1 the environment's queues stay (0): 8 queues for the four contexts
# measured 2,662-2,674 vs 2,625-2,633 in one session (profiles/r04an/) and
# 2,621-2,654 vs 2,617-2,664 in the next (three rounds, profiles/r04ao/)
HW_QUEUES_SINGLE = 0
# the last TAIL_GRID launches of a timed burst run their bounce pass on the
# full persistent grid: with frames in flight every launch takes 1.5
# workgroups per CU so the frames share the chip, but the burst's last frame
# drains alone at that grid (profiles/r03zf: 0.89 ms of the 16 ms region with
# one 384-workgroup launch on the chip). An application that renders a known
# sequence (the K timed steps) can give the launches that nothing will follow
# the whole chip; an interactive loop cannot know its last frame. Measured at
# K = 20 (profiles/r03zg/summary.txt, rounds interleaved): 1 / 2 last launches
# 1080p/10k -0.2% / +1.1%, 1080p/100k +1.7% / 0%, 4K/10k +3.1% / +2.6%,
# 4K/1M 0% / 0%: within the rounds' spread at the metric's config, so the
# bench keeps one launch plan for the whole burst (0).
TAIL_GRID = 0
# at N > 1 a rank's launch is 1/N of a frame per frame carried, and the
# burst's drain is a larger share of the timed region: the last 2 of the 5
# launches (K = 20, 4 frames each) on the full grid -- the one-frame split at
# N = 8 emulated per shard (scripts/shard_times.py --tail-grid, copy stream,
# 16 queues; profiles/r04g/): 15.4-15.6 -> 16.4 Grays/s (1 launch: 16.1)
TAIL_GRID_MULTI = 2
KERNEL = "bounce_kernel<true, 2, false>"   # dominant kernel of the default (wavefront, four-wide) schedule
# the PMC-derived bound of the timed launch shape, per workload
# (scripts/pmc_bench.sh over this script's own command + scripts/pmc_summary.py);
# the newest round's file wins
PMC_BOUND = {wl: [os.path.join(ROOT, "profiles", f"r0{r}_pmc_bound_{wl}.json") for r in (4, 3)] for wl in WORKLOADS}
# the chip's gather peak by access shape (scripts/td_probe.hip + its counter
# passes, scripts/td_probe_summary.py): the roofline's denominator
TD_PROBE = os.path.join(ROOT, "profiles", "r04_td_probe.json")
WAVE_SLOTS = 256 * 4 * 5   # CUs x SIMDs x the bounce kernel's 5 waves per SIMD (amdgpu_waves_per_eu)


def algorithmic_bytes(c, pixels):
    """per frame, sum over traced rays of 32 B per node test +
    16 B per sphere test, 4 B per hit colour, 4 B per pixel written."""
    return NODE_B * c["nodes"] + SPHERE_B * c["spheres"] + COLOR_B * c["hits"] + PIXEL_B * pixels


def bounce_bytes(c):
    """The same per-unit figures restricted to the bounce kernel's work: the
    node/sphere tests and hit colours of depth levels >= 1, plus one pixel
    write per bounce chain (one chain per camera ray that hit)."""
    return (NODE_B * (c["nodes"] - c["nodes_primary"]) + SPHERE_B * (c["spheres"] - c["spheres_primary"])
            + COLOR_B * (c["hits"] - c["hits_primary"]) + PIXEL_B * c["hits_primary"])


# ------------------------------------------------------------------ CPU leg

def host_cpu():
    """nproc, the affinity mask's size and the CPU model of this host."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "model": model,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_threads():
    """Threads for the all-core leg: the box's CPU share where the environment
    states it (OMP_NUM_THREADS: the GPU box sets it to its 16-CPU share,
    while nproc there reports the whole machine), else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return min(int(env), aff), "OMP_NUM_THREADS"
    return aff, "sched_getaffinity"


def cpu_baseline(target_s=10.0):
    """The reference render path on this host's cores: oracle/_ref (the
    unmodified reference sources compiled in-tree) if present, else the
    oracle restatement. Bounded samples of the same frame: evenly spaced
    rows, stride chosen so each leg takes about its budget.
      value              all threads, -O2 (SURVEY §8(d) CPU baseline (b))
      single_core_value  one thread, -O2 ((a))
      O0_single_core     one thread, the reference's own flags (Makefile:3,43: no -O, -g)
      config0            BASELINE configs[0]: 640x480, 100 spheres, depth 5, BVH on, full frames"""
    from oracle.lib import Oracle, Reference
    threads, source = cpu_threads()
    o = Oracle()

    def make(Wc, Hc, nsph, kind, opt="O2"):
        try:
            ref = Reference(Wc, Hc, opt)
            k = "reference"
        except (FileNotFoundError, OSError):
            if opt != "O2":
                return None
            ref, k = None, "port"
        s = o.render_scene(SEED, nsph) if kind == "render" else o.bench_scene(SEED, nsph)
        cam = mirt.default_camera()
        if ref is not None:
            tree = ref.build(s)

            def run(step, nthreads):
                t0 = time.perf_counter()
                img = ref.render(cam, s, tree, depth=DEPTH, mode=1, seed=SEED, row0=0, step=step,
                                 threads=nthreads, jitter=JITTER)
                return time.perf_counter() - t0, img.shape[0]
            free = lambda: ref.free(tree)  # noqa: E731
        else:
            tree = o.build(s)

            def run(step, nthreads):
                rows = np.arange(0, Hc, step, dtype=np.int32)
                t0 = time.perf_counter()
                o.render(cam, Wc, Hc, s, tree, depth=DEPTH, mode=1, seed=SEED, rows=rows, threads=nthreads,
                         jitter=JITTER)
                return time.perf_counter() - t0, len(rows)
            free = lambda: o.free(tree)  # noqa: E731
        return run, free, k

    def sample(run, Wc, Hc, nthreads, budget):
        probe_t, probe_rows = run(max(1, Hc // (2 * nthreads)), nthreads)   # ~2 rows per thread
        per_row = probe_t / max(probe_rows, 1)
        step = max(1, int(np.ceil(Hc * per_row / budget)))
        t = rows = reps = 0
        while t < 0.8 * budget or reps == 0:    # whole strided frames, repeated on a fast host
            dt, n = run(step, nthreads)
            t, rows, reps = t + dt, rows + n, reps + 1
        return {"value": round(rows * Wc / t / 1e6, 5), "step": step, "reps": reps, "rows": rows, "s": round(t, 2)}

    run, free, kind = make(W, H, NSPH, KIND)
    multi = sample(run, W, H, threads, target_s)
    single = sample(run, W, H, 1, target_s / 2)
    free()
    out = {"value": multi["value"], "unit": "Mrays/s", "cores": threads, "kind": kind,
           "sample": f"every {multi['step']}th row of the {W}x{H} frame (sample 0{', jittered' if JITTER else ''}) "
                     f"x {multi['reps']} ({multi['rows']} rows, {multi['rows'] * W} primary rays, depth {DEPTH}, "
                     f"{threads} OpenMP threads [{source}], row-dynamic schedule, gcc -O2 -ffp-contract=off) "
                     f"in {multi['s']} s",
           "host": host_cpu(),
           "single_core_value": single["value"],
           "single_core_sample": f"every {single['step']}th row x {single['reps']} ({single['rows']} rows) "
                                 f"in {single['s']} s, -O2"}
    # the whole host, for context: `cores` is this box's CPU share, not the machine
    hc = out["host"]
    avail = max(hc["nproc"] or 1, hc["affinity"] or 1)
    eff = multi["value"] / max(single["value"] * threads, 1e-12)
    out["cores_available"] = avail
    out["thread_scaling_efficiency"] = round(eff, 3)
    out["all_core_estimate"] = {
        "value": round(multi["value"] * avail / threads, 4), "cores": avail, "kind": "estimate",
        "note": f"linear extrapolation of the {threads}-thread rate to all {avail} cores of the host (not measured: "
                f"the box grants {threads} CPUs; {threads} threads ran at {eff:.0%} of {threads} x one core, so this "
                "is an upper bound for the reference on the whole machine)"}
    m0 = make(W, H, NSPH, KIND, "O0")
    if m0 is not None:
        run0, free0, _ = m0
        s0 = sample(run0, W, H, 1, target_s / 2)
        free0()
        out["O0_single_core_value"] = s0["value"]
        out["O0_single_core_sample"] = (f"every {s0['step']}th row x {s0['reps']} ({s0['rows']} rows) in {s0['s']} s, "
                                        "the reference's own flags (-g, no -O: Makefile:3,43)")
    # BASELINE configs[0]: 640x480, 100 random spheres, BVH on
    cfg0 = {"workload": "640x480, 100 random spheres, BVH on, depth 5 (BASELINE configs[0])"}
    for label, opt, nt in (("value", "O2", threads), ("single_core_value", "O2", 1), ("O0_single_core_value", "O0", 1)):
        m = make(640, 480, 100, "render", opt)
        if m is None:
            continue
        r_, f_, _ = m
        cfg0[label] = sample(r_, 640, 480, nt, 2.0)["value"]
        f_()
    out["config0"] = cfg0
    return out


# ------------------------------------------------------------- launching

def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, deadline_s):
    """Start n copies of this script as ranks 0..n-1 (the torchrun contract's
    environment) and wait; a failing rank ends the others. Runs before any
    GPU call in this process (the ranks are fresh processes, never a re-exec).
    A job still running after `deadline_s` seconds (a rank stuck in RCCL init
    or a gather) is ended: every rank is terminated (killed 5 s later if it
    ignores that), the stuck ranks are named on stderr and the parent exits
    124, so the driver records a failure instead of waiting out its limit."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    t_end = time.monotonic() + deadline_s
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        if live and time.monotonic() > t_end:
            stuck = [procs.index(p) for p in live]
            print(f"bench.py: ranks {stuck} still running after the {deadline_s:.0f} s deadline "
                  "(--rank-timeout); terminating the job", file=sys.stderr, flush=True)
            for q in live:
                q.terminate()
            t_kill = time.monotonic() + 5.0
            for q in live:
                try:
                    q.wait(timeout=max(0.1, t_kill - time.monotonic()))
                except subprocess.TimeoutExpired:
                    q.kill()
                    q.wait()
            return 124
        time.sleep(0.05)
    return rc


def pg_timeout(args):
    """The process group's timeout: a collective (or the rendezvous) that
    waits longer raises in the rank instead of hanging it."""
    import datetime
    return datetime.timedelta(seconds=max(10.0, args.rank_timeout - 30.0))


def timed(world, launches, body):
    """barrier + synchronize, body(*l) for every launch l of the timed steps,
    synchronize + barrier; seconds."""
    cuda = torch.cuda.is_initialized()
    if world > 1:
        dist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for launch in launches:
        body(*launch)
    if cuda:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def dry_main(args, world, rank):
    """CPU plumbing check: synthetic slabs through the shard geometry, the
    gather and the timing of the GPU path (gloo). MIRT_BENCH_DRY_HANG=r makes
    rank r ("all": every rank) sleep before joining (the deadline tests)."""
    if os.environ.get("MIRT_BENCH_DRY_HANG") in (str(rank), "all"):
        time.sleep(3600)
    if world > 1:
        dist.init_process_group("gloo", timeout=pg_timeout(args))
    fd = mirt.frame_desc(W, H, depth=DEPTH, row_block=ROW_BLOCK, shard=rank, num_shards=world)
    rows = mirt.shard_rows(fd)
    slab = torch.zeros((shard.slab_rows(H, ROW_BLOCK, world), W), dtype=torch.int32)
    slab[:len(rows)] = torch.from_numpy(rows.astype(np.int64)[:, None] * W + np.arange(W)).to(torch.int32)
    frame = [None]

    def step():
        frame[0] = shard.gather_frame(slab, H, ROW_BLOCK) if world > 1 else shard.assemble(slab[None], H, ROW_BLOCK)

    for _ in range(args.warmup):
        step()
    el = timed(world, [()] * args.steps, step)
    t = torch.tensor([el], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        want = torch.arange(H * W, dtype=torch.int64).reshape(H, W).to(torch.int32)
        ok = bool(torch.equal(frame[0], want))
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mrays/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": None, "higher_is_better": True,
                          "scaling": args.scaling, "vs_baseline": None, "dtype": "f32", "dry": True,
                          "data": "synthetic slabs (no rendering): launcher / gather plumbing check",
                          "frame_assembled_ok": ok, "gather_ms_per_step": round(float(t[0]) / args.steps * 1e3, 4),
                          "config": {"workload": WORKLOADS[args.workload]["desc"], "name": args.workload,
                                     "parallelism": f"row-block shard x{world}" + (" + gloo gather" if world > 1 else "")}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


# ------------------------------------------------------------------ main

def load_pmc_bound(name):
    """The PMC-derived bound of the frame kernels of workload `name` in the
    timed launch shape (profiles/r0N_pmc_bound_<name>.json: scripts/pmc_bench.sh
    over `bench.py --workload name` + scripts/pmc_summary.py), or None."""
    for path in PMC_BOUND.get(name, []):
        if os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            if d.get("workload") == [W, H, NSPH, DEPTH]:
                return d, path
    return None, None


def gather_peak(probe, tcp_per_inst):
    """The chip's peak rate (G wave-load instructions/s) of dwordx4 gathers
    whose instructions touch as many L1 lines as the kernel's do: linear
    interpolation, in cycles per instruction, over the probe's one-node-per-
    lane cases keyed by their measured TCP accesses per instruction."""
    pts = sorted((c["tcp_accesses_per_instruction"], 1.0 / c["ginst_per_s"]) for c in probe["cases"]
                 if c["lanes_per_node"] == 1 and "tcp_accesses_per_instruction" in c)
    if not pts:
        return None, None
    x = min(max(tcp_per_inst, pts[0][0]), pts[-1][0])
    for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
        if x0 <= x <= x1:
            y = y0 + (y1 - y0) * (x - x0) / max(x1 - x0, 1e-12)
            return 1.0 / y, [(x0, round(1 / y0, 3)), (x1, round(1 / y1, 3))]
    return 1.0 / pts[-1][1], [pts[-1]]


def trace_check():
    """The same launch shape ALONE under rocprofv3 --kernel-trace --stats
    (committed summary): its mean duration must agree with kernel_ms."""
    path = os.path.join(ROOT, "profiles", "r04q", "exclusive_bounce_trace.json")
    if W != 1920 or NSPH != 10000 or not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return {"mean_ms": d["mean_ms"], "median_ms": d["median_ms"], "dispatches": d["dispatches"],
            "source": os.path.relpath(path, ROOT) + " (profiles/r04q/prof_exclusive_kernel_stats.csv)"}


def vmem_roofline(pmc, pmc_path, ms_per_step, frames_per_launch):
    """roofline of the dominant kernel on the unit that binds it (VERDICT r3
    item 1): the bounce kernel's vector-memory gather path. achieved = its
    wave-level load instructions (SQ_INSTS_VMEM_RD) / its exclusive time
    (GRBM_GUI_ACTIVE of the same counter pass, the timed launch shape);
    peak = scripts/td_probe's chip rate for gathers of the same shape (TCP
    accesses per load instruction). Recompute: counters and derived values
    in the PMC file, the probe table in profiles/r04_td_probe.json."""
    if not pmc or not os.path.exists(TD_PROBE):
        return None
    with open(TD_PROBE) as f:
        probe = json.load(f)
    kb = pmc["kernels"].get("timed/bounce", {})
    kp = pmc["kernels"].get("timed/primary", {})
    vb, db = kb.get("vmem_pass"), kb.get("derived", {})
    vp, dp = kp.get("vmem_pass") or {}, kp.get("derived", {})
    if not vb or not vb.get("tcp_accesses_per_instruction"):
        return None
    # instructions, time and access shape from ONE counter pass
    vmem, ms, tcp_per_inst = vb["SQ_INSTS_VMEM_RD"], vb["kernel_ms_at_2400MHz"], vb["tcp_accesses_per_instruction"]
    cb = {"SQ_WAVES": vb.get("SQ_WAVES") or WAVE_SLOTS}
    cp = {"SQ_INSTS_VMEM_RD": vp.get("SQ_INSTS_VMEM_RD", 0.0)}
    peak, bracket = gather_peak(probe, tcp_per_inst)
    if not peak:
        return None
    achieved = vmem / (ms * 1e-3) / 1e9
    share = min(1.0, cb.get("SQ_WAVES", WAVE_SLOTS) / WAVE_SLOTS)
    vmem_step = (vmem + cp.get("SQ_INSTS_VMEM_RD", 0.0)) / frames_per_launch
    step_rate = vmem_step / (ms_per_step * 1e-3) / 1e9
    return {
        "bound": "vmem", "achieved": round(achieved, 3), "peak": round(peak, 3), "unit": "Ginst/s",
        "frac": round(achieved / peak, 4),
        "traffic": db.get("hbm_bytes"),
        "kernel_ms": ms,
        "kernel_ms_source": "exclusive time of one bounce launch of the timed shape (GRBM_GUI_ACTIVE / 8 XCDs at "
                            "2.4 GHz, median over the launches of the counter pass; rocprofv3 serialises the "
                            "dispatches it counts)",
        "kernel_ms_per_step_share": round(ms * share, 4),
        "kernel_wave_slot_share": round(share, 4),
        "definition": "the bounce kernel (hit.c:91-109's walk for the bounce rays) on its binding unit, the "
                      "vector-memory gather path (TA/TD: per-lane dwordx4 loads of nodes, leaf records, spheres "
                      "from an L2-resident tree): its wave-level load instructions per second of its own time, "
                      "against the chip's peak rate for gathers touching the same number of L1 lines per "
                      "instruction (scripts/td_probe.hip). kernel_ms_per_step_share = kernel_ms x the launch's "
                      "waves / the chip's wave slots at 5 per SIMD: the frames in flight share the chip.",
        "vmem_rd_per_launch": vmem, "tcp_accesses_per_instruction": round(tcp_per_inst, 3),
        "peak_bracket": bracket, "td_busy": db.get("td_busy"), "ta_busy": db.get("ta_busy"),
        "valu_busy": db.get("valu_busy"), "wait_any_per_wave_cycle": db.get("wait_any_per_wave_cycle"),
        "primary_valu_busy": dp.get("valu_busy"), "primary_kernel_ms": dp.get("kernel_ms_at_2400MHz"),
        "timed_loop": {"note": "the frame loop's gather path per step: both kernels' load instructions per frame "
                               "/ ms_per_step, against the same peak (frames in flight hide the walk's latency "
                               "that one launch alone cannot)",
                       "vmem_rd_per_frame": vmem_step, "ginst_per_s": round(step_rate, 3),
                       "frac": round(step_rate / peak, 4)},
        "source": os.path.relpath(pmc_path, ROOT) + " + " + os.path.relpath(TD_PROBE, ROOT),
        "kernel_ms_trace_check": trace_check(),
    }


def bound_line(pb, exec_b, ref_b, ms):
    """bound_measured: the busiest unit of a kernel and its utilisation, from
    the committed counters."""
    if not pb:
        return None
    return {"unit": {"td_busy": "TD (vector-memory data return)", "ta_busy": "TA (vector-memory address)",
                     "valu_busy": "VALU issue", "l2_frac_upper": "L2 bandwidth",
                     "hbm_frac": "HBM bandwidth"}.get(pb.get("busiest_unit"), pb.get("busiest_unit")),
            "td_busy": pb.get("td_busy"), "ta_busy": pb.get("ta_busy"), "valu_busy": pb.get("valu_busy"),
            "l2_hit": pb.get("l2_hit"), "l2_read_gbs_upper": pb.get("l2_read_gbs_upper"),
            "l2_peak_gbs": PEAK_L2_GBS, "l2_frac_upper": pb.get("l2_frac_upper"),
            "l2_read_latency_cycles": pb.get("l2_read_latency_cycles"),
            "wait_any_per_wave_cycle": pb.get("wait_any_per_wave_cycle"),
            "executed_bytes_per_launch": int(exec_b),
            "executed_gbs": round(exec_b / (ms / 1e3) / 1e9, 1),
            "executed_vs_reference_bytes": round(exec_b / max(ref_b, 1), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (D2H) leg")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="1080p_10k")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="device contexts alternating successive launches on their own streams (1 = serial; "
                         "0 = 4 at N = 1, 8 at N > 1)")
    ap.add_argument("--bounce-blocks", type=int, default=-1,
                    help="persistent bounce workgroups per launch (MIRT_OPT_BOUNCE_BLOCKS) in the timed loop; "
                         "-1 = the workload's BB_PER_CU (1.5 unless stated) per CU with frames in flight "
                         "(--pipeline > 1), else 0 (occupancy x CUs)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default): every step is ONE frame (the N = 1 workload) split N ways, frames in "
                         "flight; weak: N frames per step at N GPUs (reported beside it as value_weak)")
    ap.add_argument("--batch", type=int, default=0,
                    help="steps' frames per launch (frames in flight inside a launch; 0 = DEFAULT_BATCH[N])")
    ap.add_argument("--tail-grid", type=int, default=-1,
                    help="the last N launches of a timed burst take the full persistent bounce grid (nothing "
                         "later will share the chip); 0 = every launch at --bounce-blocks; -1 = TAIL_GRID at "
                         "N = 1, TAIL_GRID_MULTI at N > 1")
    ap.add_argument("--accumulate", action="store_true",
                    help="time the still-camera accumulating display loop (shared accumulation buffer) instead "
                         "of fresh frames")
    ap.add_argument("--dry", action="store_true", help="CPU plumbing check over gloo (no GPU, no measurement)")
    ap.add_argument("--rank-timeout", type=float, default=420.0,
                    help="N > 1 started by this script: seconds before a still-running job is terminated (exit "
                         "124); each rank's process group times out 30 s earlier")
    ap.add_argument("--hw-queues", type=int, default=-1,
                    help="raise GPU_MAX_HW_QUEUES to this before the HIP runtime starts (-1: the environment's at "
                         "N = 1, 16 at N > 1; 0: keep the environment's)")
    ap.add_argument("--blocking-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--opt", action="append", default=[],
                    help="OPTION=VALUE (mirt_set_option on every context; A/B of schedule options), repeatable")
    args = ap.parse_args()
    global W, H, NSPH, KIND, SPP, JITTER, WORKLOAD
    WORKLOAD = args.workload
    wl = WORKLOADS[args.workload]
    W, H, NSPH, KIND, SPP, JITTER = wl["W"], wl["H"], wl["NSPH"], wl["KIND"], wl["SPP"], wl["JITTER"]

    if args.blocking_child:
        return blocking_child()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, args.rank_timeout)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}; measuring {world} rank(s)", file=sys.stderr)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.dry:
        return dry_main(args, world, rank)
    if not args.pipeline:
        args.pipeline = 4 if world == 1 else PIPELINE_MULTI
    if args.tail_grid < 0:
        args.tail_grid = TAIL_GRID if world == 1 else TAIL_GRID_MULTI
    # MIRT_BENCH_SHARE_GPU=1: a rehearsal of the N > 1 path on a one-GPU box --
    # every rank on device 0 and gloo in place of RCCL (which refuses two ranks
    # on one device); the same launches, shard geometry, gathers (staged
    # through host memory) and max-over-ranks timing. Not a measurement.
    rehearse = world > 1 and os.environ.get("MIRT_BENCH_SHARE_GPU") == "1"
    want_q = args.hw_queues if args.hw_queues >= 0 else (HW_QUEUES_MULTI if world > 1 else HW_QUEUES_SINGLE)
    if want_q and not rehearse:
        # one hardware queue per context stream plus RCCL's, read when the HIP
        # runtime starts (before the first GPU call below). The GPU boxes export
        # GPU_MAX_HW_QUEUES=4 (HIP's default), which would put the 8 contexts
        # and RCCL on 4 queues: the one-frame split emulated per shard ran 11.9
        # Grays/s at N = 8 there against 13.8 on 16 (profiles/r03f/, r03g/), so
        # a lower value is raised to HW_QUEUES_MULTI (one rank per GPU)
        try:
            have = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
        except ValueError:
            have = 0
        if have < want_q:
            os.environ["GPU_MAX_HW_QUEUES"] = str(want_q)
    dev = (0 if rehearse else local) if world > 1 else 0
    if world > 1:
        torch.cuda.set_device(dev)
        if rehearse:
            dist.init_process_group("gloo", timeout=pg_timeout(args))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout(args))
    else:
        torch.cuda.set_device(0)

    spheres = (mirt.create_random_spheres(NSPH, SEED) if KIND == "render"
               else mirt.create_benchmark_spheres(NSPH, SEED))
    t0 = time.perf_counter()
    bvh = mirt.build_bvh(spheres)
    build_s = time.perf_counter() - t0
    rs = [mirt.Renderer(dev) for _ in range(max(1, args.pipeline))]
    # bounce workgroups per launch with frames in flight (measured: 1080p/10k
    # 2,400 -> 2,650 Mrays/s at 4 contexts, profiles/r02_ab/r02au_*); the
    # serial measurement loop and the blocking call below use the full grid
    blocks = args.bounce_blocks
    if blocks < 0:
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        blocks = int(wl.get("BB_PER_CU", 1.5) * cus) if len(rs) > 1 else 0
    for x in rs:
        x.upload(spheres, bvh)
        x.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, blocks)
        for ov in args.opt:
            o, v = (int(t) for t in ov.split("="))
            x.set_option(o, v)
    r = rs[0]
    cam = mirt.default_camera()
    # The steps are successive frames, `fps` per step: 1 (strong, the N = 1
    # workload at every N) or N (weak). A frame is main.c:358-374's fresh
    # frame (the camera moved), shown after its SPP samples (4k_1m_4spp: 4
    # jittered samples folded like main.c:379-408's accumulation); with
    # --accumulate the frames are instead successive frames of the
    # still-camera display loop (main.c:379-408), the ctxs sharing one
    # accumulation buffer (mirt_ctx_share_accum). A launch carries `batch`
    # steps' frames (frames in flight inside one launch; each frame's display
    # its own slab) and, at N > 1, every displayed frame is gathered to rank 0.
    fps = world if args.scaling == "weak" else 1
    batch = args.batch if args.batch > 0 else DEFAULT_BATCH.get(world, 1)
    if SPP > 1 and not args.accumulate:
        batch = 1          # one fresh frame of SPP samples per launch (the fold restarts per launch)
    per_launch = fps * batch if SPP == 1 or args.accumulate else 1
    if SPP > 1 and not args.accumulate and fps > 1:
        raise SystemExit("--scaling weak with several samples per frame needs --accumulate")
    sf = shard.ShardedFrame(r, W, H, ROW_BLOCK, samples=SPP * per_launch, renderers=rs,
                            share_accum=args.accumulate, accum=SPP > 1 or args.accumulate)
    my_rows = shard.shard_row_count(H, ROW_BLOCK, world, rank)

    # algorithmic work of one full launch of this rank (instrumented build,
    # untimed): the walk as configured (pruned), and the reference's
    # exhaustive DFS
    counts = r.count_frame(cam, W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, shard=rank, num_shards=world,
                           samples=SPP * per_launch, jitter=JITTER)
    r.set_option(mirt.abi.OPT_PRUNE, 0)
    ref_counts = r.count_frame(cam, W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, shard=rank,
                               num_shards=world, samples=SPP * per_launch, jitter=JITTER)
    r.set_option(mirt.abi.OPT_PRUNE, 1)

    # a non-default stream for the serial measurement loop below (the timed
    # loop runs on the ShardedFrame's own streams when pipelined)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)

    def plan(f0, steps, per):
        """(first frame, frames) of the launches covering `steps` steps from frame f0"""
        out, f, end = [], f0, f0 + steps * fps
        while f < end:
            n = min(per, end - f)
            out.append((f, n))
            f += n
        return out

    def launcher(s, depth, tail=()):
        """The launch of frames f0 .. f0 + n - 1 on the next context; a launch
        whose first frame is in `tail` (the burst's last launches) runs its
        bounce pass on the full persistent grid instead of `blocks`."""
        def run(f0, n):
            acc = args.accumulate and f0 > 0
            x = s.rs[s.k % len(s.rs)] if f0 in tail else None
            if x is not None:
                keep = x.get_option(mirt.abi.OPT_BOUNCE_BLOCKS)
                x.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, 0)
            s.render_local(cam, s.desc(depth=depth, seed=SEED, sample=f0 * SPP, accumulate=acc,
                                       frames=f0 * SPP + 1 if acc else 1, jitter=JITTER, samples=n * SPP))
            if x is not None:
                x.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, keep)
            if world > 1:
                s.gather(every=SPP)       # every frame's display; N = 1: the slabs are the frames
        return run

    def tail_of(pl):
        """first frames of the last --tail-grid launches of a pipelined plan"""
        if len(rs) < 2 or not blocks or args.tail_grid <= 0:
            return ()
        return {f0 for f0, _ in pl[-args.tail_grid:]}

    warm = plan(0, args.warmup, per_launch)
    timed_plan = plan(args.warmup * fps, args.steps, per_launch)
    run = launcher(sf, DEPTH, tail_of(timed_plan))
    for p in warm:
        run(*p)
    elapsed = timed(world, timed_plan, run)

    # the two passes of every timed launch, from the HIP events the library
    # records on each launch's own stream around its primary and bounce
    # kernels (mirt_phase_log): their durations UNDER the overlap of the timed
    # loop (launch j on ctx j % P, the warm-up launches first)
    P = len(rs)
    timed_phases = []
    for i, x in enumerate(rs):
        n_i = sum(1 for j in range(len(warm), len(warm) + len(timed_plan)) if j % P == i)
        if n_i:
            timed_phases += x.phase_log(min(n_i, 64))
    primary_ms, bounce_ms = (float(v) for v in np.mean(np.array(timed_phases), axis=0))

    # depth 1 alongside (camera rays and their shading only)
    plan_d1 = plan(0, args.steps, per_launch)
    run1 = launcher(sf, 1, tail_of(plan_d1))
    for p in plan(0, 2, per_launch):
        run1(*p)
    elapsed_d1 = timed(world, plan_d1, run1)

    # the other scaling mode at N > 1 (same contexts, its own slabs)
    elapsed_other, fps_other = None, None
    if world > 1:
        fps_other = 1 if args.scaling == "weak" else world
        fps_main, fps = fps, fps_other
        per_other = fps_other * batch if SPP == 1 or args.accumulate else 1
        sf2 = shard.ShardedFrame(r, W, H, ROW_BLOCK, samples=SPP * per_other, renderers=rs,
                                 share_accum=args.accumulate, accum=SPP > 1 or args.accumulate)
        plan2 = plan(args.warmup * fps_other, args.steps, per_other)
        run2 = launcher(sf2, DEPTH, tail_of(plan2))
        for p in plan(0, args.warmup, per_other):
            run2(*p)
        elapsed_other = timed(world, plan2, run2)
        fps = fps_main

    # the same launch alone, one context, serial (untimed loop: each launch
    # waits for its events): torch events around the launch and the HIP
    # events the library records around the primary and bounce passes
    fd = sf.desc(depth=DEPTH, seed=SEED, jitter=JITTER)          # one full launch
    slabs = torch.zeros((SPP * per_launch, sf.rows, W), dtype=torch.int32, device="cuda")
    acc = torch.zeros((sf.rows, W, 3), dtype=torch.float32, device="cuda") if SPP > 1 or args.accumulate else None
    phases, launch = [], []
    r.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, 0)   # one launch alone: the full persistent grid
    for _ in range(min(args.steps, 20)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r.render_frame_device(cam, fd, slabs.data_ptr(), acc.data_ptr() if acc is not None else None,
                              stream.cuda_stream)
        e1.record(stream)
        phases.append(r.last_phase_ms())
        e1.synchronize()
        launch.append(e0.elapsed_time(e1))
    serial_primary_ms, serial_bounce_ms = (float(v) for v in np.mean(np.array(phases), axis=0))
    kernel_ms = float(np.mean(launch))
    r.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, blocks)

    t = torch.tensor([elapsed, kernel_ms, elapsed_d1, elapsed_other or 0.0], dtype=torch.float64, device="cuda")
    # the whole job's reference-DFS bytes per launch (every
    # rank's shard), for B / t / (G x 8 TB/s)
    job_b = torch.tensor([algorithmic_bytes(ref_counts, my_rows * W * SPP * per_launch)], dtype=torch.float64,
                         device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(job_b, op=dist.ReduceOp.SUM)
    elapsed, kernel_ms_max, elapsed_d1, elapsed_other = (float(v) for v in t)
    job_bytes_per_launch = float(job_b[0])

    host = None
    if rank == 0 and world == 1 and not args.no_host:
        for x in rs:
            x.share_accum(None)          # a private buffer per ctx again (--accumulate shared one)
        host = host_inclusive(rs, cam, args.steps)

    if rank == 0:
        value = W * H * SPP * fps * args.steps / elapsed / 1e6   # primary rays: W*H per sample
        pixels = my_rows * W * SPP * per_launch
        ref_frame_bytes = algorithmic_bytes(ref_counts, pixels)
        exec_frame_bytes = algorithmic_bytes(counts, pixels)
        ref_b = bounce_bytes(ref_counts)
        exec_b = bounce_bytes(counts)
        achieved = ref_b / (bounce_ms / 1e3) / 1e9
        pmc, pmc_path = load_pmc_bound(args.workload) if world == 1 else (None, None)
        pb = pmc["kernels"].get("timed/bounce", {}).get("derived", {}) if pmc else {}
        pp = pmc["kernels"].get("timed/primary", {}).get("derived", {}) if pmc else {}
        traffic = pb.get("hbm_bytes")
        bm = bound_line(pb, exec_b, ref_b, pb.get("kernel_ms_at_2400MHz") or bounce_ms)
        kname = KERNEL.replace("<true, 2,", "<true, 4,") if r.get_option(mirt.abi.OPT_LEAF_BATCH) else KERNEL
        roof = vmem_roofline(pmc, pmc_path, elapsed / args.steps * 1e3, per_launch)
        if roof is None:
            # no counter file for this workload: the roofline is not measured here (never priced against
            # the HBM peak with the reference's bytes: VERDICT r3)
            roof = {"bound": "vmem", "achieved": None, "peak": None, "unit": "Ginst/s", "frac": None,
                    "traffic": traffic, "note": "no profiles/r0N_pmc_bound_<workload>.json or td_probe table for "
                                                "this workload"}
        roof["kernel"] = kname
        if bm:
            bm["source"] = (os.path.relpath(pmc_path, ROOT) + " (medians over the dispatches of the timed launch "
                            "shape, one rocprofv3 --pmc pass of this command per counter set; rocprofv3 serialises "
                            "the dispatches it counts)")
        line = {
            "metric": METRIC,
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
            "data": "synthetic (create_random_sphere scene, srand(1); default camera main.c:203-211)"
                    + ("; REHEARSAL: all ranks on one GPU over gloo, not a measurement" if rehearse else ""),
            "config": {"workload": wl["desc"], "name": args.workload,
                       "width": W, "height": H, "spheres": NSPH, "scene": KIND, "max_depth": DEPTH, "spp": SPP,
                       "jitter": JITTER,
                       "frames_per_step": fps, "frames_per_launch": per_launch, "launches": len(timed_plan),
                       "pipeline": len(rs), "bounce_blocks": blocks, "tail_grid": len(tail_of(timed_plan)), "bvh_nodes": len(bvh),
                       "row_block": ROW_BLOCK, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "step": (f"{fps} frame(s) of the still-camera display loop (main.c:379-408), ctxs sharing "
                                "one accumulation buffer (mirt_ctx_share_accum)" if args.accumulate else
                                f"{fps} fresh frame(s) (main.c:358-374)")
                               + f", {SPP} sample(s) each, {per_launch} frame(s) per launch with every frame's "
                                 "display in its own slab, launches rotating over `pipeline` ctxs",
                       "parallelism": f"row-block shard x{world}" + (" + RCCL gather of every frame" if world > 1
                                                                     else "")},
            "roofline": roof,
            # SURVEY 8(d)'s figure, kept beside the roofline under its own name: the REFERENCE's work per
            # second, not a use of any unit (it exceeds HBM peak because the walk skips most
            # of it and the tree is cache-resident)
            "reference_work": {
                "definition": "SURVEY 8(d): bytes of the REFERENCE's exhaustive DFS (hit.c:91-109, no pruning) at "
                              "32 B/node test + 16 B/sphere test + 4 B/hit colour + 4 B/pixel, per second. The "
                              "walk executes a fraction of them (executed_vs_reference) from an L2/MALL-resident "
                              "tree, so this is the reference's work replaced per second, not HBM use.",
                "bounce_bytes_per_launch": int(ref_b),
                "bounce_launch_ms_under_overlap": round(bounce_ms, 4),
                "bounce_launch_ms_source": f"mean over the {len(timed_phases)} timed launches of HIP events on each "
                                           "launch's own stream around its bounce kernel (mirt_phase_log): "
                                           "durations UNDER the overlap of `pipeline` launches, so longer than "
                                           "the kernel's share of a step",
                "reference_work_gbs": round(achieved, 1),
                "reference_work_vs_hbm_peak": round(achieved / PEAK_HBM_GBS, 4),
                "executed_vs_reference_bytes": round(exec_b / max(ref_b, 1), 4),
                "hbm_measured": None if traffic is None else {
                    "bytes_per_launch": traffic,
                    "gbs_over_exclusive_time": round(traffic / (pb["kernel_ms_at_2400MHz"] / 1e3) / 1e9, 2),
                    "frac": round(traffic / (pb["kernel_ms_at_2400MHz"] / 1e3) / 1e9 / PEAK_HBM_GBS, 5)},
                "bound_measured": bm,
                "primary_launch_ms_under_overlap": round(primary_ms, 4),
                "primary_bytes_per_launch": int(ref_frame_bytes - ref_b),
                "primary_bound_measured": bound_line(pp, exec_frame_bytes - exec_b, ref_frame_bytes - ref_b,
                                                     pp.get("kernel_ms_at_2400MHz") or primary_ms),
                "launch_bytes": int(ref_frame_bytes),
                "launch_executed_bytes": int(exec_frame_bytes),
                "frame_period_ms": round(elapsed / args.steps * 1e3, 4),
                "frame_reference_gbs": round(ref_frame_bytes / batch / (elapsed / args.steps) / 1e9, 1),
                "job": {"note": "SURVEY 8(e): every rank's reference-DFS bytes over the timed launches / the "
                                "max-over-ranks timed region",
                        "bytes_per_launch": int(job_bytes_per_launch),
                        "gbs": round(job_bytes_per_launch * len(timed_plan) / elapsed / 1e9, 1)},
                "serial_launch": {
                    "note": "the same launch alone (untimed serial loop, the full persistent bounce grid): not "
                            "the timed configuration",
                    "frame_ms": round(kernel_ms, 4), "primary_ms": round(serial_primary_ms, 4),
                    "bounce_ms": round(serial_bounce_ms, 4),
                    "bounce_reference_gbs": round(ref_b / (serial_bounce_ms / 1e3) / 1e9, 1)}},
            "work": {k: int(v) for k, v in counts.items()},
            "work_reference_dfs": {k: int(v) for k, v in ref_counts.items() if k != "lane_steps"},
            "traced_rays_per_s_M": round(counts["rays"] * world / (elapsed / args.steps) / 1e6, 3),
            "depth1_mrays_s": round(W * H * SPP * fps * args.steps / elapsed_d1 / 1e6, 3),
            "bvh_build_s": round(build_s, 4),
        }
        if args.opt:
            line["options"] = args.opt
        if elapsed_other:
            other = W * H * SPP * fps_other * args.steps / elapsed_other / 1e6
            line["value_weak"] = round(value if args.scaling == "weak" else other, 3)
            line["value_strong"] = round(other if args.scaling == "weak" else value, 3)
        if host is not None:
            line.update(host)
        if world == 1 and not args.no_cpu:
            cb = cpu_baseline()
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu"] = round(value / cb["value"], 1)
            line["speedup_vs_cpu_single_core"] = round(value / cb["single_core_value"], 1)
            line["speedup_vs_cpu_all_core_estimate"] = round(value / cb["all_core_estimate"]["value"], 1)
            if host is not None:
                line["host_inclusive_speedup_vs_cpu"] = round(host["host_inclusive_mrays_s"] / cb["value"], 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    for x in rs:
        x.close()
    return 0


def host_inclusive(rs, cam, steps):
    """SURVEY §8(d) t_frame: frames delivered to host memory. Pipelined: ctx
    k % n renders frame k and copies it into its page-locked buffer
    (mirt_render_frame_async), waiting first for its frame k - n; blocking:
    one mirt_render_frame at a time (blocking_leg), in a child process and in
    this one."""
    fdh = mirt.frame_desc(W, H, depth=DEPTH, seed=SEED, samples=SPP, jitter=JITTER)
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in rs]
    n = len(rs)

    def run(k0, count):
        for k in range(k0, k0 + count):
            i = k % n
            rs[i].wait()
            rs[i].render_frame_async(cam, fdh, bufs[i])
        for x in rs:
            x.wait()

    run(0, 2 * n)
    steps_h = max(steps, 50)
    t0 = time.perf_counter()
    run(0, steps_h)
    el = time.perf_counter() - t0
    last = bufs[(steps_h - 1) % n].array.copy()
    for b in bufs:
        b.close()
    # the blocking call in THIS process too, after the four-context burst
    # (same measurement as the child's; reported beside it)
    rs[0].set_option(mirt.abi.OPT_BOUNCE_BLOCKS, 0)
    here = blocking_leg(rs[0], cam)
    child = blocking_in_child()
    out = {"host_inclusive_mrays_s": round(W * H * SPP * steps_h / el / 1e6, 3),
           "host_inclusive_ms_per_frame": round(el / steps_h * 1e3, 4),
           "host_inclusive_frames": steps_h,
           "host_inclusive_method": f"{n} ctxs, kernels + async D2H into page-locked buffers "
                                    "(mirt_render_frame_async), frame k waits for frame k - n",
           "host_frame_equals_blocking_call": frame_sha(last) == here["sha"] and here["equal"]}
    src = child if child else here
    out.update({"host_blocking_mrays_s": src["pinned_mrays_s"], "host_blocking_ms": src["pinned_ms"],
                "host_blocking_registered_mrays_s": src["registered_mrays_s"],
                "host_blocking_pageable_mrays_s": src["pageable_mrays_s"],
                "host_blocking_method": (
                    "one blocking mirt_render_frame per frame (main.c:350-421's loop) into a frame buffer from "
                    "mirt_host_alloc: the kernels write the pixels straight into it (MIRT_OPT_ZERO_COPY), median "
                    "of 11; " + ("measured in a child process holding one ctx and its frame buffer, as main.c's "
                                 "loop runs (bench.py --blocking-child)" if child else
                                 "measured in this process (the child process failed)")),
                "host_blocking_after_burst": {k: here[k] for k in ("pinned_mrays_s", "registered_mrays_s",
                                                                    "pageable_mrays_s")}})
    if child:
        out["host_frame_equals_blocking_call"] = out["host_frame_equals_blocking_call"] and \
            child["sha"] == here["sha"] and child["equal"]
        out["host_blocking_after_burst"]["note"] = (
            "the same calls in the bench's own process after its four-context burst: zero-copy stores run slower "
            "there for the rest of the process (profiles/r04x: a child started at that point measures as a "
            "fresh process does)")
    return out


def frame_sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def blocking_leg(r, cam, n=11):
    """The blocking call, one frame at a time (the full persistent grid), into
    plain pageable memory, into the caller's own frame buffer registered in
    place (INTEGRATION.md's recipe for main.c's malloc'd buffer: the kernels
    write the pixels straight into it) and into mirt_host_alloc memory;
    medians: page faults make single calls noisy."""
    img = r.render_frame(cam, W, H, depth=DEPTH, seed=SEED, samples=SPP, jitter=JITTER)

    def blocking(dst):
        r.render_frame_into(cam, W, H, dst, depth=DEPTH, seed=SEED, samples=SPP, jitter=JITTER)
        dts = []
        for _ in range(n):
            t1 = time.perf_counter()
            r.render_frame_into(cam, W, H, dst, depth=DEPTH, seed=SEED, samples=SPP, jitter=JITTER)
            dts.append(time.perf_counter() - t1)
        return sorted(dts)[len(dts) // 2]
    page = np.zeros((H, W, 4), np.uint8)
    dt_page = blocking(page)
    same = bool((page == img).all())
    mirt.host_register(page)
    try:
        dt_reg = blocking(page)
        same = same and bool((page == img).all())
    finally:
        mirt.host_unregister(page)
    hb = mirt.HostBuffer((H, W, 4))
    try:
        dt_pin = blocking(hb.array)
        same = same and bool((hb.array == img).all())
    finally:
        hb.close()
    res = {"equal": same, "sha": frame_sha(img)}
    for k, dt in (("pageable", dt_page), ("registered", dt_reg), ("pinned", dt_pin)):
        res[k + "_ms"] = round(dt * 1e3, 4)
        res[k + "_mrays_s"] = round(W * H * SPP / dt / 1e6, 3)
    return res


def blocking_child():
    """bench.py --blocking-child: one ctx with the workload's scene, the
    blocking leg, one JSON line (the parent's host_blocking_*)."""
    spheres = (mirt.create_random_spheres(NSPH, SEED) if KIND == "render"
               else mirt.create_benchmark_spheres(NSPH, SEED))
    r = mirt.Renderer(0)
    try:
        r.upload(spheres, mirt.build_bvh(spheres))
        print(json.dumps(blocking_leg(r, mirt.default_camera())), flush=True)
    finally:
        r.close()
    return 0


def blocking_in_child():
    """The blocking leg in a fresh child process (a new program, not a fork
    or an exec of this one, which has the GPU open); None if it fails."""
    import subprocess
    try:
        res = subprocess.run([sys.executable, os.path.abspath(__file__), "--blocking-child", "--workload", WORKLOAD],
                             capture_output=True, text=True, timeout=240)
        line = [l for l in res.stdout.splitlines() if l.startswith("{")]
        return json.loads(line[-1]) if res.returncode == 0 and line else None
    except (subprocess.SubprocessError, ValueError, IndexError):
        return None


if __name__ == "__main__":
    sys.exit(main())
