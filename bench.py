"""Headline benchmark: Mrays/s of the primary-ray render path at 1920x1080 with
10,000 random spheres (BASELINE.json configs[1]): camera rays -> BVH
traversal + ray/sphere tests -> diffuse shading (depth 5, the reference's
MAX_DEPTH, main.c:19/366) -> RGBA8 framebuffer IN HOST MEMORY (SURVEY §8(d)
t_frame: the end point of main.c:371-372's display).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Every N runs the C-ABI multi-GPU renderer of include/mirt_multi.h -- the
path a C caller of main.c's loop uses -- in ONE process:
mirt_multi_create over devices 0..N-1 (RCCL communicators from
ncclCommInitAll), the scene replicated, `pipeline` lanes of per-GPU contexts
keeping launches in flight, and every frame delivered into page-locked host
memory. A step is ONE fresh frame (main.c:358-374) split N ways by
interleaved 8-row blocks ("scaling": "strong"); value = W*H*spp*K / the timed
region (mirt_multi_wait + wall clock on both sides: every frame of the K
steps has reached host memory when the clock stops). Delivery (--delivery
auto): at N = 1 the GPU's slab is the frame (one D2H); at N > 1 every GPU
copies its row blocks into the host frame over its own link (host-direct),
and the RCCL gather to GPU 0 is measured beside it, to host memory
(`value_gather`) and left on GPU 0 (`device_resident_mrays_s`) -- one host
link cannot carry the frame rate of 8 GPUs at 1080p.

Processes. N = 1 measures in this process. N > 1: this process never
touches a GPU; it starts ONE fresh child (`--measure-child`) with
GPU_MAX_HW_QUEUES raised to 16 in its environment (read when the child's
HIP runtime starts: one hardware queue per lane's stream) and relays its
line; a child still running after --rank-timeout seconds is terminated and
the parent exits 124 -- unless the child had already measured the headline
and saved its line (before the secondary delivery's leg, whose n-GPU RCCL
exchange is the untried part): then the parent prints that line, the
unfinished leg marked in `other_delivery`, and exits 0. Under torchrun the same happens in rank 0; the other
ranks hold no GPU work and join rank 0 only at a gloo barrier at the end.

The schedule: `pipeline` lanes (4 at N = 1, 8 at N > 1), each
context's bounce pass at 1.5 persistent workgroups per CU, `batch` frames
per launch (1 at N <= 2, 2 at N = 4, 4 at N = 8); `--tail-grid T` puts the burst's
last T launches on the full grid (MIRT_MULTI_FULL_GRID; 0 by default: it
lost through mirt_multi in round 5's emulation).

Also in the line: `device_resident_mrays_s` (the same loop with the frames
left in device 0's HBM: the previous rounds' headline), depth 1, the
blocking call per frame (N = 1, a child process holding one context, as
main.c's loop runs), `roofline` (the bounce kernel on its binding unit, the
vector-memory gather path; profiles/), `cpu_baseline` (the unmodified
reference sources, oracle/_ref, on this host's cores; N = 1 only).

`--dry` (CPU only): the launcher, the shard geometry and both deliveries'
index math (multi.hip's de-interleave and strided host copies, restated in
shard.py) over synthetic slabs -- a plumbing check; its line says "dry": true.
"""
import argparse
import importlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

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
# 9,460 / 11,243 / 13,735 Mrays/s before the gather. Round 5, through
# mirt_multi (host-direct, 8 lanes, three interleaved rounds,
# profiles/r05_logs/r05an/): N = 2 1 / 2 frames 4,707-4,752 / 4,641-4,704;
# N = 4 2 / 4 frames 8,165-8,452 / 7,359-7,566; N = 8 keeps 4 (r05h, r05k)
DEFAULT_BATCH = {1: 1, 2: 1, 4: 2, 8: 4}
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
# at N > 1 a rank's launch is 1/N of a frame per frame carried. Round 4's
# Python ranks gained from the burst's last 2 launches on the full grid
# (profiles/r04g/); through mirt_multi (round 5, the per-shard emulation,
# host-direct, best of three per shard, profiles/r05_logs/r05k/) it loses: the last
# 0 / 1 / 2 launches on the full grid 15.51 / 14.91 / 14.82 Grays/s at N = 8
TAIL_GRID_MULTI = 0
# MIRT_MULTI_QUEUE_AHEAD: each context takes its next launch behind the
# current one on its stream (own slabs, copies on a copy stream), so no
# context idles through its frame's D2H and the host's turnaround
QUEUE_AHEAD, QUEUE_AHEAD_MULTI = False, False
KERNEL = "bounce_kernel<true, 2, false>"   # dominant kernel of the default (wavefront, four-wide) schedule
# the PMC-derived bound of the timed launch shape, per workload
# (scripts/pmc_bench.sh over this script's own command + scripts/pmc_summary.py);
# the newest round's file wins
PMC_BOUND = {wl: [os.path.join(ROOT, "profiles", f"r0{r}_pmc_bound_{wl}.json") for r in (6, 5, 4, 3)] for wl in WORKLOADS}
# the chip's gather peak by access shape (scripts/td_probe.hip + its counter
# passes, scripts/td_probe_summary.py): the roofline's denominator
TD_PROBE = os.path.join(ROOT, "profiles", "r04_td_probe.json")
# the same probe's access-MIX cases (round 5: dependent chains, L2 misses, five
# waves per SIMD, VALU / LDS / dword work between the loads; scripts/td_probe
# --mix, scripts/td_mix_summary.py over profiles/r05_logs/r05o)
TD_MIX = os.path.join(ROOT, "profiles", "r05_td_mix.json")
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


# ------------------------------------------------------------------ roofline

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
    for path, stats in ((os.path.join(ROOT, "profiles", "r06_exclusive_bounce_trace.json"),
                         "profiles/r06_logs/r06pmc/prof_exclusive_kernel_stats.csv"),
                        (os.path.join(ROOT, "profiles", "r05_exclusive_bounce_trace.json"),
                         "profiles/r05_logs/r05z/prof_exclusive_kernel_stats.csv"),
                        (os.path.join(ROOT, "profiles", "r04q", "exclusive_bounce_trace.json"),
                         "profiles/r04q/prof_exclusive_kernel_stats.csv")):
        if W == 1920 and NSPH == 10000 and os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            return {"mean_ms": d["mean_ms"], "median_ms": d["median_ms"], "dispatches": d["dispatches"],
                    "pmc_exclusive_ms": d.get("pmc_exclusive_ms"),
                    "source": os.path.relpath(path, ROOT) + f" ({stats}; scripts/exclusive_trace.py)"}
    return None


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
    out = {
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
        "reconcile": reconcile_busy(probe, vb, db, kb.get("counters", {}), achieved),
    }
    rec = out["reconcile"]
    if rec and rec.get("mix_matched"):
        # the frame loop's load rate against the ceiling of the kernel's own
        # instruction mix (the probe case at 5 waves per SIMD, alone on the chip)
        out["timed_loop"]["frac_vs_mix_ceiling"] = round(step_rate / rec["mix_matched"]["ceiling_ginst_per_s"], 4)
    return out


def reconcile_busy(probe, vb, db, counters, achieved):
    """`frac` (load instructions / s against the pure-gather
    peak) and the TD-busy reading disagree ~2.4x. The mechanism, measured with
    the probe's mix cases (profiles/r05_td_mix.json): TD busy per load
    instruction rises with VALU work interleaved on the same SIMDs (the same
    dwordx4 gathers plus 48 dependent FMAs per visit: TA busy falls with the
    load rate, 0.95 -> 0.42, TD stays 0.86, TD/TA 1.0 -> 2.0, the kernel's own
    TD/TA), while dependent chains, 13% L2 misses, five waves per SIMD, LDS
    reads and dword loads leave TD busy per instruction at 0.93-1.13x. So TD
    busy overstates the gather unit's load; TA busy (address processing, one
    per load) tracks it. Reported: the rate- and TA-based fractions against
    the pure-gather probe, TD's, and the rate against the probe case whose mix
    (VALU and LDS per load) is nearest the kernel's -- the ceiling of this
    instruction mix at full occupancy, not a hardware peak."""
    if not os.path.exists(TD_MIX):
        return None
    with open(TD_MIX) as f:
        mix = json.load(f)
    cases = [c for c in mix["cases"] if "ta_busy" in c and "valu_per_vmem_rd" in c]
    pure = [c for c in probe["cases"] if c.get("lanes_per_node") == 1 and "ta_busy" in c]
    if not cases or not pure:
        return None
    tcp = vb["tcp_accesses_per_instruction"]
    p0 = min(pure, key=lambda c: abs(c["tcp_accesses_per_instruction"] - tcp))
    vmem = counters.get("SQ_INSTS_VMEM_RD") or vb["SQ_INSTS_VMEM_RD"]
    valu_per = counters.get("SQ_INSTS_VALU", 0.0) / max(vmem, 1.0)
    lds_per = counters.get("SQ_INSTS_LDS", 0.0) / max(vmem, 1.0)
    full = [c for c in cases if c["dependent"] and c["cold_frac"] > 0 and c["workgroups"] == 2048]
    near = min(full or cases, key=lambda c: abs(c["valu_per_vmem_rd"] - valu_per) + 10 * abs(c["lds_per_vmem_rd"] - lds_per))
    td, ta = db.get("td_busy"), db.get("ta_busy")
    return {
        "kernel_valu_per_load": round(valu_per, 2), "kernel_lds_per_load": round(lds_per, 3),
        "kernel_td_over_ta": round(td / ta, 3) if td and ta else None,
        "pure_gather": {"tcp_accesses_per_instruction": p0["tcp_accesses_per_instruction"],
                        "td_busy": p0["td_busy"], "ta_busy": p0["ta_busy"],
                        "frac_by_ta": round(ta / p0["ta_busy"], 4) if ta else None,
                        "frac_by_td": round(td / p0["td_busy"], 4) if td else None},
        "mix_matched": {"case": {k: near[k] for k in ("active_lanes", "dependent", "cold_frac", "waves_per_simd",
                                                      "valu_fma_per_visit", "lds_reads_per_visit",
                                                      "dword_loads_per_visit", "valu_per_vmem_rd",
                                                      "lds_per_vmem_rd")},
                        "ceiling_ginst_per_s": near["ginst_per_s"],
                        "frac": round(achieved / near["ginst_per_s"], 4),
                        "frac_by_ta": round(ta / near["ta_busy"], 4) if ta else None,
                        "frac_by_td": round(td / near["td_busy"], 4) if td else None,
                        "probe_td_over_ta": round(near["td_busy"] / near["ta_busy"], 3)},
        "mechanism": "TD busy per load instruction grows with VALU work interleaved on the SIMDs (probe: +48 "
                     "dependent FMAs per visit, TD/TA 1.0 -> 2.0, the kernel's TD/TA); dependent chains, L2 "
                     "misses, 5 waves/SIMD, LDS reads and dword loads do not (0.93-1.13x). TD busy therefore "
                     "overstates the gather unit's use; the TA (address) fraction agrees with the rate-based frac.",
        "source": os.path.relpath(TD_MIX, ROOT) + " (profiles/r05_logs/r05o)",
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


# ------------------------------------------------------------- launching

def spawn_child(extra_env, deadline_s, argv):
    """Run this script again as a FRESH process (never a re-exec: the caller
    has not touched the GPU, and the child is a new program) with `argv`,
    relaying its output. A child still running after `deadline_s` seconds
    (a rank stuck in RCCL init or a gather) is terminated (killed 5 s later if
    it ignores that) and 124 is returned, so the driver records a failure
    instead of waiting out its own limit."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK")}
    env.update(extra_env)
    p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env)
    try:
        return p.wait(timeout=deadline_s)
    except subprocess.TimeoutExpired:
        print(f"bench.py: the measuring process (pid {p.pid}) is still running after the {deadline_s:.0f} s "
              "deadline (--rank-timeout); terminating it", file=sys.stderr, flush=True)
        p.terminate()
        try:
            p.wait(timeout=5.0)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
        return 124


def child_argv():
    """This process's arguments plus --measure-child (for spawn_child)."""
    return [a for a in sys.argv[1:] if a != "--measure-child"] + ["--measure-child"]


def launcher_main(args, world_env, rank):
    """N > 1 (or --dry): the parent / every torchrun rank. Rank 0 (or the
    lone parent) measures in one fresh child over all N GPUs; other torchrun
    ranks only meet rank 0 at the end."""
    import datetime

    import torch.distributed as dist
    pg = world_env > 1
    if pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.rank_timeout + 60.0))
    rc = 0
    if rank == 0:
        q = args.hw_queues if args.hw_queues >= 0 else (HW_QUEUES_MULTI if args.gpus > 1 else HW_QUEUES_SINGLE)
        env = {}
        if q and not args.dry:
            try:
                have = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
            except ValueError:
                have = 0
            if have < q:
                env["GPU_MAX_HW_QUEUES"] = str(q)
        fd, partial = tempfile.mkstemp(prefix="mirt_bench_", suffix=".json")
        os.close(fd)
        os.remove(partial)        # the child creates it once the headline is measured
        env[PARTIAL_ENV] = partial
        try:
            rc = spawn_child(env, args.rank_timeout, child_argv())
            if os.path.exists(partial):
                # the child measured the headline, then did not finish (its
                # status is in the line): print the saved line in its place
                with open(partial) as f:
                    part = json.load(f)
                part["measuring_process_exit"] = rc
                print(f"bench.py: the measuring process exited {rc} after saving its headline; printing the "
                      "saved line (the unfinished leg is marked in other_delivery)", file=sys.stderr, flush=True)
                print(json.dumps(part), flush=True)
                rc = 0
        finally:
            if os.path.exists(partial):
                os.remove(partial)
    if pg:
        # the job ends together: rank 0 reports the child's status
        t = torch.tensor([rc], dtype=torch.int64)
        dist.broadcast(t, src=0)
        rc = int(t[0])
        dist.barrier()
        dist.destroy_process_group()
    return rc


def dry_main(args):
    """CPU plumbing check (the measuring child with --dry): synthetic shard
    slabs through both deliveries' index math (shard.py's restatements of
    multi.hip's deinterleave_kernel and strided host copies), the frame plan
    and the timing. MIRT_BENCH_DRY_HANG=1 makes the child hang (the deadline
    tests; "after-headline": the child saves its line as measure() does
    before the secondary leg, then hangs)."""
    if os.environ.get("MIRT_BENCH_DRY_HANG") == "1":
        time.sleep(3600)
    n = args.gpus
    frames = frames_per_launch(args, n)
    slabs = []
    for s in range(n):
        fd = mirt.frame_desc(W, H, depth=DEPTH, row_block=ROW_BLOCK, shard=s, num_shards=n)
        rows = mirt.shard_rows(fd).astype(np.int64)
        # frame j's pixel (y, x) = j * H * W + y * W + x
        slabs.append(np.stack([(j * H + rows[:, None]) * W + np.arange(W) for j in range(frames)]).astype(np.int64))
    want = np.arange(frames * H * W, dtype=np.int64).reshape(frames, H, W)
    t0 = time.perf_counter()
    got_g = shard.assemble_gather(slabs, H, ROW_BLOCK)
    got_d = shard.assemble_direct(slabs, H, ROW_BLOCK)
    dt = time.perf_counter() - t0
    ok = bool((got_g == want).all() and (got_d == want).all())
    line = {"metric": METRIC, "value": None, "unit": "Mrays/s", "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "dry": True,
            "data": "synthetic slabs (no rendering): launcher / shard geometry / delivery plumbing check",
            "frame_assembled_ok": ok, "assemble_ms": round(dt * 1e3, 3),
            "config": {"workload": WORKLOADS[args.workload]["desc"], "name": args.workload,
                       "frames_per_launch": frames, "delivery": "gather" if n == 1 else "host-direct",
                       "parallelism": f"row-block shard x{n}, one process (mirt_multi)"}}
    if os.environ.get("MIRT_BENCH_DRY_HANG") == "after-headline":
        save_partial(line, n, args)
        time.sleep(3600)
    drop_partial()
    print(json.dumps(line), flush=True)
    return 0


# ------------------------------------------------------------- the frame loop

def frame_desc_for(f0, n, depth, accumulate):
    """The descriptor of a launch of frames f0 .. f0 + n - 1: fresh frames
    (main.c:358-374) of RNG samples f0 * SPP ..., or successive frames of
    the still-camera display loop (main.c:379-408) with --accumulate; a
    frame of SPP > 1 jittered samples is one launch of its own."""
    acc = accumulate and f0 > 0
    return mirt.frame_desc(W, H, depth=depth, seed=SEED, sample=f0 * SPP, accumulate=acc,
                           frames=f0 * SPP + 1 if acc else 1, row_block=ROW_BLOCK, samples=SPP if n == 1 else 1,
                           jitter=JITTER)


def plan(f0, steps, per, ramp=0):
    """(first frame, frames) of the launches covering `steps` frames from f0;
    `ramp`: the first `ramp` launches carry one frame each (their frames are
    done, and their delivery starts, before a full launch's would be)"""
    out, f, end = [], f0, f0 + steps
    while f < end:
        k = min(1 if len(out) < ramp else per, end - f)
        out.append((f, k))
        f += k
    return out


def run_launches(m, cam, launches, bufs, depth, accumulate=False, tail=(), device_only=False):
    """Enqueue every launch (on lane m.launches % lanes, frame j into
    bufs[lane][j]; device_only: the frames stay on the devices)."""
    seq = []
    for f0, k in launches:
        # the display loop's first frame is fresh, a launch of its own
        # (several frames with accumulate = 0 are successive FRESH frames)
        seq += [(0, 1), (1, k - 1)] if accumulate and f0 == 0 and k > 1 else [(f0, k)]
    for f0, k in seq:
        lane = m.launches % m.lanes
        outs = None if device_only else bufs[lane][:k]
        t0 = time.perf_counter()
        m.render_frames_async(cam, frame_desc_for(f0, k, depth, accumulate), outs, nframes=k, full_grid=f0 in tail)
        ENQUEUE.append(time.perf_counter() - t0)


# host time of each render_frames_async call of the last loop (the enqueue of
# every rank's launch; at N GPUs one host thread issues N ranks' work)
ENQUEUE = []


def timed_loop(m, cam, warm, timed_launches, bufs, depth, accumulate=False, tail=(), device_only=False):
    """Warm-up launches, then the timed ones bracketed by mirt_multi_wait on
    both sides (every frame delivered when the clock stops); seconds."""
    run_launches(m, cam, warm, bufs, depth, accumulate, (), device_only)
    m.wait()
    ENQUEUE.clear()
    t0 = time.perf_counter()
    run_launches(m, cam, timed_launches, bufs, depth, accumulate, tail, device_only)
    m.wait()
    return time.perf_counter() - t0


def prime(m, cam, bufs, per):
    """Untimed, before the warm-up steps: two launches per lane through every
    page-locked buffer and two without a delivery. A process's first frame
    loop into host memory ran ~9 ms slower than the same loop repeated
    (profiles/r05_logs/r05f/n1_sweep.log: 4 lanes, K = 20, 1,635 -> 2,558 Mrays/s;
    device-only 2,557 -> 2,658), a one-off start-up cost of the copy path,
    not part of the steady frame loop the metric describes."""
    run_launches(m, cam, plan(0, 2 * m.lanes * per, per), bufs, DEPTH)
    run_launches(m, cam, plan(0, 2 * m.lanes * per, per), bufs, DEPTH, device_only=True)
    m.wait()


def make_scene():
    spheres = (mirt.create_random_spheres(NSPH, SEED) if KIND == "render"
               else mirt.create_benchmark_spheres(NSPH, SEED))
    t0 = time.perf_counter()
    bvh = mirt.build_bvh(spheres)
    return spheres, bvh, time.perf_counter() - t0


# --same-device (rehearsal on a one-GPU box): the N ranks all on GPU 0 -- the
# copy exchange instead of RCCL, otherwise the N > 1 flow of a real node
SAME_DEVICE = False


def devices_for(n):
    return [0] * n if SAME_DEVICE else list(range(n))


def open_multi(n, lanes, host_direct, spheres, bvh, blocks, opts, timeout_ms=120000, ahead=False):
    m = mirt.MultiRenderer(devices_for(n), lanes=lanes, host_direct=host_direct, queue_ahead=ahead)
    m.set_option(mirt.abi.MULTI_OPT_TIMEOUT_MS, timeout_ms)
    for ov in opts:   # before the upload (an option may shape the layout the upload builds)
        o, v = (int(t) for t in ov.split("="))
        m.set_option(o, v)
    m.upload(spheres, bvh)
    if blocks >= 0:
        m.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, blocks)
    return m


def host_bufs(lanes, per):
    return [[mirt.HostBuffer((H, W, 4)) for _ in range(per)] for _ in range(lanes)]


def close_bufs(bufs):
    for lane in bufs:
        for b in lane:
            b.close()


def frames_per_launch(args, n):
    if SPP > 1 and not args.accumulate:
        return 1             # one fresh frame of SPP samples per launch (the fold restarts per launch)
    return args.batch if args.batch > 0 else DEFAULT_BATCH.get(n, 1 if n <= 2 else 4)


def queue_ahead(args, n):
    """MIRT_MULTI_QUEUE_AHEAD for the timed loop (two launch slots per context)."""
    return bool(args.queue_ahead) if args.queue_ahead >= 0 else (QUEUE_AHEAD if n == 1 else QUEUE_AHEAD_MULTI)


def schedule(args, n):
    """(lanes, frames per launch, tail launches, bounce workgroups) of the timed loop at n GPUs."""
    lanes = args.pipeline or (4 if n == 1 else PIPELINE_MULTI)
    per = frames_per_launch(args, n)
    tail = args.tail_grid if args.tail_grid >= 0 else (TAIL_GRID if n == 1 else TAIL_GRID_MULTI)
    blocks = args.bounce_blocks
    if blocks < 0:
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        blocks = int(WORKLOADS[WORKLOAD].get("BB_PER_CU", 1.5) * cus) if lanes > 1 else 0
    return lanes, per, tail, blocks


def tail_of(launches, tail, lanes, blocks):
    if lanes < 2 or not blocks or tail <= 0:
        return set()
    return {f0 for f0, _ in launches[-tail:]}


def last_delivered(m, bufs, launches):
    """The last frame a timed loop delivered (host copy)."""
    f0, k = launches[-1]
    return bufs[(m.launches - 1) % m.lanes][k - 1].array.copy(), (f0 + k - 1) * SPP


def measure(args):
    """The GPU measurement over args.gpus devices in THIS process. The
    headline delivers every frame to page-locked host memory (SURVEY §8(d)
    t_frame): at N = 1 the rank's slab is the frame (one D2H); at N > 1 by
    default every GPU copies its row blocks into the host frame (host-direct),
    and the RCCL gather to GPU 0 is measured beside it -- with the frames
    then copied to the host (value_gather) and left on GPU 0
    (device_resident_mrays_s)."""
    n = args.gpus
    delivery = args.delivery if args.delivery != "auto" else ("gather" if n == 1 else "host-direct")
    lanes, per, tail_n, blocks = schedule(args, n)
    spheres, bvh, build_s = make_scene()
    cam = mirt.default_camera()
    ahead = queue_ahead(args, n)
    m = open_multi(n, lanes, delivery == "host-direct", spheres, bvh, blocks, args.opt, ahead=ahead)
    bufs = host_bufs(m.lanes, per)
    prime(m, cam, bufs, per)
    warm = plan(0, args.warmup, per)
    timed_launches = plan(args.warmup, args.steps, per)
    tail = tail_of(timed_launches, tail_n, lanes, blocks)
    elapsed = timed_loop(m, cam, warm, timed_launches, bufs, DEPTH, args.accumulate, tail)
    enqueue_ms = [round(float(np.median(ENQUEUE)) * 1e3, 4), round(float(np.max(ENQUEUE)) * 1e3, 4)]
    last_frame, last_sample = last_delivered(m, bufs, timed_launches)
    # the passes of rank 0's timed launches (HIP events on each launch's own
    # stream, under the overlap of the lanes in flight)
    phases = []
    for lane in range(lanes):   # the context sets (with queue-ahead two launch slots share one)
        k_lane = sum(1 for i in range(len(warm), len(warm) + len(timed_launches)) if i % m.lanes % lanes == lane)
        if k_lane:
            phases += m.phase_log(lane, 0, min(k_lane, 64))
    primary_ms, bounce_ms = (float(v) for v in np.mean(np.array(phases), axis=0)) if phases else (0.0, 0.0)
    # depth 1 (camera rays and their shading only), frames to host memory, and
    # (one GPU) the same loop with the frames left on the device
    el_d1 = timed_loop(m, cam, plan(0, 2, per), plan(args.warmup, args.steps, per), bufs, 1, False, tail)
    el_d1_dev = None
    if n == 1:
        el_d1_dev = timed_loop(m, cam, plan(0, 2, per), plan(args.warmup, args.steps, per), bufs, 1, False, tail,
                               device_only=True)
    # the same loop with the frames left on the device(s): N = 1 in the
    # rank's slabs; N > 1 gathered on GPU 0 over RCCL (below)
    el_dev = None
    if n == 1:
        el_dev = timed_loop(m, cam, plan(0, 2, per), plan(args.warmup, args.steps, per), bufs, DEPTH,
                            args.accumulate, tail, device_only=True)
    m.close()
    close_bufs(bufs)
    # the last delivered frame against one context rendering the same frame
    # alone (the N-GPU frame must equal the one-GPU frame byte for byte);
    # checked before the other delivery runs, so a failure there cannot cost it
    same = None
    if not args.accumulate:
        with mirt.Renderer(0) as r1:
            r1.upload(spheres, bvh)
            one = r1.render_frame(cam, W, H, depth=DEPTH, seed=SEED, sample=last_sample, samples=SPP, jitter=JITTER)
            same = frame_sha(one) == frame_sha(last_frame)
    value = W * H * SPP * args.steps / elapsed / 1e6
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (create_random_sphere scene, srand(1); default camera main.c:203-211)",
        "config": {"workload": WORKLOADS[WORKLOAD]["desc"], "name": WORKLOAD,
                   "width": W, "height": H, "spheres": NSPH, "scene": KIND, "max_depth": DEPTH, "spp": SPP,
                   "jitter": JITTER, "frames_per_step": 1, "frames_per_launch": per,
                   "launches": len(timed_launches), "pipeline": lanes, "queue_ahead": ahead,
                   "bounce_blocks": blocks,
                   "tail_grid": len(tail), "bvh_nodes": len(bvh), "row_block": ROW_BLOCK,
                   "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                   "delivery": delivery,
                   "step": ("1 frame of the still-camera display loop (main.c:379-408), lanes sharing one "
                            "accumulation buffer" if args.accumulate else "1 fresh frame (main.c:358-374)")
                           + f", {SPP} sample(s), {per} frame(s) per launch, launches rotating over {lanes} lanes, "
                             "every frame delivered to page-locked host memory",
                   "parallelism": ("one GPU, one process: mirt_multi with one rank (no exchange: the rank's slab "
                                   "is the frame), one D2H per frame" if n == 1 else
                                   f"row-block shard x{n}, one process: mirt_multi, "
                                   + ("RCCL gather to GPU 0 (ncclCommInitAll communicators) + D2H"
                                      if delivery == "gather" else "per-GPU strided D2H into the host frame"))},
        "timing": "one process drives all GPUs (include/mirt_multi.h); the timed region is bracketed by "
                  "mirt_multi_wait on both sides, so it ends when every frame is in host memory on every lane",
        "device_resident_mrays_s": round(W * H * SPP * args.steps / el_dev / 1e6, 3) if el_dev else None,
        "device_resident_note": ("the same launches with the frames left in device memory (no D2H)" if n == 1 else
                                 "the same launches with every frame gathered on GPU 0 over RCCL and "
                                 "de-interleaved there (no D2H)"),
        "depth1_mrays_s": round(W * H * SPP * args.steps / el_d1 / 1e6, 3),
        "depth1_device_resident_mrays_s": round(W * H * SPP * args.steps / el_d1_dev / 1e6, 3) if el_d1_dev else None,
        "depth1_note": "depth 1 through the same loop: frames delivered to page-locked host memory (depth1_mrays_s; "
                       "a 1080p frame's D2H is 0.155 ms at the link's 53.5 GB/s) and left in HBM "
                       "(depth1_device_resident_mrays_s)",
        "bvh_build_s": round(build_s, 4),
        "frame_sha_last": frame_sha(last_frame),
        "last_frame_equals_one_context": same,
        "phases_under_overlap_ms": {"primary": round(primary_ms, 4), "bounce": round(bounce_ms, 4),
                                    "launches": len(phases)},
        "host_enqueue_ms_per_launch": {"median": enqueue_ms[0], "max": enqueue_ms[1],
                                       "note": "host time of one mirt_multi_render_frames_async (every rank's "
                                               "launch issued from this one thread; includes waiting for the "
                                               "lane's previous launch)"},
    }
    if n > 1:
        line["reference_work"] = multi_reference_work(spheres, bvh, cam, n, elapsed, args.steps)
    if SAME_DEVICE:
        line["rehearsal_same_device"] = "every rank on GPU 0 (copy exchange): a plumbing rehearsal, not a measurement"
    if args.opt:
        line["options"] = args.opt
    save_partial(line, n, args)
    # the other delivery at N > 1: the RCCL gather to GPU 0, to host memory
    # and device-resident (a second renderer, same schedule). It is measured
    # BESIDE the headline: an error in it (the n-GPU RCCL exchange has not run
    # on a multi-GPU node before) is reported in the line, not raised, and its
    # waits are bounded by a shorter timeout so a stuck exchange fails fast.
    other = None
    if n > 1 and not args.no_other:
        od = "gather" if delivery == "host-direct" else "host-direct"
        other = {"delivery": od}
        m2 = bufs2 = None
        try:
            m2 = open_multi(n, lanes, od == "host-direct", spheres, bvh, blocks, args.opt, timeout_ms=60000,
                            ahead=ahead)
            bufs2 = host_bufs(m2.lanes, per)
            prime(m2, cam, bufs2, per)
            tl2 = plan(args.warmup, args.steps, per)
            el2 = timed_loop(m2, cam, plan(0, args.warmup, per), tl2, bufs2, DEPTH, args.accumulate, tail)
            other_frame = last_delivered(m2, bufs2, tl2)
            other.update({"mrays_s": round(W * H * SPP * args.steps / el2 / 1e6, 3),
                          "ms_per_step": round(el2 / args.steps * 1e3, 4), "backend": m2.backend,
                          "lead_skip_option": m2.get_option(mirt.abi.MULTI_OPT_LEAD_SKIP)})
            if od == "gather":
                el_dev = timed_loop(m2, cam, plan(0, 2, per), plan(args.warmup, args.steps, per), bufs2, DEPTH,
                                    args.accumulate, tail, device_only=True)
            if not args.accumulate:
                with mirt.Renderer(0) as r1:
                    r1.upload(spheres, bvh)
                    one2 = r1.render_frame(cam, W, H, depth=DEPTH, seed=SEED, sample=other_frame[1], samples=SPP,
                                           jitter=JITTER)
                    other["last_frame_equals_one_context"] = frame_sha(one2) == frame_sha(other_frame[0])
        except Exception as e:   # noqa: BLE001 -- reported in the line, the headline stands
            other["error"] = f"{type(e).__name__}: {e}"
            print(f"bench.py: the {od} leg failed: {other['error']}", file=sys.stderr, flush=True)
        finally:
            if m2 is not None:
                try:   # what the n-GPU exchange issued (mirt_multi_get_stats): RCCL calls, bytes, copies
                    other["exchange_stats"] = m2.stats()
                except Exception as e:   # noqa: BLE001
                    other["exchange_stats_error"] = str(e)
                m2.close()
            if bufs2 is not None:
                close_bufs(bufs2)
        if not args.accumulate and "error" not in other:
            # one blocking frame through a ONE-lane renderer of that delivery (the
            # simplest form of the n-GPU exchange) against one context's frame
            try:
                with mirt.MultiRenderer(devices_for(n), lanes=1, host_direct=od == "host-direct") as m1:
                    m1.set_option(mirt.abi.MULTI_OPT_TIMEOUT_MS, 60000)
                    m1.upload(spheres, bvh)
                    f1 = m1.render_frame(cam, W, H, depth=DEPTH, seed=SEED, sample=0, samples=SPP, jitter=JITTER)
                with mirt.Renderer(0) as r1:
                    r1.upload(spheres, bvh)
                    one1 = r1.render_frame(cam, W, H, depth=DEPTH, seed=SEED, sample=0, samples=SPP, jitter=JITTER)
                other["one_lane_frame_equals_one_context"] = frame_sha(f1) == frame_sha(one1)
            except Exception as e:   # noqa: BLE001
                other["one_lane_error"] = f"{type(e).__name__}: {e}"

    if other:
        line["value_" + other["delivery"].replace("-", "_")] = other.get("mrays_s")
        line["other_delivery"] = other
    if el_dev:
        line["device_resident_mrays_s"] = round(W * H * SPP * args.steps / el_dev / 1e6, 3)
    if n == 1:
        line.update(single_gpu_extras(args, spheres, bvh, cam, value, elapsed, bounce_ms, primary_ms, per))
    drop_partial()
    print(json.dumps(line), flush=True)
    return 0


# N > 1: the measuring child saves its line here once the headline loop and
# its frame check are done, before the other delivery's leg (whose n-GPU RCCL
# exchange has not yet run on a multi-GPU node). If the child is then stopped
# at the deadline or dies, the parent prints this line, so a stuck secondary
# leg cannot cost the headline; the file is removed before the child prints.
PARTIAL_ENV = "MIRT_BENCH_PARTIAL"


def save_partial(line, n, args):
    path = os.environ.get(PARTIAL_ENV)
    if not path or n == 1:
        return
    part = dict(line)
    if not args.no_other:
        od = "gather" if part["config"]["delivery"] == "host-direct" else "host-direct"
        part["other_delivery"] = {"delivery": od, "error": "not finished: the measuring process ended in this leg "
                                                           "(terminated at --rank-timeout, or died); this line was "
                                                           "saved before it"}
    with open(path + ".tmp", "w") as f:
        json.dump(part, f)
    os.replace(path + ".tmp", path)


def drop_partial():
    path = os.environ.get(PARTIAL_ENV)
    if path:
        try:
            os.remove(path)
        except FileNotFoundError:
            pass


def multi_reference_work(spheres, bvh, cam, n, elapsed, steps):
    """N > 1, SURVEY §8(e)'s scaling figure: the REFERENCE's exhaustive-DFS
    bytes of one frame (the same at every N: the frame does not change) per
    second of the timed loop, over N GPUs' HBM peak -- B / t / (G x 8 TB/s).
    Counted by the instrumented build on GPU 0 (pruning off), after the
    measurement."""
    try:
        with mirt.Renderer(0) as r:
            r.upload(spheres, bvh)
            r.set_option(mirt.abi.OPT_PRUNE, 0)
            ref = r.count_frame(cam, W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, samples=SPP, jitter=JITTER)
        b = algorithmic_bytes(ref, H * W * SPP)
        gbs = b * steps / elapsed / 1e9
        return {"definition": "SURVEY 8(d)/(e): the reference's exhaustive-DFS bytes per frame (32 B/node test + 16 "
                              "B/sphere test + 4 B/hit colour + 4 B/pixel) per second, over G x the HBM peak",
                "bytes_per_frame": int(b), "gbs": round(gbs, 1),
                "frac_of_g_hbm_peak": round(gbs / (n * PEAK_HBM_GBS), 4)}
    except Exception as e:   # noqa: BLE001 -- a counting failure must not cost the line
        return {"error": f"{type(e).__name__}: {e}"}


def single_gpu_extras(args, spheres, bvh, cam, value, elapsed, bounce_ms, primary_ms, per):
    """N = 1: the work counters, the serial launch, the roofline, the blocking
    call and the CPU baseline."""
    r = mirt.Renderer(0)
    r.upload(spheres, bvh)
    samples = SPP * per
    counts = r.count_frame(cam, W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, samples=samples, jitter=JITTER)
    r.set_option(mirt.abi.OPT_PRUNE, 0)
    ref_counts = r.count_frame(cam, W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, samples=samples,
                               jitter=JITTER)
    r.set_option(mirt.abi.OPT_PRUNE, 1)
    # the same launch alone, serial, full persistent grid: torch events
    # around the launch and the library's HIP events around its passes
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    fd = mirt.frame_desc(W, H, depth=DEPTH, seed=SEED, row_block=ROW_BLOCK, samples=samples, jitter=JITTER)
    slabs = torch.zeros((samples, H, W), dtype=torch.int32, device="cuda")
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda") if SPP > 1 else None
    phases, launch = [], []
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
    pixels = H * W * samples
    ref_frame_bytes = algorithmic_bytes(ref_counts, pixels)
    exec_frame_bytes = algorithmic_bytes(counts, pixels)
    ref_b = bounce_bytes(ref_counts)
    exec_b = bounce_bytes(counts)
    achieved = ref_b / (max(bounce_ms, 1e-6) / 1e3) / 1e9
    pmc, pmc_path = load_pmc_bound(WORKLOAD)
    pb = pmc["kernels"].get("timed/bounce", {}).get("derived", {}) if pmc else {}
    pp = pmc["kernels"].get("timed/primary", {}).get("derived", {}) if pmc else {}
    traffic = pb.get("hbm_bytes")
    bm = bound_line(pb, exec_b, ref_b, pb.get("kernel_ms_at_2400MHz") or bounce_ms)
    kname = KERNEL.replace("<true, 2,", "<true, 4,") if r.get_option(mirt.abi.OPT_LEAF_BATCH) else KERNEL
    roof = vmem_roofline(pmc, pmc_path, elapsed / args.steps * 1e3, per)
    if roof is None:
        roof = {"bound": "vmem", "achieved": None, "peak": None, "unit": "Ginst/s", "frac": None,
                "traffic": traffic, "note": "no profiles/r0N_pmc_bound_<workload>.json or td_probe table for "
                                            "this workload"}
    roof["kernel"] = kname
    if bm:
        bm["source"] = (os.path.relpath(pmc_path, ROOT) + " (medians over the dispatches of the timed launch shape, "
                        "one rocprofv3 --pmc pass of this command per counter set; rocprofv3 serialises the "
                        "dispatches it counts)")
    # the blocking leg in THIS process, after the timed burst (beside the
    # child's figure below: zero-copy stores ran ~3% slower here)
    after_burst = None
    if not args.no_host:
        try:
            ab = blocking_leg(r, cam, n=11)
            after_burst = {k: ab[k] for k in ("pinned_ms", "pinned_mrays_s", "registered_mrays_s",
                                              "pageable_mrays_s", "equal")}
        except Exception as e:   # noqa: BLE001 -- an extra figure must not cost the line
            after_burst = {"error": f"{type(e).__name__}: {e}"}
    r.close()
    out = {
        "roofline": roof,
        # SURVEY 8(d)'s figure, kept beside the roofline under its own name: the REFERENCE's work per second,
        # not a use of any unit (it exceeds HBM peak because the walk skips most of it from cache)
        "reference_work": {
            "definition": "SURVEY 8(d): bytes of the REFERENCE's exhaustive DFS (hit.c:91-109, no pruning) at "
                          "32 B/node test + 16 B/sphere test + 4 B/hit colour + 4 B/pixel, per second. The walk "
                          "executes a fraction of them (executed_vs_reference) from an L2/MALL-resident tree, so "
                          "this is the reference's work replaced per second, not HBM use.",
            "bounce_bytes_per_launch": int(ref_b),
            "bounce_launch_ms_under_overlap": round(bounce_ms, 4),
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
            "frame_reference_gbs": round(ref_frame_bytes / per / (elapsed / args.steps) / 1e9, 1),
            "serial_launch": {
                "note": "the same launch alone (untimed serial loop, the full persistent bounce grid): not the "
                        "timed configuration",
                "frame_ms": round(kernel_ms, 4), "primary_ms": round(serial_primary_ms, 4),
                "bounce_ms": round(serial_bounce_ms, 4),
                "bounce_reference_gbs": round(ref_b / (serial_bounce_ms / 1e3) / 1e9, 1)}},
        "work": {k: int(v) for k, v in counts.items()},
        "work_reference_dfs": {k: int(v) for k, v in ref_counts.items() if k != "lane_steps"},
        "traced_rays_per_s_M": round(counts["rays"] / per / (elapsed / args.steps) / 1e6, 3),
    }
    if not args.no_host:
        child = blocking_in_child()
        if child:
            out.update({"host_blocking_mrays_s": child["pinned_mrays_s"], "host_blocking_ms": child["pinned_ms"],
                        "host_blocking_registered_mrays_s": child["registered_mrays_s"],
                        "host_blocking_pageable_mrays_s": child["pageable_mrays_s"],
                        "host_blocking_equals_frames": child["equal"],
                        "host_blocking_sha": child["sha"],
                        "host_blocking_method": (
                            "one blocking mirt_render_frame per frame (main.c:350-421's loop) into a frame buffer "
                            "from mirt_host_alloc: the kernels write the pixels straight into it "
                            "(MIRT_OPT_ZERO_COPY), median of 11, in a child process holding one ctx and its frame "
                            "buffer, as main.c's loop runs (bench.py --blocking-child); pageable = the caller's "
                            "plain malloc'd buffer, the same process")})
        if after_burst:
            after_burst["note"] = ("the same blocking leg in the bench's own process after the timed burst "
                                   "(pinned = zero-copy into mirt_host_alloc memory, pageable = a malloc'd buffer)")
            out["host_blocking_after_burst"] = after_burst
    if not args.no_cpu:
        cb = cpu_baseline()
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu"] = round(value / cb["value"], 1)
        out["speedup_vs_cpu_single_core"] = round(value / cb["single_core_value"], 1)
        out["speedup_vs_cpu_all_core_estimate"] = round(value / cb["all_core_estimate"]["value"], 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-host", action="store_true", help="skip the blocking-call leg (child process)")
    ap.add_argument("--no-other", action="store_true", help="N > 1: skip the other delivery's leg")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="1080p_10k")
    ap.add_argument("--delivery", choices=("auto", "gather", "host-direct"), default="auto",
                    help="gather: RCCL gather of the slabs to GPU 0, de-interleave, one D2H per frame (SURVEY "
                         "8(e)); host-direct: every GPU copies its row blocks straight into the host frame; "
                         "auto: gather at N = 1 (no exchange: the slab is the frame), host-direct at N > 1 (one "
                         "host link cannot carry the frame rate of 8 GPUs: DESIGN §7)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="lanes of contexts keeping launches in flight (0 = 4 at N = 1, 8 at N > 1)")
    ap.add_argument("--bounce-blocks", type=int, default=-1,
                    help="persistent bounce workgroups per launch (MIRT_OPT_BOUNCE_BLOCKS); -1 = the workload's "
                         "BB_PER_CU (1.5 unless stated) per CU with lanes > 1, else 0 (occupancy x CUs)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per launch (0 = DEFAULT_BATCH[N])")
    ap.add_argument("--queue-ahead", type=int, default=-1,
                    help="1: two launch slots per context (MIRT_MULTI_QUEUE_AHEAD), 0: one; default per N")
    ap.add_argument("--tail-grid", type=int, default=-1,
                    help="the last N launches of the timed burst take the full persistent bounce grid; -1 = "
                         "TAIL_GRID at N = 1, TAIL_GRID_MULTI at N > 1")
    ap.add_argument("--accumulate", action="store_true",
                    help="time the still-camera accumulating display loop instead of fresh frames")
    ap.add_argument("--dry", action="store_true", help="CPU plumbing check (no GPU, no measurement)")
    ap.add_argument("--rank-timeout", type=float, default=420.0,
                    help="N > 1: seconds before a still-running measuring process is terminated (exit 124)")
    ap.add_argument("--hw-queues", type=int, default=-1,
                    help="GPU_MAX_HW_QUEUES for the measuring process (-1: the environment's at N = 1, 16 at "
                         "N > 1; 0: keep the environment's)")
    ap.add_argument("--measure-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: all N ranks on GPU 0 (copy exchange, no RCCL); not a measurement")
    ap.add_argument("--blocking-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--opt", action="append", default=[],
                    help="OPTION=VALUE (mirt_multi_set_option on every context), repeatable")
    args = ap.parse_args()
    global W, H, NSPH, KIND, SPP, JITTER, WORKLOAD, SAME_DEVICE
    SAME_DEVICE = args.same_device
    WORKLOAD = args.workload
    wl = WORKLOADS[args.workload]
    W, H, NSPH, KIND, SPP, JITTER = wl["W"], wl["H"], wl["NSPH"], wl["KIND"], wl["SPP"], wl["JITTER"]

    if args.blocking_child:
        return blocking_child()
    if args.measure_child:
        return dry_main(args) if args.dry else measure(args)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world_env > 1 and world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} under WORLD_SIZE {world_env}: measuring {args.gpus} GPU(s) from rank 0",
              file=sys.stderr)
    if args.gpus > 1 or args.dry or world_env > 1:
        return launcher_main(args, world_env, rank)
    return measure(args)


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
