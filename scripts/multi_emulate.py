"""Per-shard emulation of bench.py's N-GPU timed loop on ONE GPU, through the
same C-ABI path the N-GPU run takes (include/mirt_multi.h): a one-rank
mirt_multi with MIRT_MULTI_OPT_EMULATE_WORLD = N / _RANK = k renders shard k
of every frame with bench.py's schedule at N (lanes, frames per launch, the
1.5-per-CU bounce grid, the burst's last launches on the full grid), and
delivers what rank k delivers at N GPUs:
  gather:      its slabs through RCCL (a self send/recv on the one device) and,
               as rank 0, the other shards' receives (HBM writes), the
               de-interleave and every frame's D2H into page-locked memory;
  host-direct: its own strided copies of its row blocks into the host frames.
Rank k's time at N GPUs is its time here (xGMI wire time and cross-GPU
interference aside), so the job's predicted rate is W*H*K / max_k(t_k).

    python scripts/multi_emulate.py --worlds 1,2,4,8 [--delivery gather|host-direct] [--steps 20]

The script raises GPU_MAX_HW_QUEUES to --hw-queues (16, as bench.py's N > 1
measuring child) before the HIP runtime starts; pass 0 to keep the
environment's (bench.py's N = 1 leg keeps it).
"""
import argparse
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
mirt = bench.mirt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--workload", default="1080p_10k", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--delivery", default="gather", choices=("gather", "host-direct"))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5,
                    help="measure every shard this many times, rounds interleaved across the shards")
    ap.add_argument("--ranks", default="", help="only these shards (comma list; default every shard)")
    ap.add_argument("--pipeline", type=int, default=0)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--ramp", type=int, default=0, help="the timed region's first RAMP launches carry one frame each")
    ap.add_argument("--tail-grid", type=int, default=-1)
    ap.add_argument("--bounce-blocks", type=int, default=-1)
    ap.add_argument("--accumulate", action="store_true")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--hw-queues", type=int, default=16)
    ap.add_argument("--device-only", action="store_true", help="frames left on the devices (no delivery to host)")
    ap.add_argument("--sweep", default="", help="LANES:BATCH:TAIL[,...] schedules to emulate instead of the bench's")
    ap.add_argument("--direct-copy", type=int, default=0, help="MIRT_MULTI_OPT_DIRECT_COPY for host-direct")
    ap.add_argument("--queue-ahead", type=int, default=-1, help="MIRT_MULTI_QUEUE_AHEAD (default: bench.py's per N)")
    ap.add_argument("--row-block", type=int, default=8, help="rows per interleaved shard block (fd->row_block)")
    a = ap.parse_args()
    if a.hw_queues and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < a.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)   # before the first HIP call of this process
    wl = bench.WORKLOADS[a.workload]
    bench.WORKLOAD = a.workload
    bench.W, bench.H, bench.NSPH, bench.KIND, bench.SPP, bench.JITTER = (wl["W"], wl["H"], wl["NSPH"], wl["KIND"],
                                                                          wl["SPP"], wl["JITTER"])
    W, H, SPP = bench.W, bench.H, bench.SPP
    bench.ROW_BLOCK = a.row_block
    spheres, bvh, _ = bench.make_scene()
    cam = mirt.default_camera()
    combos = [tuple(int(v) for v in c.split(":")) for c in a.sweep.split(",")] if a.sweep else [None]
    for world, combo in ((int(w), c) for w in a.worlds.split(",") for c in combos):
        if combo:
            a.pipeline, a.batch, a.tail_grid = combo
        lanes, per, tail_n, blocks = bench.schedule(a, world)
        ahead = bench.queue_ahead(a, world)
        m = bench.open_multi(1, lanes, a.delivery == "host-direct", spheres, bvh, blocks, a.opt, ahead=ahead)
        m.set_option(mirt.abi.MULTI_OPT_DIRECT_COPY, a.direct_copy)
        bufs = bench.host_bufs(m.lanes, per)
        bench.prime(m, cam, bufs, per)
        timed = bench.plan(a.warmup, a.steps, per, a.ramp)
        tail = bench.tail_of(timed, tail_n, lanes, blocks)
        ranks = [int(k) for k in a.ranks.split(",")] if a.ranks else list(range(world))
        runs, enq, enq_runs = {k: [] for k in ranks}, [], []
        for _ in range(a.rounds):          # rounds interleaved across the shards
            for k in ranks:
                m.emulate(world, k)
                el = bench.timed_loop(m, cam, bench.plan(0, a.warmup, per), timed, bufs, bench.DEPTH, a.accumulate,
                                      tail, device_only=a.device_only)
                runs[k].append(el)
                enq += bench.ENQUEUE
                enq_runs.append([round(x * 1e3, 3) for x in bench.ENQUEUE])
        st = m.stats()
        m.close()
        bench.close_bufs(bufs)
        med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
        per_rank = [med[k] for k in ranks]
        slow = max(per_rank)
        best_slow = max(min(v) for v in runs.values())
        print(json.dumps({
            "workload": a.workload, "delivery": "device-only" if a.device_only else a.delivery,
            "direct_copy": a.direct_copy, "world": world, "steps": a.steps, "warmup": a.warmup,
            "lanes": lanes, "queue_ahead": ahead, "row_block": a.row_block, "frames_per_launch": per, "ramp": a.ramp, "tail_grid": len(tail),
            "bounce_blocks": blocks,
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "ranks": ranks, "rounds": a.rounds,
            "rank_ms_per_frame": [round(t / a.steps * 1e3, 4) for t in per_rank],
            "rank_ms_per_frame_runs": {k: [round(t / a.steps * 1e3, 4) for t in v] for k, v in runs.items()},
            "slowest_rank": ranks[per_rank.index(slow)],
            "enqueue_ms_per_launch_median": round(sorted(enq)[len(enq) // 2] * 1e3, 4) if enq else None,
            "enqueue_ms_first_runs": enq_runs[:3],   # each timed launch's host call, in order
            "estimator": "N x the slowest shard's MEDIAN over the rounds (pred_job_mrays_s); "
                         "pred_job_mrays_s_best: the slowest shard's best round",
            "pred_job_mrays_s": round(W * H * SPP * a.steps / slow / 1e6, 1),
            "pred_job_mrays_s_best": round(W * H * SPP * a.steps / best_slow / 1e6, 1),
            "rccl": {k: st[k] for k in ("comm_inits", "rccl_sends", "rccl_recvs")}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
