"""What the bench's timed loop looks like on the device, from the
`rocprofv3 --kernel-trace` CSV of `bench.py --steps K --warmup W` (the
driver's command): the frames of the timed region are the K frames after the
W warm-up frames of the pipelined launch shape (bounce grid = --bounce-blocks
workgroups; the serial loop later runs the full grid, the depth-1 loop uses
render_kernel). Per kernel: mean dispatch duration UNDER OVERLAP (start ->
end of the dispatch while the other frames in flight share the chip), and
for the region: the union of busy time, the sum of dispatch durations over
it (overlap factor), and the frame period.

    python scripts/timed_profile.py gpurun_out/r03a/prof_timed/run_kernel_trace.csv --steps 20 --warmup 5
"""
import argparse
import csv
import json

BOUNCE = "bounce_kernel<true, 2, false>"   # <true, 4, false> on trees past the L2 (MIRT_OPT_LEAF_BATCH)
PRIMARY = "primary_kernel<true, true>"


def short(name):
    for k in (BOUNCE, BOUNCE.replace("<true, 2,", "<true, 4,"), PRIMARY, "fold_samples_kernel", "mark_deferred_kernel", "render_kernel<true, false>"):
        if k in name:
            return k
    return name.split("(")[0][-60:]


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bounce-grid", type=int, default=384 * 256, help="work-items of a pipelined bounce launch")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the pipelined frames: bounce launches of the pipelined grid, in start order
    bounces = [r for r in rows if BOUNCE in r["Kernel_Name"] and int(r["Grid_Size_X"]) == a.bounce_grid]
    if len(bounces) < a.warmup + a.steps:
        raise SystemExit(f"{len(bounces)} pipelined bounce launches, expected {a.warmup + a.steps}")
    timed = bounces[a.warmup:a.warmup + a.steps]
    # the region: from the first timed frame's primary launch (the dispatch of
    # that frame's primary kernel precedes its bounce on the same queue) to
    # the last timed bounce's end
    prim = [r for r in rows if PRIMARY in r["Kernel_Name"]]
    first_b = timed[0]
    cand = [p for p in prim if p["Queue_Id"] == first_b["Queue_Id"]
            and int(p["End_Timestamp"]) <= int(first_b["Start_Timestamp"]) + 1]
    t0 = int(cand[-1]["Start_Timestamp"]) if cand else int(first_b["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in timed)
    region = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
    per = {}
    for r in region:
        k = short(r["Kernel_Name"])
        per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    busy = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in region]) / 1e6
    summed = sum(sum(v) for v in per.values())
    span = (t1 - t0) / 1e6
    out = {
        "trace": a.trace, "steps": a.steps, "warmup": a.warmup,
        "region_ms": round(span, 4), "frame_period_ms": round(span / a.steps, 4),
        "gpu_busy_union_ms": round(busy, 4), "busy_frac": round(busy / span, 4),
        "sum_of_dispatch_ms": round(summed, 4), "mean_dispatches_in_flight": round(summed / busy, 3),
        "queues": sorted({int(r["Queue_Id"]) for r in region}),
        "kernels": {k: {"dispatches": len(v), "mean_ms_under_overlap": round(sum(v) / len(v), 4),
                        "min_ms": round(min(v), 4), "max_ms": round(max(v), 4),
                        "ms_per_step": round(sum(v) / a.steps, 4)} for k, v in sorted(per.items())},
    }
    # the serial loop that follows (full grid, one launch at a time)
    full = [r for r in rows if BOUNCE in r["Kernel_Name"] and int(r["Grid_Size_X"]) != a.bounce_grid]
    if full:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in full]
        out["serial_full_grid_bounce_ms"] = round(sum(d) / len(d), 4)
        out["serial_full_grid_launches"] = len(d)
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
