"""Timeline of one emulated shard's launches from a rocprofv3 kernel (+ memory
copy) trace of scripts/multi_emulate.py --ranks K: per launch (a primary pass
and its bounce pass on one stream) its start, primary / bounce spans and the
copies behind it, relative to the first dispatch of each timed region, and how
busy the GPU was over the region (union of kernel intervals).

    python scripts/shard_timeline.py gpurun_out/r06n/tr8 [--launches 5] [--warmup 2]
"""
import argparse
import csv
import glob
import os


def rows(d, name):
    out = []
    for f in glob.glob(os.path.join(d, "**", f"*{name}*.csv"), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def union(iv):
    tot, cur = 0, None
    for a, b in sorted(iv):
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    return tot + (cur[1] - cur[0] if cur else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--launches", type=int, default=5, help="launches of a timed region")
    ap.add_argument("--warmup", type=int, default=2, help="launches before each timed region")
    a = ap.parse_args()
    ks = rows(a.dir, "kernel_trace")
    cps = rows(a.dir, "memory_copy_trace")
    ks = [k for k in ks if "primary_kernel" in k["Kernel_Name"] or "bounce_kernel" in k["Kernel_Name"]]
    ks.sort(key=lambda k: int(k["Start_Timestamp"]))
    prim = [k for k in ks if "primary_kernel" in k["Kernel_Name"]]
    per = a.launches + a.warmup
    print(f"{len(prim)} primary passes, {len(ks) - len(prim)} bounce passes, {len(cps)} copies")
    # the last two timed regions: each is `launches` primaries after `warmup` ones
    for reg in range(max(0, len(prim) // per - 2), len(prim) // per):
        ps = prim[reg * per + a.warmup: (reg + 1) * per]
        if len(ps) < a.launches:
            continue
        t0 = int(ps[0]["Start_Timestamp"])
        launches = []
        for p in ps:
            q = p["Queue_Id"] if "Queue_Id" in p else None
            s = int(p["Start_Timestamp"])
            b = next((k for k in ks if "bounce_kernel" in k["Kernel_Name"] and int(k["Start_Timestamp"]) >= s
                      and (q is None or k.get("Queue_Id") == q)), None)
            launches.append((p, b))
        end_k = max(int(b["End_Timestamp"]) for _, b in launches if b)
        cs = [c for c in cps if int(c["Start_Timestamp"]) >= t0]
        end_c = max([int(c["End_Timestamp"]) for c in cs if int(c["Start_Timestamp"]) <= end_k + 2_000_000] or [end_k])
        iv = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"])) for k in ks
              if t0 <= int(k["Start_Timestamp"]) <= end_k]
        print(f"-- region {reg}: kernels end at {(end_k - t0) / 1e3:.1f} us, copies at {(end_c - t0) / 1e3:.1f} us, "
              f"GPU busy (any kernel) {union(iv) / 1e3:.1f} us")
        for p, b in launches:
            ps_, pe = int(p["Start_Timestamp"]) - t0, int(p["End_Timestamp"]) - t0
            line = f"   primary {ps_ / 1e3:8.1f} .. {pe / 1e3:8.1f}"
            if b:
                bs, be = int(b["Start_Timestamp"]) - t0, int(b["End_Timestamp"]) - t0
                line += f" | bounce {bs / 1e3:8.1f} .. {be / 1e3:8.1f} ({(be - bs) / 1e3:.1f} us)"
            print(line)
        for c in sorted(cs, key=lambda c: int(c["Start_Timestamp"]))[:3 * a.launches]:
            s, e = int(c["Start_Timestamp"]) - t0, int(c["End_Timestamp"]) - t0
            if s > end_c - t0:
                break
            print(f"   copy {s / 1e3:8.1f} .. {e / 1e3:8.1f} ({(e - s) / 1e3:.1f} us, {c.get('Bytes', '?')} B)")


if __name__ == "__main__":
    main()
