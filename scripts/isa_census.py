"""Static ISA census of one kernel: its instructions by class (VALU, SALU,
VMEM, LDS, SMEM, branch/wait) attributed to the innermost source function
they were inlined from (the .loc line tables of a -gline-tables-only build,
which does not change code generation).

    hipcc -O3 -std=c++17 -ffp-contract=off -gline-tables-only --offload-arch=gfx950 \
          --cuda-device-only -S -o /tmp/render-g.s cs201_sah-bvh_ray_tracer_amd/csrc/render.hip
    python scripts/isa_census.py /tmp/render-g.s 'bounce_kernelILb1ELi2ELb0E' [--json out.json]

Static counts say what one pass over each function's code costs; the
dynamic mix is these weighted by how often each function runs per node
visit (the instrumented build's counters).
"""
import argparse
import collections
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cs201_sah-bvh_ray_tracer_amd", "csrc")

FN_START = re.compile(r"^(?:template\s*<.*>\s*)?(?:__device__|__global__|inline|static|struct|auto|bool|int|float|void|"
                      r"uint32_t|uint64_t|Ray|Prune|SlabRay|SphRay|WideWalk|NodeV|PNodeV|float4|uint4)\b.*?\b(\w+)\s*\(")


def function_map(path):
    """line -> name of the function (or struct) whose definition the line lies in."""
    names, cur = {}, "?"
    with open(path) as f:
        for i, line in enumerate(f, 1):
            m = FN_START.match(line)
            if m and not line.rstrip().endswith(";"):
                cur = m.group(1)
            names[i] = cur
    return names


def classify(op):
    if op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_setpc", "s_endpgm", "s_barrier", "s_nop",
                      "s_sleep", "s_getpc")):
        return "branch_wait"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_rd"
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "global_atomic", "flat_atomic",
                      "buffer_atomic")):
        return "vmem_wr"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the kernel's mangled name")
    ap.add_argument("--json", default="")
    ap.add_argument("--loop", default="", help="only the blocks of this loop (e.g. BB18_26: the llc 'in Loop: Header=' tag)")
    ap.add_argument("--depth", type=int, default=0, help="with --loop: only blocks at exactly this loop depth")
    a = ap.parse_args()
    files, fmaps = {}, {}
    counts = collections.defaultdict(collections.Counter)
    inside, loc, cur_loop = False, None, None
    with open(a.asm) as f:
        for line in f:
            s = line.strip()
            if s.startswith(".file"):
                m = re.match(r'\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', s)
                if m:
                    files[int(m.group(1))] = m.group(3)
                continue
            if not inside:
                if re.match(r"^_Z\S*" + re.escape(a.kernel) + r"\S*:", line):
                    inside = True
                continue
            if s.startswith(".Lfunc_end"):
                break
            if s.startswith(".loc"):
                p = s.split()
                loc = (int(p[1]), int(p[2]))
                continue
            if not line.startswith("\t") and (s.endswith(":") or "; %bb" in s or s.startswith(".LBB")):
                m = re.search(r"in Loop: Header=(\S+) Depth=(\d+)", line)
                cur_loop = (m.group(1), int(m.group(2))) if m else None
                continue
            if a.loop and not (cur_loop and cur_loop[0] == a.loop and (not a.depth or cur_loop[1] == a.depth)):
                continue
            if not s or s.startswith((";", ".", "_")) or s.endswith(":"):
                continue
            op = s.split()[0]
            fn = "?"
            if loc:
                fname = files.get(loc[0], "?")
                if fname not in fmaps and os.path.exists(os.path.join(CSRC, fname)):
                    fmaps[fname] = function_map(os.path.join(CSRC, fname))
                fn = fmaps.get(fname, {}).get(loc[1], os.path.basename(fname)) if fname in fmaps else os.path.basename(fname)
            counts[fn][classify(op)] += 1
    classes = ["valu", "salu", "vmem_rd", "vmem_wr", "lds", "smem", "branch_wait", "other"]
    total = collections.Counter()
    rows = sorted(counts.items(), key=lambda kv: -kv[1]["valu"])
    print(f"{'function':32s} " + " ".join(f"{c:>8s}" for c in classes))
    for fn, c in rows:
        total.update(c)
        print(f"{fn:32s} " + " ".join(f"{c[k]:8d}" for k in classes))
    print(f"{'TOTAL':32s} " + " ".join(f"{total[k]:8d}" for k in classes))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"kernel": a.kernel, "by_function": {k: dict(v) for k, v in counts.items()},
                       "total": dict(total)}, f, indent=1)


if __name__ == "__main__":
    main()
