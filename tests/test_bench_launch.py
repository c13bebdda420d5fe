"""bench.py's launcher on CPU: `python bench.py --gpus N --dry` starts N rank
processes itself (no torchrun), runs the shard geometry, the gloo gather and
the max-over-ranks timing with synthetic slabs, and rank 0 prints one JSON
line whose frame assembled correctly. No GPU, no measurement."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3])
def test_self_launch_dry(n):
    d = _run("--gpus", str(n), "--dry", "--steps", "2", "--warmup", "1")
    assert d["dry"] is True and d["value"] is None
    assert d["n_gpus"] == n
    assert d["frame_assembled_ok"] is True
    assert d["metric"].startswith("Mrays/s at 1080p")


def test_failing_rank_fails_the_launch():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry",
                        "--workload", "no-such-workload"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0


@pytest.mark.parametrize("hang,want_rc", [("1", None), ("all", 124)])
def test_stuck_rank_hits_the_deadline(hang, want_rc):
    """A rank that never joins must not hold the launch. MIRT_BENCH_DRY_HANG=1:
    rank 1 sleeps before init_process_group, so rank 0's rendezvous times out
    (the process group's timeout) and the parent ends the job. "all": no rank
    joins, nothing raises inside the ranks, and the parent's own deadline
    (--rank-timeout) terminates them: exit 124. Either way the parent exits
    non-zero within the deadline + 10 s."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MIRT_BENCH_DRY_HANG"] = hang
    deadline = 20.0
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry", "--steps", "2",
                        "--warmup", "1", "--rank-timeout", str(deadline)], capture_output=True, text=True,
                       timeout=120, env=env, cwd=ROOT)
    dt = time.monotonic() - t0
    assert p.returncode != 0 and dt < deadline + 10, (p.returncode, dt, p.stderr[-2000:])
    if want_rc is not None:
        assert p.returncode == want_rc and "deadline" in p.stderr and "[0, 1]" in p.stderr, p.stderr[-2000:]


@pytest.mark.gpu
def test_multi_rank_bench_rehearsal_on_one_gpu():
    """The N > 1 bench path on a one-GPU box (MIRT_BENCH_SHARE_GPU=1: both
    ranks on device 0, gloo in place of RCCL): the strong split with frames
    in flight, every frame's slabs gathered to rank 0, max-over-ranks timing
    -- runs to its JSON line (a rehearsal, no measurement)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MIRT_BENCH_SHARE_GPU"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "8", "--warmup",
                        "2", "--no-cpu", "--no-host"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert "REHEARSAL" in d["data"] and d["value_weak"] > 0 and d["value_strong"] == d["value"]


RCCL_ONE_RANK = r'''
import hashlib, importlib, json, os, sys
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
from importlib import import_module
shard = import_module("cs201_sah-bvh_ray_tracer_amd.shard")
g = json.load(open(os.path.join(sys.argv[1], "tests", "golden", "golden.json")))
want = g["frames"]["1920x1080_render10000_d5_m1_b1_s1_c0_step1"]["sha"]
s = m.create_random_spheres(10000, 1)
b = m.build_bvh(s)
rs = [m.Renderer(0) for _ in range(4)]
for r in rs:
    r.upload(s, b)
sf = shard.ShardedFrame(rs[0], 1920, 1080, renderers=rs)
cam = m.default_camera()
ok = []
for k in range(6):
    sf.render_local(cam, sf.desc(seed=1))
    f = sf.gather()
    torch.cuda.synchronize()
    ok.append(hashlib.sha256(shard.as_rgba(f).cpu().numpy().tobytes()).hexdigest() == want)
dist.destroy_process_group()
print(json.dumps({"backend": "nccl", "frames_ok": ok}))
sys.exit(0 if all(ok) else 3)
'''


@pytest.mark.gpu
def test_rccl_gather_one_rank():
    """The RCCL leg of the N > 1 path on the one-GPU box: a world-1 nccl
    process group, four contexts rotating frames on their own streams, each
    frame's slab gathered by dist.gather (RCCL) under its context's stream,
    every gathered frame equal to the golden 1080p frame. (Two ranks cannot
    share one device under RCCL; the multi-rank geometry is the gloo
    rehearsal above and tests/test_shard_gloo.py.)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29731", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "-c", RCCL_ONE_RANK, ROOT], capture_output=True, text=True, timeout=240,
                       env=env, cwd=ROOT)
    assert p.returncode == 0, (p.stdout[-1000:], p.stderr[-3000:])
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["frames_ok"] == [True] * 6
