"""bench.py's launcher on CPU. At N > 1 the parent (or torchrun's rank 0)
never touches a GPU: it starts ONE fresh measuring process over all N GPUs
(include/mirt_multi.h from one host thread) under a deadline; `--dry` makes
that child a plumbing check (shard geometry + both deliveries' index math
over synthetic slabs). Other torchrun ranks join rank 0 at a gloo barrier.
No GPU, no measurement here; the GPU test at the end runs the real N = 2
launcher on one GPU's worth of the path (same-device ranks are refused by
RCCL, so it runs N = 1 through the child)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLEAN = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "LOCAL_WORLD_SIZE")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in CLEAN}
    env.update(kw)
    return env


def _lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _run(*args, env=None, timeout=240):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env or _env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _lines(p.stdout)
    assert len(lines) == 1, p.stdout
    return lines[0]


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_self_launch_dry(n):
    d = _run("--gpus", str(n), "--dry", "--steps", "2", "--warmup", "1")
    assert d["dry"] is True and d["value"] is None
    assert d["n_gpus"] == n
    assert d["frame_assembled_ok"] is True
    assert d["metric"].startswith("Mrays/s at 1080p")
    assert d["config"]["frames_per_launch"] == {1: 1, 2: 1, 3: 4, 8: 4}[n]


def test_bad_arguments_fail_the_launch():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry",
                        "--workload", "no-such-workload"], capture_output=True, text=True, timeout=120, env=_env())
    assert p.returncode != 0


def test_stuck_child_hits_the_deadline():
    """A measuring process that never finishes (a rank stuck in RCCL init or
    a gather) must not hold the job: the parent terminates it at
    --rank-timeout and exits 124, naming the deadline."""
    deadline = 15.0
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry", "--steps", "2",
                        "--warmup", "1", "--rank-timeout", str(deadline)], capture_output=True, text=True,
                       timeout=120, env=_env(MIRT_BENCH_DRY_HANG="1"), cwd=ROOT)
    dt = time.monotonic() - t0
    assert p.returncode == 124 and deadline <= dt < deadline + 10, (p.returncode, dt, p.stderr[-2000:])
    assert "deadline" in p.stderr


def test_stuck_secondary_leg_keeps_the_headline():
    """A measuring process stuck AFTER its headline (in the other delivery's
    n-GPU RCCL leg) costs that leg only: at --rank-timeout the parent prints
    the line the child saved before the leg, the leg marked unfinished, the
    child's exit status in the line, and exits 0 with exactly one line."""
    deadline = 15.0
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry", "--steps", "2",
                        "--warmup", "1", "--rank-timeout", str(deadline)], capture_output=True, text=True,
                       timeout=120, env=_env(MIRT_BENCH_DRY_HANG="after-headline"), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["frame_assembled_ok"] is True and d["measuring_process_exit"] == 124
    assert d["other_delivery"]["delivery"] == "gather" and "not finished" in d["other_delivery"]["error"]


def test_finished_child_leaves_no_saved_line(tmp_path):
    """A child that finishes prints its own line and removes the saved one."""
    path = str(tmp_path / "partial.json")
    with open(path, "w") as f:
        f.write("{}")         # as if saved before a secondary leg
    d = _run("--gpus", "2", "--dry", "--steps", "2", "--warmup", "1", "--measure-child",
             env=_env(MIRT_BENCH_PARTIAL=path))
    assert "measuring_process_exit" not in d and not os.path.exists(path)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_torchrun_world_dry(world):
    """The driver's N > 1 command (torch.distributed.run, one process per
    GPU): rank 0 measures in its child, the other ranks meet it at the gloo
    barrier, exactly one JSON line, exit 0."""
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dry", "--steps", "2", "--warmup",
                        "1"], capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _lines(p.stdout)
    assert len(lines) == 1 and lines[0]["n_gpus"] == world and lines[0]["frame_assembled_ok"], p.stdout


def test_torchrun_rank0_failure_fails_every_rank():
    """A failing measuring child on rank 0 fails the whole job (its status is
    broadcast at the barrier), not only rank 0."""
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry", "--steps", "2", "--warmup", "1",
                        "--rank-timeout", "10"], capture_output=True, text=True, timeout=300,
                       env=_env(MIRT_BENCH_DRY_HANG="1"), cwd=ROOT)
    assert p.returncode != 0


@pytest.mark.gpu
def test_bench_line_one_gpu_short():
    """The driver's N = 1 command, short: the headline through mirt_multi
    (RCCL, frames into page-locked host memory), its last frame equal to one
    context's, the device-resident and depth-1 legs beside it."""
    d = _run("--steps", "8", "--warmup", "2", "--no-cpu", "--no-host", timeout=400)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["device_resident_mrays_s"] > 0
    assert d["last_frame_equals_one_context"] is True
    assert d["config"]["delivery"] == "gather" and d["depth1_mrays_s"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_line_two_ranks_same_device_rehearsal():
    """The N > 1 flow on one GPU (--same-device: the copy exchange in place of
    RCCL): the measuring child, the host-direct headline, the gather leg
    beside it and the one-lane check, every checked frame equal to one
    context's; the line is marked as a rehearsal."""
    d = _run("--gpus", "2", "--same-device", "--steps", "8", "--warmup", "2", "--no-cpu", "--no-host", timeout=400)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["rehearsal_same_device"]
    assert d["config"]["delivery"] == "host-direct" and d["last_frame_equals_one_context"] is True
    o = d["other_delivery"]
    assert o["delivery"] == "gather" and "error" not in o, o
    assert o["last_frame_equals_one_context"] is True and o["one_lane_frame_equals_one_context"] is True
    assert d["reference_work"]["bytes_per_frame"] > 0 and d["reference_work"]["frac_of_g_hbm_peak"] > 0
