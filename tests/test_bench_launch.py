"""bench.py's multi-process launcher and host gather on CPU with gloo.

`python bench.py --gpus N` started without WORLD_SIZE must launch N ranks itself (a
torch.distributed.run child, before anything touches a GPU), take the MAX over ranks and
print ONE JSON line from rank 0; `--global-batch` splits the images over the ranks and
`--gather` assembles every rank's output slice in one shared host buffer. The `selftest`
workload is a CPU stand-in per-image function, so the whole path runs here.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "selftest",
                        "--no-cpu-baseline", *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_single_process_line():
    rec = _bench("--steps", "2", "--warmup", "1", "--size", "8")
    assert rec["n_gpus"] == 1 and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 4 and rec["steps"] == 2
    assert rec["value"] > 0 and len(rec["per_rank_s"]) == 1


@pytest.mark.parametrize("gpus,gbatch,micro", [(2, 7, None), (3, 6, None), (2, 9, 2)])
def test_launcher_strong_split_with_host_gather(gpus, gbatch, micro):
    extra = ("--micro-batch", str(micro)) if micro else ()
    rec = _bench("--gpus", str(gpus), "--global-batch", str(gbatch), "--gather",
                 "--steps", "2", "--warmup", "1", "--size", "8", *extra)
    assert rec["config"]["micro_batch"] == (micro or (gbatch + gpus - 1) // gpus)
    assert rec["n_gpus"] == gpus and rec["scaling"] == "strong"
    assert rec["config"]["global_batch"] == gbatch
    assert len(rec["per_rank_s"]) == gpus and all(t > 0 for t in rec["per_rank_s"])
    # value = all images of all ranks / the slowest rank's time
    assert abs(rec["value"] - gbatch * 2 / (rec["ms_per_step"] * 2e-3)) / rec["value"] < 1e-2
    assert rec["host_gather"]["all_finite"] is True  # bit-exact vs the unsplit batch


def test_launcher_weak_scaling():
    rec = _bench("--gpus", "2", "--batch", "3", "--steps", "1", "--warmup", "0", "--size", "8")
    assert rec["n_gpus"] == 2 and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 6 and rec["config"]["per_gpu_batch"] == 3


def test_inference_creates_no_rccl_group():
    """north_star: the inference path has no collective; only training's gradient
    all-reduce may use RCCL (bench.py process_group_backend)."""
    sys.path.insert(0, ROOT)
    import bench
    for kind in ("adain", "wct", "sanet", "multiscale", "source", "adaptive", "selftest"):
        assert bench.process_group_backend(kind, cuda=True) == "gloo", kind
    for kind in bench.TRAIN_KINDS:
        assert bench.process_group_backend(kind, cuda=True) == "nccl", kind
    rec = _bench("--gpus", "2", "--batch", "2", "--steps", "1", "--warmup", "0", "--size", "8")
    assert rec["config"]["process_group"] == "gloo"


def test_cpu_share_follows_omp_num_threads(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.cpu_share()[0] == 16
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_share()[0] == len(os.sched_getaffinity(0))


def test_world_size_mismatch_rejected():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "selftest",
                        "--gpus", "2"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
