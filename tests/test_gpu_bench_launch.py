"""GPU: the path the driver's SCALE run takes — `python bench.py --gpus N` started
as a plain process launches its N ranks itself (torch.distributed.run on 127.0.0.1,
bench.launch) and rank 0 prints one JSON line with the whole-job value.  Here N = 2
on the one-GPU box, the ranks sharing cuda:0 over gloo (T2O_DIST_BACKEND=gloo:
RCCL keeps one rank per GPU), on a tiny TD update; a fresh child process, so the
launcher's "nothing touched the GPU before the ranks start" rule holds."""
import json
import os
import subprocess
import sys

import pytest

from tests.gpu_util import require_gpu

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_launches_two_ranks():
    require_gpu()
    env = dict(os.environ, T2O_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "16", "--T", "6", "--no-cpu-baseline", "--no-fp32-companion", "--kernel-timer-every", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 32
    assert d["value"] > 0 and d["steps"] == 2 and d["warmup"] == 1
    # what the process group itself saw (a SCALE line shows RCCL's rank count the same way)
    di = d["distributed"]
    assert di["world_size"] == 2 and di["backend"] == "gloo" and di["env_world_size"] == 2, di
    rm = di["rank_ms_per_step"]
    assert len(rm["per_rank"]) == 2 and rm["min"] <= rm["max"] and abs(rm["max"] - d["ms_per_step"]) < 1e-6 * rm["max"] + 1e-9
    print("bench --gpus 2 (gloo, one device):", {k: d[k] for k in ("value", "ms_per_step", "n_gpus")})
