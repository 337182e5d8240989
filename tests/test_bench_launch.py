"""CPU: bench.py's multi-GPU launcher.  `python bench.py --gpus N` (the driver's
SCALE invocation) must start N ranks itself when no launcher set WORLD_SIZE, and
run as one rank when torch.distributed.run did."""
import importlib.util
import os
import subprocess
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_needs_launch_only_without_a_launcher():
    b = _bench()
    a = types.SimpleNamespace(gpus=8)
    assert b.needs_launch(a, {})
    assert not b.needs_launch(a, {"WORLD_SIZE": "8"})
    assert not b.needs_launch(types.SimpleNamespace(gpus=1), {})


def test_launcher_cmd_is_one_process_per_gpu_on_loopback():
    b = _bench()
    cmd = b.launcher_cmd(["--gpus", "4", "--steps", "5"], 4, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))


def test_launcher_cmd_starts_n_ranks_with_rank_env(tmp_path):
    """The same torch.distributed.run command line, pointed at a probe script,
    really starts N processes with RANK / LOCAL_RANK / WORLD_SIZE set."""
    b = _bench()
    probe = tmp_path / "probe.py"
    probe.write_text("import os, sys\n"
                     "open(os.path.join(sys.argv[1], 'r' + os.environ['RANK']), 'w').write(\n"
                     "    os.environ['LOCAL_RANK'] + ' ' + os.environ['WORLD_SIZE'])\n")
    cmd = b.launcher_cmd([str(tmp_path)], 2, b.free_port())
    cmd[-2] = str(probe)
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sorted(p.name for p in tmp_path.iterdir() if p.name.startswith("r")) == ["r0", "r1"]
    assert (tmp_path / "r1").read_text() == "1 2"
