"""GPU: the RCCL (backend "nccl") path bench.py and the learner take under data
parallelism, on the one GPU this box has: a 1-rank process group initialised as
bench.py does (init_process_group("nccl", device_id=...)), the learner's two
all-reduce halves issued the way TDLearner.train issues them (the mixer half from
a side stream, async; the agent half from the main stream; both waited on by the
main stream), a barrier and a broadcast.  More ranks need more GPUs (RCCL keeps one
rank per device); the multi-rank arithmetic is covered by test_gpu_dp_learner.py
(gloo, 2 ranks on one GPU) and test_distributed.py."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from tests.gpu_util import require_gpu

pytestmark = pytest.mark.gpu


def _worker(port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    try:
        from t2omca_amd.distributed import wait_all
        grad = torch.arange(1000, dtype=torch.float32, device=dev)
        main = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            grad[600:].mul_(2.0)
            w_m = dist.all_reduce(grad[600:], op=dist.ReduceOp.SUM, async_op=True)
        grad[:600].add_(1.0)
        w_a = dist.all_reduce(grad[:600], op=dist.ReduceOp.SUM, async_op=True)
        main.wait_stream(side)
        wait_all((w_m, w_a))
        res = grad * 1.0  # consumed on the main stream after the waits
        p = torch.full((7,), 3.0, device=dev)
        dist.broadcast(p, 0)
        dist.barrier()
        torch.cuda.synchronize()
        out.put((dist.get_backend(), res.cpu(), p.cpu()))
    finally:
        dist.destroy_process_group()


def test_rccl_process_group_and_split_allreduce():
    require_gpu()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_worker, args=(port, q))
    proc.start()
    try:
        backend, res, p = q.get(timeout=100)
    finally:
        proc.join(timeout=60)
    assert proc.exitcode == 0
    assert backend == "nccl"
    ref = torch.arange(1000, dtype=torch.float32)
    ref[600:] *= 2.0
    ref[:600] += 1.0
    assert torch.equal(res, ref)
    assert torch.equal(p, torch.full((7,), 3.0))
