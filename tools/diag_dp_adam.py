"""Diagnostic (not a test): the DP learner scenario of tests/test_gpu_dp_learner.py, printing
per update the normwise distance of the all-reduced gradient to the full-batch gradient and,
at the parameters whose post-Adam values differ most, both gradients and Adam's second moment.
Run on the GPU box:  python tools/diag_dp_adam.py   (T2O_LIB selects the library build)."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_dp_learner import B, UPDATES, _batch, _learner  # noqa: E402


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from t2omca_amd.distributed import shard_bounds
        learner = _learner(100 + rank, dev)
        batch, w = _batch(dev)
        lo, hi = shard_bounds(B, rank, world)
        shard = {k: v[lo:hi] for k, v in batch.items()}
        ps, gs = [learner.params.detach().cpu().clone()], []
        for u in range(UPDATES):
            learner.train(shard, 0, u, per_weight=w[lo:hi])
            torch.cuda.synchronize()
            ps.append(learner.params.detach().cpu().clone())
            gs.append(learner.grad[:-1].detach().cpu().clone())
        out.put((rank, torch.stack(ps), torch.stack(gs)))
    finally:
        dist.destroy_process_group()


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ps, gs = q.get(timeout=240)
        res[r] = (ps, gs)
    for p in procs:
        p.join(timeout=60)
    ps, gs = res[0]
    dev = torch.device("cuda", 0)
    full = _learner(100, dev)
    batch, w = _batch(dev)
    for u in range(UPDATES):
        full.train(batch, 0, u, per_weight=w)
        torch.cuda.synchronize()
        fp, fg = full.params.cpu(), full.grad[:-1].cpu()
        gerr = float((gs[u] - fg).abs().max() / fg.abs().max())
        d = (ps[u + 1] - fp).abs()
        perr = float((ps[u + 1] - fp).abs().max() / fp.abs().max())
        print(f"update {u}: grad normwise {gerr:.2e}, params normwise {perr:.2e}")
        top = torch.topk(d, 5).indices
        v = full.exp_avg_sq.cpu()
        for i in top.tolist():
            print(f"   param {i}: |dp| {float(d[i]):.3e} grad dp {float(gs[u][i]):+.3e} full {float(fg[i]):+.3e} "
                  f"v {float(v[i]):.3e}")


if __name__ == "__main__":
    main()
