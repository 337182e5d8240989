"""Diagnostic: the DP-vs-full-batch learner comparison of tests/test_gpu_dp_learner.py,
printing per-parameter errors after every update (which tensors drift, by how much)."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_dp_learner import UPDATES, _batch, _learner, _worker  # noqa: E402


def names(learner):
    out = []
    for mod in (learner.agent, learner.mixer):
        for n, p in mod.named_parameters():
            out.append((n, p.numel()))
    return out


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    r0 = torch.from_numpy(res[0])
    dev = torch.device("cuda", 0)
    full = _learner(100, dev)
    batch, w = _batch(dev)
    nm = names(full)
    for u in range(UPDATES):
        g_before = None
        full.train(batch, 0, u, per_weight=w)
        torch.cuda.synchronize()
        a, b = r0[u + 1], full.params.cpu()
        d = (a - b).abs()
        o, rows = 0, []
        for n, k in nm:
            rows.append((float(d[o:o + k].max()), n, float(b[o:o + k].abs().max())))
            o += k
        rows.sort(reverse=True)
        print(f"update {u}: normwise {float((a - b).norm() / b.norm()):.3e}; worst:",
              "; ".join(f"{n} {e:.2e} (|p|max {m:.2e})" for e, n, m in rows[:5]), flush=True)


if __name__ == "__main__":
    main()
