"""Probe (GPU box): config-3 TD update timed eager vs replayed from one hipGraph.

The graph bakes in the Adam step count, so it is a timing experiment only:
  python tools/graph_probe.py [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from t2omca_amd.learner import TDLearner  # noqa: E402
from t2omca_amd.modules import TransformerAgent, TransformerMixer  # noqa: E402
from t2omca_amd.synthetic import make_args, make_batch  # noqa: E402


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--A", type=int, default=8)
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--T", type=int, default=60)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    margs = make_args(a.A, device=str(dev))
    agent, mixer = TransformerAgent(None, margs).to(dev), TransformerMixer(margs).to(dev)
    learner = TDLearner(agent, mixer, target_update_interval=10 ** 9, precision="bf16", priorities_to_cpu=False)
    batch, w = make_batch(a.B, a.T, a.A, seed=1, device=dev)
    for i in range(3):
        learner.train(batch, 0, i, per_weight=w)
    eager = timed(lambda i: learner.train(batch, 0, i, per_weight=w), a.steps)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        learner.train(batch, 0, 0, per_weight=w)
    g.replay()
    torch.cuda.synchronize()
    graph = timed(lambda i: g.replay(), a.steps)
    eager2 = timed(lambda i: learner.train(batch, 0, i, per_weight=w), a.steps)
    print(json.dumps({"eager_ms": eager, "graph_ms": graph, "eager_again_ms": eager2}), flush=True)


if __name__ == "__main__":
    main()
