"""Run-to-run determinism probe: the same TD update from the same
state, N times in one process, each result compared with the first.

    T2O_LIB=t2omca_amd/lib/pf.so python tools/diag_repro.py --repeats 12 8,64,12,bf16 16,4,6,bf16

Prints, per configuration, how many runs differ from the first and where (agent /
mixer parameter range of the differing gradient elements).  T2O_POISON=1 fills
every fresh float device tensor with NaN first (as tests/conftest.py does)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("T2O_POISON") == "1":
    from tests.conftest import _poison_empty
    _poison_empty()


def one(A, B, T, precision, seed=5):
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args, make_batch
    torch.manual_seed(seed)
    args = make_args(A, device="cuda")
    agent, mixer = TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()
    learner = TDLearner(agent, mixer, precision=precision, priorities_to_cpu=False)
    batch, w = make_batch(B, T, A, seed=11)
    info = learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    return learner.grad.clone(), info["td_errors_abs"].clone(), learner.na


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=8)
    ap.add_argument("configs", nargs="+", help="A,B,T,precision")
    a = ap.parse_args()
    print("library:", os.environ.get("T2O_LIB", "default"), "poison:", os.environ.get("T2O_POISON", "0"))
    bad = 0
    for cfg in a.configs:
        A, B, T, prec = cfg.split(",")
        A, B, T = int(A), int(B), int(T)
        g0, p0, na = one(A, B, T, prec)
        nan0 = int((~torch.isfinite(g0)).sum())
        ndiff_runs, where = 0, []
        for _ in range(a.repeats - 1):
            g, p, _ = one(A, B, T, prec)
            d = torch.nonzero(g != g0).flatten().cpu()
            if d.numel() or not torch.equal(p, p0):
                ndiff_runs += 1
                if d.numel():
                    where.append((d.numel(), int(d.min()), int(d.max()), float((g - g0).abs().max())))
        bad += ndiff_runs + (nan0 > 0)
        print(f"A={A} B={B} T={T} {prec}: non-finite grads {nan0}; {ndiff_runs} of {a.repeats - 1} runs differ "
              f"from the first (agent params < {na}); (count, min idx, max idx, max|diff|): {where[:6]}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
