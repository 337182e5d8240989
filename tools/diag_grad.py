"""Per-parameter normwise gradient error of the GPU TD update vs the fp64 oracle
(diagnostic; run on the GPU box)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_learner  # noqa: E402
from tests.gpu_util import normwise  # noqa: E402
from tests.test_gpu_configs import _cfg, _modules  # noqa: E402


def run(A, B, T, precision="fp32", seed=3):
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    agent, mixer = _modules(A)
    pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
    pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
    learner = TDLearner(agent, mixer, precision=precision)
    batch, w = make_batch(B, T, A, seed=seed)
    cpu = {k: (v.cpu().double() if v.is_floating_point() else v.cpu()) for k, v in batch.items()}
    pa_g = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
    pm_g = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
    loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, pa, pm, cpu, _cfg(A), per_weight=w.cpu().double())
    loss.backward()
    learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    g = (learner.grad[:-1] / learner.grad[-1]).cpu().double()
    ref = torch.cat([v.grad.reshape(-1) for v in list(pa_g.values()) + list(pm_g.values())])
    print(f"A={A} B={B} T={T} seed={seed} {precision} total normwise {normwise(g, ref):.3e}  max|ref| {ref.abs().max():.3e}")
    off = 0
    rows = []
    for net, p in (("agent", pa_g), ("mixer", pm_g)):
        for k, v in p.items():
            n = v.numel()
            gg, rr = g[off:off + n], ref[off:off + n]
            rows.append((float((gg - rr).abs().max()), net, k, float(rr.abs().max())))
            off += n
    for e, net, k, m in sorted(rows, reverse=True)[:8]:
        print(f"   {net:5s} {k:45s} max|err| {e:.3e}  max|ref| {m:.3e}  rel {e / max(m, 1e-30):.2e}")


if __name__ == "__main__":
    cases = [tuple(int(v) for v in c.split(",")) for c in sys.argv[1:]] or [(8, 16, 60), (16, 4, 150), (64, 2, 60)]
    for A, B, T in cases:
        run(A, B, T)
