"""Per-parameter gradient error of one GPU TD update vs the fp64 oracle (diagnostic).
    python tools/diag_rt.py A B T [precision]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import ref_learner  # noqa: E402
from tests.gpu_util import normwise  # noqa: E402
from tests.test_gpu_generic import _args, _cfg_of  # noqa: E402


def main():
    A, B, T = map(int, sys.argv[1:4])
    prec = sys.argv[4] if len(sys.argv) > 4 else "fp32"
    force = os.environ.get("DIAG_GENERIC_KIND")  # "0" agent / "1" mixer: that network only runs generic
    if force is not None:
        from t2omca_amd import _lib, ops
        cache = {}

        def layout(s):
            if s not in cache:
                flags = _lib.LAYOUT_FORCE_GENERIC if s.kind == int(force) else 0
                cache[s] = _lib.make_layout(s.kind, s.E, s.H, s.D, s.F, s.NA, s.FF, s.n_ent, s.prec, s.n_agents,
                                            s.pos_func, s.pos_beta, flags=flags)
            return cache[s]
        ops._layout_cached = layout
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_batch
    cfg = _cfg_of(A)
    torch.manual_seed(0)
    args = _args(cfg)
    agent, mixer = TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()
    pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
    pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
    learner = TDLearner(agent, mixer, precision=prec)
    batch, w = make_batch(B, T, A, seed=int(os.environ.get("DIAG_SEED", "3")), obs_feats=9, state_feats=8)
    cpu = {k: (v.cpu().double() if v.is_floating_point() else v.cpu()) for k, v in batch.items()}
    pa_g = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
    pm_g = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
    import torch.nn.functional as Fn
    from oracle import ref_model
    relu, mins = Fn.relu, []

    def hook(x, *a, **k):  # |FFN pre-activation| of the kept token (agent: row 0)
        mins.append(float((x.detach()[:, 0] if x.dim() == 3 else x.detach()).abs().min()))
        return relu(x, *a, **k)
    ref_model.F.relu = hook
    loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, pa, pm, cpu, cfg, per_weight=w.cpu().double())
    ref_model.F.relu = relu
    print(f"   min |ReLU pre-activation| of kept rows: {min(mins):.2e}")
    loss.backward()
    learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    g = (learner.grad[:-1] / learner.grad[-1]).cpu().double()
    off = 0
    worst = []
    gmax = max(float(v.grad.abs().max()) for v in list(pa_g.values()) + list(pm_g.values()))
    for pre, d in (("agent.", pa_g), ("mixer.", pm_g)):
        for k, v in d.items():
            n = v.numel()
            err = float((g[off:off + n] - v.grad.reshape(-1)).abs().max()) / gmax
            worst.append((err, pre + k))
            off += n
    worst.sort(reverse=True)
    print(f"A={A} B={B} T={T} seed={os.environ.get('DIAG_SEED', '3')} {prec} instances agent={agent.shape.instance} mixer={mixer.shape.instance} "
          f"env={os.environ.get('T2O_MIXER_BWD', '')}/{os.environ.get('T2O_AGENT_BWD', '')} "
          f"generic kind {force}")
    for e, k in worst[:6]:
        print(f"   {e:.2e} {k}")


if __name__ == "__main__":
    main()
