"""GPU: one full TD update (fwd + bwd + Adam) vs the CPU oracle learner; drop-in modules."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_learner, ref_model
from tests.gpu_util import flat_from_npz, normwise, require_gpu, tuned_fixtures
from tests.test_oracle_golden import _cfg

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cfg_dict(A):
    return dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
                n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)


def _setup(A, seed=0):
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args
    torch.manual_seed(seed)
    args = make_args(A)
    agent = TransformerAgent(None, args).cuda()
    mixer = TransformerMixer(args).cuda()
    pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
    pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
    return agent, mixer, pa, pm


@pytest.mark.parametrize("A,B,T,lam", [(8, 6, 5, 0.6), (3, 5, 4, 0.0), (16, 3, 4, 0.6), (64, 2, 3, 0.6)])
def test_td_update_matches_oracle(A, B, T, lam):
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    agent, mixer, pa, pm = _setup(A)
    learner = TDLearner(agent, mixer, td_lambda=lam)
    batch, w = make_batch(B, T, A, seed=3)
    # make the target networks differ from the online ones
    learner.target_params.add_(0.01 * torch.randn_like(learner.target_params))
    learner._pack_targets()
    cfg = _cfg_dict(A)
    cpu = {k: v.cpu() for k, v in batch.items()}
    cpu_d = {k: (v.double() if v.is_floating_point() else v) for k, v in cpu.items()}
    tgt = learner.target_params.cpu().double()
    pat, pmt, off = {}, {}, 0
    for src, dst in ((pa, pat), (pm, pmt)):
        for k, v in src.items():
            dst[k] = tgt[off:off + v.numel()].view_as(v)
            off += v.numel()
    pa_g = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
    pm_g = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
    loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, pat, pmt, cpu_d, cfg, td_lambda=lam,
                                            per_weight=w.cpu().double())
    loss.backward()
    info = learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    assert normwise(info["qtot"], ex["qtot"]) < 1e-5
    assert normwise(info["targets"], ex["targets"]) < 1e-5
    assert normwise(info["td_errors_abs"], prio) < 1e-5
    msum = float(info["mask_sum"])
    assert abs(float(info["loss_sum"]) / msum - float(loss)) < 1e-5 * max(1.0, abs(float(loss)))
    g = (learner.grad[:-1] / learner.grad[-1]).cpu()
    ref_g = torch.cat([v.grad.reshape(-1) for v in list(pa_g.values()) + list(pm_g.values())])
    assert normwise(g, ref_g) < 3e-5
    # the parameter update equals clip_grad_norm_(10) + Adam applied to those grads
    p0 = torch.cat([v.reshape(-1) for v in list(pa.values()) + list(pm.values())]).float()
    ref_p = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref_p], lr=1e-3)
    ref_p.grad = g.clone()
    torch.nn.utils.clip_grad_norm_([ref_p], 10.0)
    opt.step()
    assert (learner.params.cpu() - ref_p.detach()).abs().max() < 1e-6


@pytest.mark.parametrize("path", tuned_fixtures("agent", ("a8_e32_h3_d2",)))
def test_dropin_agent_module_step_and_autograd(path):
    """TransformerAgent.forward (reference signature) per step + autograd through it."""
    require_gpu()
    from t2omca_amd.modules import TransformerAgent
    from t2omca_amd.synthetic import make_args
    z = np.load(path)
    p, cfg = _cfg(z, "agent")
    agent = TransformerAgent(None, make_args(cfg["n_agents"])).cuda()
    agent.load_state_dict({k: v.float() for k, v in p.items()})
    obs = torch.from_numpy(z["obs"]).float().cuda()
    h = torch.from_numpy(z["h0"]).float().cuda().requires_grad_(True)
    hh, qs, hs = h, [], []
    for t in range(obs.shape[1]):
        q, hh = agent.forward(obs[:, t].contiguous(), hh)
        qs.append(q)
        hs.append(hh)
    qs, hs = torch.stack(qs, 1), torch.stack(hs, 1)
    assert normwise(qs, z["q_f64"]) < 1e-5 and normwise(hs, z["h_f64"]) < 1e-5
    loss = (qs * torch.from_numpy(z["cq"]).float().cuda()).sum() + \
        (hs * torch.from_numpy(z["ch"]).float().cuda()).sum()
    loss.backward()
    for k, prm in agent.named_parameters():
        assert normwise(prm.grad, z["grad/" + k]) < 3e-5, k
    assert normwise(h.grad, z["grad_h0"]) < 3e-5


@pytest.mark.parametrize("path", tuned_fixtures("mixer", ("a8_e32_h3_d2",)))
def test_dropin_mixer_module_step_and_autograd(path):
    require_gpu()
    from t2omca_amd.modules import TransformerMixer
    from t2omca_amd.synthetic import make_args
    z = np.load(path)
    p, cfg = _cfg(z, "mixer")
    mixer = TransformerMixer(make_args(cfg["n_agents"])).cuda()
    mixer.load_state_dict({k: v.float() for k, v in p.items()})
    f = lambda k: torch.from_numpy(z[k]).float().cuda()  # noqa: E731
    qv, hid, st = f("qvals").requires_grad_(True), f("hidden").requires_grad_(True), f("states")
    hw = f("hw0").requires_grad_(True)
    cur, ys, hws = hw, [], []
    for t in range(qv.shape[1]):
        y, cur = mixer.forward(qv[:, t:t + 1], hid[:, t], cur, st[:, t], None)
        ys.append(y.view(-1))
        hws.append(cur)
    ys, hws = torch.stack(ys, 1), torch.stack(hws, 1)
    assert normwise(ys, z["y_f64"]) < 1e-5 and normwise(hws, z["hw_f64"]) < 1e-5
    loss = (ys * f("cy")).sum() + (hws * f("chw")).sum()
    loss.backward()
    for k, prm in mixer.named_parameters():
        assert normwise(prm.grad, z["grad/" + k]) < 3e-5, k
    assert normwise(qv.grad, z["grad_qvals"]) < 3e-5
    assert normwise(hid.grad, z["grad_hidden"]) < 3e-5
    assert normwise(hw.grad, z["grad_hw0"]) < 3e-5
