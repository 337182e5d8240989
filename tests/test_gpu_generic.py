"""GPU: the runtime-shaped kernels (t2o_generic.hip; t2o_layout.generic = 1) against
the reference modules' own goldens and the fp64 oracle, for every shape / option
the tuned MFMA instances do not cover (tests/golden/make_golden.py EXTENDED):

  * 5 and 32 AGVs, emb 64 with 4 heads, emb 16 / 1 head / depth 3 / ff_hidden_mult 2,
    n_entities_obs != n_agents (agent), n_entities_state != n_agents (mixer);
  * every qmix_pos_func (softplus with beta, quadratic, identity) and the
    state_entity_mode=False obs branch of the mixer (n_transf_mixer.py:60-63,95-103);
  * the drop-in modules' per-step forward + autograd (reference signatures),
    the full TD update vs oracle/ref_learner, and T2O_GENERIC=1 (the generic path
    forced on the tuned headline shape) against the tuned kernels.

The default network (emb 32, 3 heads, depth 2) at 5 / 32 AGVs now has runtime-entity
MFMA instances (tests/test_gpu_runtime_shapes.py covers them); here those shapes run
with T2O_GENERIC=1 so the runtime-shaped kernels stay pinned at them too.

Bars (normwise): forward <= 1e-5, gradients <= 3e-5 (fp32; the
generic kernels compute in fp32 whatever precision is asked).
"""
import glob
import os
import types

import numpy as np
import pytest
import torch

from tests.gpu_util import normwise, oracle_td_tie_aware, require_gpu
from tests.test_oracle_golden import _cfg

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
EXT = ("a5_", "a32_", "a8_e64", "a6_e16", "a4_ne6", "a4_ns6", "a8_softplus", "a8_quadratic", "a8_identity",
       "a3_obsbranch")


def _ext(kind):
    return sorted(p for p in glob.glob(os.path.join(GOLD, f"{kind}_*.npz"))
                  if os.path.basename(p)[len(kind) + 1:].startswith(EXT))


def _args(cfg, device="cuda"):
    a = types.SimpleNamespace(
        n_agents=cfg["n_agents"], n_entities=cfg["n_entities"], obs_entity_feats=9, emb=cfg["emb"],
        heads=cfg["heads"], depth=cfg["depth"], ff_hidden_mult=cfg["ff_hidden_mult"], dropout=0.0,
        action_selector="epsilon_greedy", n_actions=5, device=device,
        state_entity_feats=cfg["state_entity_feats"], mixer_emb=cfg["mixer_emb"], mixer_heads=cfg["mixer_heads"],
        mixer_depth=cfg["mixer_depth"], env_args={"state_entity_mode": bool(cfg.get("state_entity_mode", True))})
    for k in ("n_entities_obs", "n_entities_state", "qmix_pos_func", "qmix_pos_func_beta"):
        if k in cfg:
            setattr(a, k, cfg[k])
    return a


@pytest.fixture(autouse=True)
def _generic_everywhere(monkeypatch):
    """Shapes that have a tuned (exact or runtime-entity) MFMA instance run generic here."""
    monkeypatch.setenv("T2O_GENERIC", "1")


@pytest.mark.parametrize("path", _ext("agent"), ids=os.path.basename)
def test_generic_agent_module_step_and_autograd(path):
    require_gpu()
    assert agent_module_check(path) == "generic"


def agent_module_check(path):
    """The drop-in agent's per-step forward + autograd vs a reference golden; returns
    which kernels ran (NetShape.instance)."""
    from t2omca_amd.modules import TransformerAgent
    z = np.load(path)
    p, cfg = _cfg(z, "agent")
    agent = TransformerAgent(None, _args(cfg)).cuda()
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
    return agent.shape.instance


@pytest.mark.parametrize("path", _ext("mixer"), ids=os.path.basename)
def test_generic_mixer_module_step_and_autograd(path):
    require_gpu()
    assert mixer_module_check(path) == "generic"


def mixer_module_check(path):
    """The drop-in mixer's per-step forward + autograd vs a reference golden; returns
    which kernels ran (NetShape.instance)."""
    from t2omca_amd.modules import TransformerMixer
    z = np.load(path)
    p, cfg = _cfg(z, "mixer")
    mixer = TransformerMixer(_args(cfg)).cuda()
    mixer.load_state_dict({k: v.float() for k, v in p.items()})
    f = lambda k: torch.from_numpy(z[k]).float().cuda()  # noqa: E731
    qv, hid, st = f("qvals").requires_grad_(True), f("hidden").requires_grad_(True), f("states")
    hw = f("hw0").requires_grad_(True)
    obs_branch = not mixer.custom_space
    cur, ys, hws = hw, [], []
    for t in range(qv.shape[1]):
        if obs_branch:
            y, cur = mixer.forward(qv[:, t:t + 1], hid[:, t], cur, None, st[:, t])
        else:
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
    return mixer.shape.instance


RELU_MARGIN = 1e-6


def _td(cfg, B, T, precision="fp32", seed=3, tol=None):
    """GPU TD update vs the fp64 oracle for a model described by cfg (bars: tol =
    (forward, gradient), default the fp32 (1e-5, 3e-5)); returns the learner and the
    errors.  fp32: the oracle's ReLU is tie-aware (tests/gpu_util.oracle_td_tie_aware):
    a kept FFN pre-activation within RELU_MARGIN of 0 may take the other branch in
    fp32 than in fp64 whatever the summation order (seed 3 at 40 AGVs has one
    1.8e-8 from 0), and the oracle's backward takes the branch the GPU result agrees
    with; the number of such records is printed."""
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_batch
    A = cfg["n_agents"]
    torch.manual_seed(0)
    args = _args(cfg)
    agent, mixer = TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()
    pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
    pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
    learner = TDLearner(agent, mixer, precision=precision)
    batch, w = make_batch(B, T, A, seed=seed, obs_feats=9, state_feats=8)
    info = learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    g = (learner.grad[:-1] / learner.grad[-1]).cpu()
    prio, ex, ref_g, ties = oracle_td_tie_aware(pa, pm, cfg, batch, w, g if precision == "fp32" else None,
                                                margin=RELU_MARGIN)
    errs = dict(qtot=normwise(info["qtot"], ex["qtot"]), targets=normwise(info["targets"], ex["targets"]),
                prio=normwise(info["td_errors_abs"], prio), grad=normwise(g, ref_g))
    print(cfg.get("tag"), precision, errs, "relu ties", ties)
    tf, tg = tol or (1e-5, 3e-5)
    assert errs["qtot"] < tf and errs["targets"] < tf and errs["prio"] < tf, errs
    assert errs["grad"] < tg, errs
    return learner, errs


def _cfg_of(A, E=32, H=3, D=2, ff=4, **kw):
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=E, heads=H, depth=D, ff_hidden_mult=ff,
               n_actions=5, state_entity_feats=8, mixer_emb=E, mixer_heads=H, mixer_depth=D)
    cfg.update(kw)
    return cfg


@pytest.mark.parametrize("tag,cfg,B,T", [
    ("A5", _cfg_of(5), 4, 6),
    ("A32", _cfg_of(32), 2, 4),
    ("E64H4", _cfg_of(8, E=64, H=4), 3, 5),
    ("E16H1D3", _cfg_of(6, E=16, H=1, D=3, ff=2), 3, 5),
    ("softplus", _cfg_of(8, qmix_pos_func="softplus", qmix_pos_func_beta=0.5), 3, 5),
    ("quadratic", _cfg_of(4, qmix_pos_func="quadratic"), 3, 5),
    # the mixer's obs-token branch through the learner (state = obs.flatten(2),
    # n_tok = A * n_entities; n_transf_mixer.py:60-63), target mixer included
    ("obsbranch", _cfg_of(4, state_entity_mode=False, state_entity_feats=9), 3, 5),
])
def test_generic_td_update_matches_oracle(tag, cfg, B, T):
    require_gpu()
    cfg = dict(cfg, tag=tag)
    _td(cfg, B, T)


def test_headline_shape_with_softplus_head_matches_oracle(monkeypatch):
    """configs[2]'s model with a softplus head: the agent and the mixer run their exact
    8-AGV instances (the mixer's with the head as a run-time parameter, t2o_dispatch.hpp
    T2O_DISPATCH_MIXER mode 2)."""
    require_gpu()
    monkeypatch.setenv("T2O_GENERIC", "0")
    cfg = _cfg_of(8, qmix_pos_func="softplus", qmix_pos_func_beta=2.0, tag="headline-softplus")
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    assert TransformerMixer(_args(cfg)).shape.instance == "exact"
    assert TransformerAgent(None, _args(cfg)).shape.instance == "exact"
    _td(cfg, 4, 6)


def test_forced_generic_equals_tuned_on_headline_shape(monkeypatch):
    """T2O_GENERIC=1 on configs[2]'s model: the runtime-shaped kernels vs the tuned ones."""
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args, make_batch
    A, B, T = 8, 6, 7
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("T2O_GENERIC", mode)
        torch.manual_seed(0)
        args = make_args(A)
        agent, mixer = TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()
        assert agent.shape.generic == (mode == "1") and mixer.shape.generic == (mode == "1")
        learner = TDLearner(agent, mixer)
        batch, w = make_batch(B, T, A, seed=5)
        info = learner.train(batch, 0, 0, per_weight=w)
        torch.cuda.synchronize()
        out[mode] = (info["qtot"].cpu(), (learner.grad[:-1] / learner.grad[-1]).cpu(), learner.params.cpu())
    assert normwise(out["1"][0], out["0"][0]) < 1e-5
    assert normwise(out["1"][1], out["0"][1]) < 3e-5
    # post-Adam: the first Adam step is ~lr·sign(g) elementwise, so grads that differ
    # in rounding move near-zero-gradient entries by up to a few 1e-6 (lr = 1e-3)
    assert normwise(out["1"][2], out["0"][2]) < 2e-5
