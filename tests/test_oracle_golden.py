"""Pin the CPU oracle (oracle/ref_model.py) to golden vectors produced by the
reference modules themselves (tests/golden/make_golden.py)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import ref_model

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cfg(z, kind):
    p = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param/")}
    E = p["feat_embedding.weight"].shape[0]
    H = p["transformer.tblocks.0.attention.tokeys.weight"].shape[0] // E
    D = len({k.split(".")[2] for k in p if k.startswith("transformer.tblocks.")})
    if kind == "agent":
        A = z["obs"].shape[2]
    else:
        A = z["qvals"].shape[2]
    FF = p["transformer.tblocks.0.ff.0.weight"].shape[0]
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=E, heads=H, depth=D,
               ff_hidden_mult=FF // E, n_actions=5, state_entity_feats=8, mixer_emb=E,
               mixer_heads=H, mixer_depth=D)
    # EXTENDED fixtures (make_golden.py): the args fields they override
    for k in z.files:
        if k.startswith("meta/"):
            v = z[k].item()
            cfg[k[5:]] = v.decode() if isinstance(v, bytes) else v
    return p, cfg


def _mixer_inputs(z, dt):
    """(states, obs) for mixer_unroll: the obs branch (state_entity_mode off) feeds obs."""
    st = torch.from_numpy(z["states"]).to(dt)
    if "meta/state_entity_mode" in z.files and not bool(z["meta/state_entity_mode"]):
        return None, st
    return st, None


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "agent_*.npz"))))
def test_agent_oracle_matches_reference(path):
    z = np.load(path)
    p, cfg = _cfg(z, "agent")
    for dt, name, tol in [(torch.float64, "f64", 1e-13), (torch.float32, "f32", 2e-6)]:
        pp = {k: v.to(dt) for k, v in p.items()}
        q, h = ref_model.agent_unroll(pp, torch.from_numpy(z["obs"]).to(dt),
                                      torch.from_numpy(z["h0"]).to(dt), cfg=cfg)
        assert _rel(q.numpy(), z[f"q_{name}"]) < tol
        assert _rel(h.numpy(), z[f"h_{name}"]) < tol


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "agent_*.npz"))))
def test_agent_oracle_grads_match_reference(path):
    z = np.load(path)
    p, cfg = _cfg(z, "agent")
    pp = {k: v.double().requires_grad_(True) for k, v in p.items()}
    obs = torch.from_numpy(z["obs"]).requires_grad_(True)
    h0 = torch.from_numpy(z["h0"]).requires_grad_(True)
    q, h = ref_model.agent_unroll(pp, obs, h0, cfg=cfg)
    loss = (q * torch.from_numpy(z["cq"])).sum() + (h * torch.from_numpy(z["ch"])).sum()
    loss.backward()
    for k, v in pp.items():
        assert _rel(v.grad.numpy(), z["grad/" + k]) < 1e-12, k
    assert _rel(obs.grad.numpy(), z["grad_obs"]) < 1e-12
    assert _rel(h0.grad.numpy(), z["grad_h0"]) < 1e-12


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "mixer_*.npz"))))
def test_mixer_oracle_matches_reference(path):
    z = np.load(path)
    p, cfg = _cfg(z, "mixer")
    for dt, name, tol in [(torch.float64, "f64", 1e-13), (torch.float32, "f32", 2e-6)]:
        pp = {k: v.to(dt) for k, v in p.items()}
        st, ob = _mixer_inputs(z, dt)
        y, hw = ref_model.mixer_unroll(pp, torch.from_numpy(z["qvals"]).to(dt),
                                       torch.from_numpy(z["hidden"]).to(dt), st,
                                       torch.from_numpy(z["hw0"]).to(dt), cfg=cfg, obs=ob)
        assert _rel(y.numpy(), z[f"y_{name}"]) < tol
        assert _rel(hw.numpy(), z[f"hw_{name}"]) < tol


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "mixer_*.npz"))))
def test_mixer_oracle_grads_match_reference(path):
    z = np.load(path)
    p, cfg = _cfg(z, "mixer")
    pp = {k: v.double().requires_grad_(True) for k, v in p.items()}
    qv = torch.from_numpy(z["qvals"]).requires_grad_(True)
    hd = torch.from_numpy(z["hidden"]).requires_grad_(True)
    hw0 = torch.from_numpy(z["hw0"]).requires_grad_(True)
    st, ob = _mixer_inputs(z, torch.float64)
    y, hw = ref_model.mixer_unroll(pp, qv, hd, st, hw0, cfg=cfg, obs=ob)
    loss = (y * torch.from_numpy(z["cy"])).sum() + (hw * torch.from_numpy(z["chw"])).sum()
    loss.backward()
    for k, v in pp.items():
        assert _rel(v.grad.numpy(), z["grad/" + k]) < 1e-12, k
    assert _rel(qv.grad.numpy(), z["grad_qvals"]) < 1e-12
    assert _rel(hd.grad.numpy(), z["grad_hidden"]) < 1e-12
    assert _rel(hw0.grad.numpy(), z["grad_hw0"]) < 1e-12
