"""Generate golden vectors from the REFERENCE modules (build container only).

Run:  python tests/golden/make_golden.py   (needs /root/reference; never on the GPU box)

The reference agent/mixer (transf_agent.py, n_transf_mixer.py, transformer.py)
are imported through a throw-away shim in a temp dir (SURVEY.md §8 c): package
stubs for the relative imports, a NoisyLinear / orthogonal_init_ stub and a
``turtle`` stub for n_transf_mixer.py:1.  No reference source is copied into
the repository; only the produced input/output arrays are committed.

Fixtures written (numpy .npz, allow_pickle=False):
  agent_<tag>.npz   params (fp32 values), obs [b,T,A,A*F], h0, and for
                    fp64 and fp32: q [b,T,A,nA], h [b,T,A,E]; fp64 gradients of
                    L = sum(cq*q) + sum(ch*h) w.r.t. every parameter, obs and h0.
  mixer_<tag>.npz   params, qvals [b,T,A], hidden [b,T,A,E], states [b,T,ns*8]
                    (or, state_entity_mode off, obs [b,T,A,A*F]), hw0 [b,3,E];
                    y [b,T], hw [b,T,3,E] (fp64 + fp32); fp64 gradients of
                    L = sum(cy*y) + sum(chw*hw) w.r.t. params, qvals and hidden.
  meta/<field>      the args fields an EXTENDED fixture overrides.

    python tests/golden/make_golden.py [tag ...]   (default: every fixture)
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.ref_model import init_params  # noqa: E402

REF = "/root/reference"

CONFIGS = {
    # tag: (A, E, H, D, b, T)
    "a3_e16_h2_d1": (3, 16, 2, 1, 3, 4),
    "a8_e32_h3_d2": (8, 32, 3, 2, 4, 5),
    "a16_e32_h3_d2": (16, 32, 3, 2, 2, 4),
}

# Shapes / options outside the tuned kernel instances (the runtime-shaped path):
# tag: (kinds, A, E, H, D, b, T, extra args).  Extra args override make_args'
# fields and are stored in the fixture as meta/<name> (test_oracle_golden._cfg).
EXTENDED = {
    "a5_e32_h3_d2": ("am", 5, 32, 3, 2, 3, 4, {}),
    "a32_e32_h3_d2": ("am", 32, 32, 3, 2, 2, 3, {}),
    "a8_e64_h4_d2": ("am", 8, 64, 4, 2, 2, 3, {}),
    "a6_e16_h1_d3_ff2": ("am", 6, 16, 1, 3, 2, 4, {"ff_hidden_mult": 2}),
    "a4_ne6": ("a", 4, 32, 3, 2, 2, 4, {"n_entities_obs": 6}),
    "a4_ns6": ("m", 4, 32, 3, 2, 2, 4, {"n_entities_state": 6}),
    "a8_softplus": ("m", 8, 32, 3, 2, 3, 4, {"qmix_pos_func": "softplus", "qmix_pos_func_beta": 0.5}),
    "a8_quadratic": ("m", 8, 32, 3, 2, 3, 4, {"qmix_pos_func": "quadratic"}),
    "a8_identity": ("m", 8, 32, 3, 2, 3, 4, {"qmix_pos_func": "none"}),
    "a3_obsbranch": ("m", 3, 32, 3, 2, 2, 3, {"state_entity_mode": False, "state_entity_feats": 9}),
}


def build_shim():
    root = tempfile.mkdtemp(prefix="t2o_shim_")
    for d in ["modules", "modules/layer", "modules/agents", "modules/mixers", "utils"]:
        os.makedirs(os.path.join(root, d), exist_ok=True)
        open(os.path.join(root, d, "__init__.py"), "w").close()
    os.symlink(f"{REF}/transformer.py", f"{root}/modules/layer/transformer.py")
    os.symlink(f"{REF}/transf_agent.py", f"{root}/modules/agents/transf_agent.py")
    os.symlink(f"{REF}/n_transf_mixer.py", f"{root}/modules/mixers/n_transf_mixer.py")
    with open(f"{root}/utils/noisy_liner.py", "w") as f:
        f.write("class NoisyLinear:\n    pass\n")
    with open(f"{root}/utils/th_utils.py", "w") as f:
        f.write("def orthogonal_init_(m, gain=1):\n    pass\n")
    sys.path.insert(0, root)
    sys.modules["turtle"] = types.SimpleNamespace(forward=None)
    from modules.agents.transf_agent import TransformerAgent
    from modules.mixers.n_transf_mixer import TransformerMixer
    return TransformerAgent, TransformerMixer


def make_args(A, E, H, D, extra=None):
    a = types.SimpleNamespace(
        n_agents=A, n_entities=A, obs_entity_feats=9, emb=E, heads=H, depth=D,
        ff_hidden_mult=4, dropout=0.0, action_selector="epsilon_greedy", n_actions=5,
        device="cpu", state_entity_feats=8, mixer_emb=E, mixer_heads=H, mixer_depth=D,
        env_args={"state_entity_mode": True})
    for k, v in (extra or {}).items():
        if k == "state_entity_mode":
            a.env_args = {"state_entity_mode": v}
        else:
            setattr(a, k, v)
    return a


def cfg_of(args):
    cfg = dict(n_agents=args.n_agents, n_entities=args.n_entities, obs_entity_feats=9,
               emb=args.emb, heads=args.heads, depth=args.depth, ff_hidden_mult=args.ff_hidden_mult,
               n_actions=5, state_entity_feats=args.state_entity_feats, mixer_emb=args.emb,
               mixer_heads=args.heads, mixer_depth=args.depth)
    for k in ("n_entities_obs", "n_entities_state", "qmix_pos_func", "qmix_pos_func_beta"):
        if hasattr(args, k):
            cfg[k] = getattr(args, k)
    cfg["state_entity_mode"] = args.env_args["state_entity_mode"]
    return cfg


def meta(extra):
    return {"meta/" + k: np.asarray(v) for k, v in (extra or {}).items()}


def gen_agent(TA, tag, A, E, H, D, b, T, seed, extra=None):
    args = make_args(A, E, H, D, extra)
    cfg = cfg_of(args)
    params = init_params("agent", cfg, seed)
    g = torch.Generator().manual_seed(seed + 1)
    ne = getattr(args, "n_entities_obs", A)
    obs = torch.randn(b, T, A, ne * 9, generator=g, dtype=torch.float64)
    h0 = 0.5 * torch.randn(b, A, E, generator=g, dtype=torch.float64)
    cq = torch.randn(b, T, A, 5, generator=g, dtype=torch.float64)
    ch = torch.randn(b, T, A, E, generator=g, dtype=torch.float64)
    out = {"obs": obs.numpy(), "h0": h0.numpy(), "cq": cq.numpy(), "ch": ch.numpy(), **meta(extra)}
    for k, v in params.items():
        out["param/" + k] = v.numpy()
    for dt, name in [(torch.float64, "f64"), (torch.float32, "f32")]:
        agent = TA(None, args).to(dt)
        agent.load_state_dict({k: v.to(dt) for k, v in params.items()})
        o = obs.to(dt).clone().requires_grad_(dt == torch.float64)
        h = h0.to(dt).clone().requires_grad_(dt == torch.float64)
        qs, hs = [], []
        hh = h
        for t in range(T):
            q, hh = agent.forward(o[:, t].contiguous(), hh)
            qs.append(q)
            hs.append(hh)
        qs, hs = torch.stack(qs, 1), torch.stack(hs, 1)
        out[f"q_{name}"] = qs.detach().numpy()
        out[f"h_{name}"] = hs.detach().numpy()
        if dt == torch.float64:
            loss = (qs * cq).sum() + (hs * ch).sum()
            loss.backward()
            for k, p in agent.named_parameters():
                out["grad/" + k] = p.grad.numpy()
            out["grad_obs"] = o.grad.numpy()
            out["grad_h0"] = h.grad.numpy()
    np.savez(os.path.join(HERE, f"agent_{tag}.npz"), **out)


def gen_mixer(TM, tag, A, E, H, D, b, T, seed, extra=None):
    args = make_args(A, E, H, D, extra)
    cfg = cfg_of(args)
    params = init_params("mixer", cfg, seed)
    g = torch.Generator().manual_seed(seed + 2)
    qvals = torch.randn(b, T, A, generator=g, dtype=torch.float64)
    hidden = torch.randn(b, T, A, E, generator=g, dtype=torch.float64)
    ns = getattr(args, "n_entities_state", A)
    state_mode = args.env_args["state_entity_mode"]
    # state_entity_mode off: the mixer reads obs [b, A, n_entities * feats] (n_transf_mixer.py:63)
    states = (torch.randn(b, T, ns * 8, generator=g, dtype=torch.float64) if state_mode
              else torch.randn(b, T, A, A * args.state_entity_feats, generator=g, dtype=torch.float64))
    hw0 = 0.5 * torch.randn(b, 3, E, generator=g, dtype=torch.float64)
    cy = torch.randn(b, T, generator=g, dtype=torch.float64)
    chw = torch.randn(b, T, 3, E, generator=g, dtype=torch.float64)
    out = {"qvals": qvals.numpy(), "hidden": hidden.numpy(), "states": states.numpy(),
           "hw0": hw0.numpy(), "cy": cy.numpy(), "chw": chw.numpy(), **meta(extra)}
    for k, v in params.items():
        out["param/" + k] = v.numpy()
    for dt, name in [(torch.float64, "f64"), (torch.float32, "f32")]:
        mixer = TM(args).to(dt)
        mixer.load_state_dict({k: v.to(dt) for k, v in params.items()})
        qv = qvals.to(dt).clone().requires_grad_(dt == torch.float64)
        hd = hidden.to(dt).clone().requires_grad_(dt == torch.float64)
        hw = hw0.to(dt).clone().requires_grad_(dt == torch.float64)
        st = states.to(dt)
        ys, hws = [], []
        cur = hw
        for t in range(T):
            if state_mode:
                y, cur = mixer.forward(qv[:, t:t + 1], hd[:, t], cur, st[:, t], None)
            else:
                y, cur = mixer.forward(qv[:, t:t + 1], hd[:, t], cur, None, st[:, t])
            ys.append(y.view(-1))
            hws.append(cur)
        ys, hws = torch.stack(ys, 1), torch.stack(hws, 1)
        out[f"y_{name}"] = ys.detach().numpy()
        out[f"hw_{name}"] = hws.detach().numpy()
        if dt == torch.float64:
            loss = (ys * cy).sum() + (hws * chw).sum()
            loss.backward()
            for k, p in mixer.named_parameters():
                out["grad/" + k] = p.grad.numpy()
            out["grad_qvals"] = qv.grad.numpy()
            out["grad_hidden"] = hd.grad.numpy()
            out["grad_hw0"] = hw.grad.numpy()
    np.savez(os.path.join(HERE, f"mixer_{tag}.npz"), **out)


def main():
    TA, TM = build_shim()
    only = set(sys.argv[1:])  # tags to (re)write; default all
    for i, (tag, (A, E, H, D, b, T)) in enumerate(CONFIGS.items()):
        if only and tag not in only:
            continue
        gen_agent(TA, tag, A, E, H, D, b, T, seed=100 + i)
        gen_mixer(TM, tag, A, E, H, D, b, T, seed=200 + i)
        print("wrote", tag)
    for i, (tag, (kinds, A, E, H, D, b, T, extra)) in enumerate(EXTENDED.items()):
        if only and tag not in only:
            continue
        if "a" in kinds:
            gen_agent(TA, tag, A, E, H, D, b, T, seed=300 + i, extra=extra)
        if "m" in kinds:
            gen_mixer(TM, tag, A, E, H, D, b, T, seed=400 + i, extra=extra)
        print("wrote", tag)


if __name__ == "__main__":
    main()
