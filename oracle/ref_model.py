"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

PyTorch-CPU restatement of the reference transformer agent and mixer, written
from scratch as functions over ``state_dict``-keyed parameter dicts.  The op
order mirrors the reference so that the fp64 restatement equals the reference
to rounding and the fp32 one is the "reference CPU path" timed by bench.py:

* ``mha``            — transformer.py:40-84 (wide heads: every head has width
  ``emb``; Q and K both scaled by emb**-1/4; bias-free Q/K/V projections;
  ``unifyheads`` with bias; the mask branches are dead on this path).
* ``block``          — transformer.py:120-140 (post-LN; returns the ORIGINAL
  keys, so every block attends over the layer-0 input).
* ``transformer``    — transformer.py:169-178.
* ``agent_forward``  — transf_agent.py:54-76 (hidden token first, Q read from
  token 0).
* ``mixer_forward``  — n_transf_mixer.py:55-103 (w1/b1/w2/b2 from the last A+3
  output tokens, elu hidden layer; pos_func abs / softplus(beta) / quadratic /
  identity; state tokens from the state, or from every agent's obs when
  state_entity_mode is off, :60-63).
"""
import torch
import torch.nn.functional as F


def _lin(x, p, name, bias=True):
    w = p[name + ".weight"]
    b = p.get(name + ".bias") if bias else None
    return F.linear(x, w, b)


def mha(p, pre, q, k, heads):
    """transformer.py:40-84 with mask=None and self.mask=False."""
    h = heads
    b_q, t_q, e_q = q.size()
    b, t_k, e = k.size()
    keys = F.linear(k, p[pre + "tokeys.weight"]).view(b, t_k, h, e)
    values = F.linear(k, p[pre + "tovalues.weight"]).view(b, t_k, h, e)
    queries = F.linear(q, p[pre + "toqueries.weight"]).view(b, t_q, h, e)
    keys = keys.transpose(1, 2).contiguous().view(b * h, t_k, e)
    values = values.transpose(1, 2).contiguous().view(b * h, t_k, e)
    queries = queries.transpose(1, 2).contiguous().view(b * h, t_q, e)
    queries = queries / (e ** (1 / 4))
    keys = keys / (e ** (1 / 4))
    dot = torch.bmm(queries, keys.transpose(1, 2))
    dot = F.softmax(dot, dim=2)
    out = torch.bmm(dot, values).view(b, h, t_q, e)
    out = out.transpose(1, 2).contiguous().view(b, t_q, h * e)
    return F.linear(out, p[pre + "unifyheads.weight"], p[pre + "unifyheads.bias"])


# The FFN's ReLU (transformer.py:113).  Tests may install a TieAwareRelu here
# (oracle/ref_learner.py td_forward(relu=...)) to choose the backward branch of
# pre-activations that lie within rounding of 0; None = F.relu.
_ffn_relu = None


def block(p, pre, q, k, heads, keep=None):
    """transformer.py:120-140 (dropout p=0 is the identity).  keep: the token rows
    whose block output is consumed downstream (token pruning; only a tie-aware
    ReLU hook reads it)."""
    e = q.shape[-1]
    attended = mha(p, pre + "attention.", q, k, heads)
    x = F.layer_norm(attended + q, (e,), p[pre + "norm1.weight"], p[pre + "norm1.bias"])
    ff = F.linear(x, p[pre + "ff.0.weight"], p[pre + "ff.0.bias"])
    if _ffn_relu is None:
        ff = F.relu(ff)
    else:  # (the hook also gets Σ_e |W1[j,e] x_e| + |c1[j]|: the pre-activation's rounding scale)
        scale = F.linear(x.detach().abs(), p[pre + "ff.0.weight"].detach().abs(), p[pre + "ff.0.bias"].detach().abs())
        ff = _ffn_relu(ff, keep, scale)
    ff = F.linear(ff, p[pre + "ff.2.weight"], p[pre + "ff.2.bias"])
    x = F.layer_norm(ff + x, (e,), p[pre + "norm2.weight"], p[pre + "norm2.bias"])
    return x


def transformer(p, pre, q, k, heads, depth, keep=None):
    """transformer.py:169-178: keys are never updated across blocks."""
    x = q
    for d in range(depth):
        x = block(p, f"{pre}tblocks.{d}.", x, k, heads, keep)
    return x


def agent_forward(p, inputs, hidden_state, *, n_entities, feat_dim, emb, heads, depth):
    """transf_agent.py:54-76 -> (q [b,a,nA], h [b,a,E])."""
    b, a, _ = inputs.size()
    inputs = inputs.reshape(-1, n_entities, feat_dim)
    hidden_state = hidden_state.reshape(-1, 1, emb)
    embs = _lin(inputs, p, "feat_embedding")
    x = torch.cat((hidden_state, embs), 1)
    embs = transformer(p, "transformer.", x, x, heads, depth, keep=slice(0, 1))
    h = embs[:, 0:1, :]
    q = _lin(h, p, "q_basic")
    return q.view(b, a, -1), h.view(b, a, -1)


def mixer_forward(p, qvals, hidden_states, hyper_weights, states, *, n_agents, n_entities,
                  feat_dim, emb, heads, depth, pos_func="abs", pos_beta=1.0, obs=None):
    """n_transf_mixer.py:55-103 -> (y [b,1,1], hw [b,3,E]).  obs given: the
    custom_space=False branch (tokens = obs.reshape(b, n_agents*n_entities, feat_dim))."""
    b, _, _ = qvals.size()
    if obs is None:
        inputs = states.reshape(b, n_entities, feat_dim)
    else:
        inputs = obs.reshape(b, n_agents * n_entities, feat_dim)
    embs = _lin(inputs, p, "feat_embedding")
    x = torch.cat((embs, hidden_states, hyper_weights), 1)
    embs = transformer(p, "transformer.", x, x, heads, depth, keep=slice(x.shape[1] - n_agents - 3, None))
    w1 = embs[:, -3 - n_agents:-3, :]
    b1 = embs[:, -3, :].view(-1, 1, emb)
    w2 = embs[:, -2, :].view(-1, emb, 1)
    b2 = F.relu(_lin(embs[:, -1, :], p, "hyper_b2")).view(-1, 1, 1)
    if pos_func == "softplus":
        w1, w2 = F.softplus(w1, beta=pos_beta), F.softplus(w2, beta=pos_beta)  # nn.Softplus: threshold 20
    elif pos_func == "quadratic":
        w1, w2 = 0.5 * w1 ** 2, 0.5 * w2 ** 2
    elif pos_func == "abs":
        w1, w2 = torch.abs(w1), torch.abs(w2)
    hidden = F.elu(torch.matmul(qvals, w1) + b1)
    y = torch.matmul(hidden, w2) + b2
    return y, embs[:, -3:, :]


def agent_unroll(p, obs, h0, *, cfg):
    """Unroll the agent over obs [b, T, A, n_ent*F] from hidden h0 [b, A, E].

    Returns q [b, T, A, nA] and h [b, T, A, E] (h[:, t] = hidden after step t)."""
    qs, hs = [], []
    h = h0
    for t in range(obs.shape[1]):
        q, h = agent_forward(p, obs[:, t].contiguous(), h, n_entities=cfg.get("n_entities_obs", cfg["n_entities"]),
                             feat_dim=cfg["obs_entity_feats"], emb=cfg["emb"],
                             heads=cfg["heads"], depth=cfg["depth"])
        qs.append(q)
        hs.append(h)
    return torch.stack(qs, 1), torch.stack(hs, 1)


def mixer_unroll(p, qvals, hidden, states, hw0, *, cfg, obs=None):
    """Unroll the mixer over qvals [b,T,A], hidden [b,T,A,E], states [b,T,S]
    (or, state_entity_mode False, obs [b,T,A,n_ent*F]).

    The 3 hyper-weight tokens are recurrent (n_transf_mixer.py:69,91).
    Returns y [b, T] and hw [b, T, 3, E] (hw[:, t] = hyper tokens after step t)."""
    ys, hws = [], []
    hw = hw0
    for t in range(qvals.shape[1]):
        y, hw = mixer_forward(p, qvals[:, t:t + 1], hidden[:, t], hw, states[:, t] if states is not None else None,
                              n_agents=cfg["n_agents"], n_entities=cfg.get("n_entities_state", cfg["n_entities"]),
                              feat_dim=cfg["state_entity_feats"], emb=cfg["mixer_emb"],
                              heads=cfg["mixer_heads"], depth=cfg["mixer_depth"],
                              pos_func=cfg.get("qmix_pos_func", "abs"), pos_beta=cfg.get("qmix_pos_func_beta", 1.0),
                              obs=None if obs is None else obs[:, t])
        ys.append(y.view(-1))
        hws.append(hw)
    return torch.stack(ys, 1), torch.stack(hws, 1)


def init_params(kind, cfg, seed, dtype=torch.float32):
    """torch-default-initialised parameters with the reference state_dict keys
    (SURVEY.md §8 b).  Uses nn.Linear/nn.LayerNorm constructors so the init
    distribution equals the reference modules' own."""
    g = torch.Generator().manual_seed(seed)
    E = cfg["emb"] if kind == "agent" else cfg["mixer_emb"]
    H = cfg["heads"] if kind == "agent" else cfg["mixer_heads"]
    D = cfg["depth"] if kind == "agent" else cfg["mixer_depth"]
    Fd = cfg["obs_entity_feats"] if kind == "agent" else cfg["state_entity_feats"]
    FF = cfg.get("ff_hidden_mult", 4) * E
    shapes = [("feat_embedding", (E, Fd), True)]
    for d in range(D):
        pre = f"transformer.tblocks.{d}."
        shapes += [(pre + "attention.tokeys", (H * E, E), False),
                   (pre + "attention.toqueries", (H * E, E), False),
                   (pre + "attention.tovalues", (H * E, E), False),
                   (pre + "attention.unifyheads", (E, H * E), True),
                   (pre + "norm1", None, "ln"), (pre + "norm2", None, "ln"),
                   (pre + "ff.0", (FF, E), True), (pre + "ff.2", (E, FF), True)]
    if kind == "agent":
        shapes.append(("q_basic", (cfg["n_actions"], E), True))
    else:
        shapes.append(("hyper_b2", (1, E), True))
    p = {}
    for name, shp, bias in shapes:
        if bias == "ln":
            # LayerNorm defaults are ones/zeros; perturb so LN affine is exercised.
            p[name + ".weight"] = (1.0 + 0.1 * torch.randn(E, generator=g)).to(dtype)
            p[name + ".bias"] = (0.1 * torch.randn(E, generator=g)).to(dtype)
            continue
        fan_in = shp[1]
        bound = 1.0 / (fan_in ** 0.5)
        p[name + ".weight"] = ((torch.rand(shp, generator=g) * 2 - 1) * bound).to(dtype)
        if bias:
            p[name + ".bias"] = ((torch.rand(shp[0], generator=g) * 2 - 1) * bound).to(dtype)
    return p


class _MaskedRelu(torch.autograd.Function):
    """relu(x) = x * mask with mask = [x > 0]; the backward multiplies by the mask
    as it is WHEN THE BACKWARD RUNS, so a caller may flip entries between
    backward passes of one graph (TieAwareRelu)."""

    @staticmethod
    def forward(ctx, x, mask):
        ctx.mask = mask  # not save_for_backward: it is meant to be edited in place
        return x * mask

    @staticmethod
    def backward(ctx, g):
        return g * ctx.mask, None


class TieAwareRelu:
    """FFN ReLU that records every pre-activation of a consumed token row lying
    within `margin` of 0 (a "tie": fp32 arithmetic in any summation order may put
    it on the other side of 0 than fp64 does) and lets the caller choose each tie's
    backward branch.  The forward value at a tie differs between the branches by
    less than `margin`, so only the backward is overridden; ties are recorded in
    execution order, for tensors that require grad (the online networks)."""

    def __init__(self, margin):
        self.margin = margin
        self.ties = []  # (mask tensor, flat index, fp64 pre-activation)
        self.scales = []  # per tie: Σ_e |W1[j,e] x_e| + |c1[j]| (0 when the caller gave none)
        self.where = []  # per tie: (hook call number, [token, unit] shape of the call, flat index)
        self.calls = 0

    def __call__(self, x, keep, scale=None):
        mask = (x.detach() > 0).to(x.dtype)
        if x.requires_grad:
            near = x.detach().abs() < self.margin
            if keep is not None:
                kept = torch.zeros_like(near)
                kept[:, keep] = True
                near &= kept
            for i in near.reshape(-1).nonzero().reshape(-1).tolist():
                self.ties.append((mask, i, float(x.detach().reshape(-1)[i])))
                self.scales.append(0.0 if scale is None else float(scale.reshape(-1)[i]))
                self.where.append((self.calls, tuple(x.shape), i))
        self.calls += 1
        return _MaskedRelu.apply(x, mask)

    def branches(self):
        return [bool(m.reshape(-1)[i] > 0) for m, i, _ in self.ties]

    def set_branches(self, on):
        for (m, i, _), b in zip(self.ties, on):
            m.reshape(-1)[i] = 1.0 if b else 0.0
