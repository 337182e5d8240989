"""Drop-in replacements for the reference's hot-path modules.

``TransformerAgent`` and ``TransformerMixer`` keep the reference constructor
signatures, the args fields they read, ``init_hidden`` and the forward
signatures (transf_agent.py:9-76, n_transf_mixer.py:13-91) and register
exactly the reference parameter tree, so ``state_dict`` keys/shapes match
(SURVEY.md §8 b) and checkpoints move between the two frameworks.

The forward passes run the HIP kernels (one-step unrolls of
t2o_agent_unroll_fwd / t2o_mixer_unroll_fwd); autograd is supported through
the BPTT kernels with T = 1.  The TD update itself does not go through these
per-step forwards: ``t2omca_amd.learner.TDLearner`` runs whole-unroll kernels
on the same parameters.  CPU tensors raise — there is no CPU fallback.
"""
import torch
import torch.nn as nn

from . import _lib, ops


class MultiHeadAttention(nn.Module):
    """Parameter container with the reference names (transformer.py:34-38)."""

    def __init__(self, emb, heads=8, mask=False):
        super().__init__()
        self.emb, self.heads, self.mask = emb, heads, mask
        self.tokeys = nn.Linear(emb, emb * heads, bias=False)
        self.toqueries = nn.Linear(emb, emb * heads, bias=False)
        self.tovalues = nn.Linear(emb, emb * heads, bias=False)
        self.unifyheads = nn.Linear(heads * emb, emb)


class TransformerBlock(nn.Module):
    """Parameter container (transformer.py:103-118)."""

    def __init__(self, emb, heads, mask, ff_hidden_mult=4, dropout=0.0):
        super().__init__()
        self.attention = MultiHeadAttention(emb, heads=heads, mask=mask)
        self.mask = mask
        self.norm1 = nn.LayerNorm(emb)
        self.norm2 = nn.LayerNorm(emb)
        self.ff = nn.Sequential(nn.Linear(emb, ff_hidden_mult * emb), nn.ReLU(),
                                nn.Linear(ff_hidden_mult * emb, emb))
        self.do = nn.Dropout(dropout)


class Transformer(nn.Module):
    """Parameter container (transformer.py:143-167); the compute is fused in HIP."""

    def __init__(self, emb, heads, depth, ff_hidden_mult=4, dropout=0.0):
        super().__init__()
        if dropout != 0.0:
            raise ValueError("t2omca_amd: dropout > 0 is not supported (the reference path uses 0)")
        self.tblocks = nn.Sequential(*[TransformerBlock(emb=emb, heads=heads, mask=False,
                                                        ff_hidden_mult=ff_hidden_mult, dropout=dropout)
                                       for _ in range(depth)])


class _PackCache:
    """The flat parameters and folded kernel pack of a module, rebuilt only when a
    parameter changes.

    The reference MAC calls the agent once per env step (parallel_runner.py:121 ->
    transf_agent.py:54-76) with the same weights until the learner's next update.
    Concatenating and re-packing them on every call (forward and again in the
    backward) cost two extra launches per step.  The key is every parameter's
    storage pointer and autograd version counter: optimiser steps,
    ``load_state_dict`` and ``copy_`` bump the version, re-binding a parameter
    changes its pointer, so a stale pack is never used.  A rebuild allocates new
    tensors, so a pack saved for an earlier backward is never overwritten.
    Writes the version counter cannot see — through ``p.data`` (``p.data.copy_``
    shares the storage, not the counter) or through raw device pointers (the
    learner's Adam kernel) — must be followed by ``invalidate()``."""

    def __init__(self):
        self.key = None
        self.flat = None
        self.pack = None
        self.rebuilds = 0

    def get(self, module, shape):
        params = tuple(module.parameters())
        key = tuple((p.data_ptr(), p._version) for p in params)
        if key != self.key:
            with torch.no_grad():
                flat = torch.cat([p.detach().reshape(-1) for p in params])
            self.flat, self.pack = flat, ops.pack_params(shape, flat)
            self.key = key
            self.rebuilds += 1
        return params, self.flat, self.pack

    def invalidate(self):
        """For writers that bypass autograd's version counters (the learner's Adam
        kernel and broadcasts write the parameters through raw device pointers)."""
        self.key = None


def _split_like(gflat, shapes):
    """The flat gradient (reference parameter order) as one view per parameter."""
    out, o = [], 0
    for sh in shapes:
        n = sh.numel()
        out.append(gflat[o:o + n].view(sh))
        o += n
    return tuple(out)


def orthogonal_init_(m, gain=1.0):
    """PyMARL2's utils.th_utils.orthogonal_init_ (imported by n_transf_mixer.py:6,
    applied to every submodule at :48-50; the module itself is absent from the
    reference, so this restates its published form): orthogonal Linear weights,
    zero biases.  Bias-free Linears (the attention projections) keep no bias."""
    if isinstance(m, nn.Linear):
        nn.init.orthogonal_(m.weight.data, gain=gain)
        if m.bias is not None:
            nn.init.constant_(m.bias.data, 0)


class _AgentStep(torch.autograd.Function):
    """One agent step on the HIP kernels.  The parameters enter as separate inputs
    (their gradients leave as views of one flat buffer), and the cached flat copy
    and pack serve both directions."""

    @staticmethod
    def forward(ctx, shape, flat, pack, inputs, hidden, *params):
        b, a, nf = inputs.shape
        obs = inputs.detach().contiguous().view(b, 1, a, nf)
        h0 = hidden.detach().reshape(b * a, shape.E).contiguous()
        q, h = ops.agent_unroll_fwd(shape, pack, obs, h0_on=h0)
        ctx.save_for_backward(flat, pack, obs, h0, h)
        ctx.shape, ctx.param_shapes = shape, [p.shape for p in params]
        return q[:, 0], h[:, 0]

    @staticmethod
    def backward(ctx, gq, gh):
        flat, pack, obs, h0, h = ctx.saved_tensors
        shape = ctx.shape
        b, _, a, _ = obs.shape
        gq = (gq if gq is not None else torch.zeros_like(h[:, 0, :, :0])).contiguous().view(b, 1, a, -1)
        gh = (gh if gh is not None else torch.zeros_like(h[:, 0])).contiguous().view(b, 1, a, shape.E)
        gpack, gh0 = ops.agent_unroll_bwd(shape, pack, obs, h, h0=h0, gq=gq, gh=gh, want_gh0=True)
        gflat = torch.zeros_like(flat)
        ops.unpack_grads(shape, flat, gpack, gflat)
        return (None, None, None, None, gh0.view(b, a, shape.E)) + _split_like(gflat, ctx.param_shapes)


class TransformerAgent(nn.Module):
    """transf_agent.py:8-76 drop-in (HIP forward/backward)."""

    def __init__(self, input_shape, args):
        super().__init__()
        self.args = args
        self.n_agents = args.n_agents
        self.n_entities = getattr(self.args, "n_entities_obs", self.args.n_entities)
        self.feat_dim = args.obs_entity_feats
        self.emb_dim = args.emb
        self.feat_embedding = nn.Linear(self.feat_dim, self.emb_dim)
        self.transformer = Transformer(args.emb, args.heads, args.depth, args.ff_hidden_mult, args.dropout)
        if getattr(self.args, "action_selector", None) == "noisy-new":
            raise NotImplementedError("t2omca_amd: the NoisyLinear head (transf_agent.py:37-39) is not on "
                                      "the fused path")
        self.q_basic = nn.Linear(args.emb, args.n_actions)
        self.shape = ops.NetShape(ops.AGENT, args.emb, args.heads, args.depth, self.feat_dim, args.n_actions,
                                  args.ff_hidden_mult * args.emb, self.n_entities)
        self._pack_cache = _PackCache()

    def init_hidden(self):
        return torch.zeros(1, self.args.emb, device=self.args.device)

    def forward(self, inputs, hidden_state):
        b, a, _ = inputs.size()
        if b * a * self.emb_dim != hidden_state.numel():
            hidden_state = hidden_state.expand(b, a, self.emb_dim)
        params, flat, pack = self._pack_cache.get(self, self.shape)
        q, h = _AgentStep.apply(self.shape, flat, pack, inputs, hidden_state, *params)
        return q.view(b, a, -1), h.view(b, a, -1)


class _MixerStep(torch.autograd.Function):
    """One mixer step on the HIP kernels (parameters as separate inputs, as _AgentStep)."""

    @staticmethod
    def forward(ctx, shape, flat, pack, qvals, hidden_states, hyper_weights, states, *params):
        b = qvals.shape[0]
        A, E = shape.agents, shape.E
        qv = qvals.detach().reshape(b, 1, A).contiguous()
        hid = hidden_states.detach().reshape(b, 1, A, E).contiguous()
        hw0 = hyper_weights.detach().reshape(b, 3, E).contiguous()
        st = states.detach().reshape(b, 1, -1).contiguous()
        out = ops.mixer_unroll_fwd(shape, pack, st, hid, qmode_on=0, qv_on=qv, hw0_on=hw0)
        ctx.save_for_backward(flat, pack, qv, hid, hw0, st, out["y"], out["hw"], out["qv"], out["xout"])
        ctx.xmid = out["xmid"]
        ctx.shape, ctx.param_shapes = shape, [p.shape for p in params]
        return out["y"].view(b, 1, 1), out["hw"][:, 0]

    @staticmethod
    def backward(ctx, gy, ghw):
        flat, pack, qv, hid, hw0, st, y, hw, qvo, xout = ctx.saved_tensors
        shape = ctx.shape
        b = qv.shape[0]
        gy = (gy if gy is not None else torch.zeros_like(y)).reshape(b, 1).contiguous()
        ghw = ghw.reshape(b, 1, 3, shape.E).contiguous() if ghw is not None else None
        fwd = dict(y=y, hw=hw, qv=qvo, xout=xout, xmid=ctx.xmid)
        gpack, gqv, ghid, ghw0 = ops.mixer_unroll_bwd(shape, pack, st, hid, fwd, gy, hw0=hw0, ghw_ext=ghw,
                                                      want_ghw0=True)
        gflat = torch.zeros_like(flat)
        ops.unpack_grads(shape, flat, gpack, gflat)
        return ((None, None, None, gqv.view(b, 1, -1), ghid.view(b, -1, shape.E), ghw0, None)
                + _split_like(gflat, ctx.param_shapes))


class TransformerMixer(nn.Module):
    """n_transf_mixer.py:12-102 drop-in (HIP forward/backward).

    Every pos_func of the reference (:95-103: softplus with qmix_pos_func_beta,
    quadratic, abs, anything else = identity), both input branches (:60-63:
    state_entity_mode -> the n_entities_state state tokens; otherwise the
    n_agents * n_entities obs tokens, which needs state_entity_feats == the obs
    feature width), n_entities_state != n_agents and use_orthogonal (:48-50).
    Shapes without a tuned MFMA instance run the runtime-shaped kernels."""

    def __init__(self, args, abs=True):
        super().__init__()
        self.args = args
        self.n_agents = args.n_agents
        self.n_entities = getattr(self.args, "n_entities_state", self.args.n_entities)
        self.feat_dim = args.state_entity_feats
        self.emb_dim = args.mixer_emb
        self.feat_embedding = nn.Linear(self.feat_dim, self.emb_dim)
        self.transformer = Transformer(args.mixer_emb, args.mixer_heads, args.mixer_depth,
                                       args.ff_hidden_mult, args.dropout)
        self.qmix_pos_func = getattr(self.args, "qmix_pos_func", "abs")
        self.custom_space = args.env_args.get("state_entity_mode", True)
        self.hyper_b2 = nn.Linear(self.emb_dim, 1)
        if getattr(args, "use_orthogonal", False):
            for m in self.modules():
                orthogonal_init_(m)
        pos = _lib.POS_FUNCS.get(self.qmix_pos_func, 3)
        beta = float(getattr(args, "qmix_pos_func_beta", 1.0)) if self.qmix_pos_func == "softplus" else 1.0
        # state tokens: the state's entities, or (obs branch) every agent's obs entities
        n_tok = self.n_entities if self.custom_space else self.n_agents * self.n_entities
        self.shape = ops.NetShape(ops.MIXER, args.mixer_emb, args.mixer_heads, args.mixer_depth, self.feat_dim, 1,
                                  args.ff_hidden_mult * args.mixer_emb, n_tok, n_agents=self.n_agents,
                                  pos_func=pos, pos_beta=beta)
        self._pack_cache = _PackCache()

    def init_hidden(self):
        # n_transf_mixer.py:52-53 (shape [1, A, E] as in the reference)
        return torch.zeros(1, self.n_agents, self.args.emb, device=self.args.device)

    def forward(self, qvals, hidden_states, hyper_weights, states, obs):
        b = qvals.size(0)
        hyper_weights = hyper_weights.expand(b, 3, self.emb_dim)
        tokens = states if self.custom_space else obs  # n_transf_mixer.py:60-63
        params, flat, pack = self._pack_cache.get(self, self.shape)
        return _MixerStep.apply(self.shape, flat, pack, qvals, hidden_states, hyper_weights, tokens, *params)
