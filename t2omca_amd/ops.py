"""Thin torch-tensor wrappers over the C-ABI entry points (include/t2omca.h).

Every function checks device/dtype/contiguity on the host, then launches on
the current HIP stream.  There is no CPU path: CPU tensors raise.
"""
import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import (AgentBwdArgs, AgentFwdArgs, MixerBwdArgs, MixerFwdArgs, TapeArgs, TDArgs, check, lib, ptr,
                   stream_ptr)

AGENT, MIXER = 0, 1


def _dev(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("t2omca_amd ops need HIP-device tensors (no CPU fallback); "
                               "the CPU restatement lives in oracle/ and is test-only")
        if t.dtype not in (torch.float32, torch.int64):
            raise TypeError(f"t2omca_amd: unsupported dtype {t.dtype}")


@dataclass(frozen=True)
class NetShape:
    kind: int
    E: int
    H: int
    D: int
    F: int
    NA: int
    FF: int
    n_ent: int
    prec: int = 0   # 0 fp32, 1 bf16 MFMA operands (fp32 accumulate / LayerNorm / softmax / state)
    n_agents: int = 0  # mixer: agents (hidden tokens / qvals); 0 = n_ent (its state tokens)
    pos_func: int = 0  # mixer head positivity (_lib.POS_FUNCS; 3 = identity)
    pos_beta: float = 1.0

    def layout(self):
        return _layout_cached(self)

    @property
    def generic(self):
        """True when no tuned kernel instance exists: the runtime-shaped kernels run."""
        return bool(self.layout().generic)

    @property
    def instance(self):
        """Which kernels run this network: "exact" (MFMA instance compiled for its entity
        count), "runtime" (MFMA instance of a capacity class, entity count read at run
        time) or "generic" (runtime-shaped fp32 kernels) — include/t2omca.h."""
        if not hasattr(lib(), "t2o_layout_instance"):  # an older build under A/B timing (T2O_LIB)
            return "generic" if self.generic else "exact"
        return ("exact", "runtime", "generic")[int(lib().t2o_layout_instance(ctypes.byref(self.layout())))]

    @property
    def agents(self):
        return self.n_agents or self.n_ent

    @property
    def n_params(self):
        return int(lib().t2o_param_count(self.kind, self.E, self.H, self.D, self.F, self.NA, self.FF))


_LAYOUTS = {}


def _layout_cached(s):
    key = (s, _lib.force_generic())
    L = _LAYOUTS.get(key)
    if L is None:
        L = _lib.make_layout(s.kind, s.E, s.H, s.D, s.F, s.NA, s.FF, s.n_ent, s.prec, s.n_agents, s.pos_func,
                             s.pos_beta)
        _LAYOUTS[key] = L
    return L


def pack_params(shape: NetShape, params: torch.Tensor, out: torch.Tensor = None):
    """params (flat, reference state_dict order) -> folded kernel pack."""
    _dev(params)
    L = shape.layout()
    assert params.numel() == shape.n_params and params.is_contiguous()
    if out is None:
        out = torch.empty(L.pack_floats, device=params.device, dtype=torch.float32)
    check(lib().t2o_pack_params(ctypes.byref(L), ptr(params), ptr(out), stream_ptr()), "pack_params")
    return out


def unpack_grads(shape: NetShape, params, gpack, grad):
    """grad += unfold(gpack)   (grad in reference parameter order)."""
    _dev(params, gpack, grad)
    L = shape.layout()
    check(lib().t2o_unpack_grads(ctypes.byref(L), ptr(params), ptr(gpack), ptr(grad), stream_ptr()),
          "unpack_grads")
    return grad


def reduce_slabs(slabs, nslab, out):
    _dev(slabs, out)
    check(lib().t2o_reduce_slabs(ptr(slabs), int(nslab), out.numel(), ptr(out), stream_ptr()),
          "reduce_slabs")
    return out


def _p(t):
    """Device address of a tensor for an argument struct's pointer field (None -> NULL)."""
    return None if t is None else t.data_ptr()


def _mark(timer, tag):
    if timer is not None:
        timer(tag)


def agent_unroll_fwd(shape: NetShape, pack_on, obs, h0_on=None, pack_tg=None, h0_tg=None, timer=None,
                     hmid_on=None, steps=None, outs=None, launcher=False):
    """Unroll the agent over obs [B, T, A, n_ent*F] (any stride over B, T; inner
    [A, n_ent*F] contiguous).  Returns (q_on, h_on[, q_tg, h_tg]) with
    q [B, T, A, NA], h [B, T, A, E].  hmid_on: optional [B, T, D-1, A, E]
    output buffer for the inter-block activations (used by the backward).
    steps=(t0, t1): only those steps (t2o_agent_fwd_args.t0 / t1: t0 > 0 continues
    from h[t0 - 1]) into the given outs=(q_on, h_on, q_tg, h_tg)."""
    _dev(pack_on, obs, h0_on, pack_tg, h0_tg)
    B, T, A, nf = obs.shape
    assert obs.dtype == torch.float32 and nf == shape.n_ent * shape.F
    assert obs.stride(3) == 1 and obs.stride(2) == nf, "obs rows must be contiguous per timestep"
    L = shape.layout()
    dev = obs.device
    if outs is not None:
        q_on, h_on, q_tg, h_tg = outs
    else:
        q_on = torch.empty(B, T, A, shape.NA, device=dev)
        h_on = torch.empty(B, T, A, shape.E, device=dev)
        q_tg = h_tg = None
        if pack_tg is not None:
            q_tg = torch.empty_like(q_on)
            h_tg = torch.empty_like(h_on)
    for h0 in (h0_on, h0_tg):
        if h0 is not None:
            assert h0.is_contiguous() and h0.numel() == B * A * shape.E
    a = AgentFwdArgs(L=ctypes.pointer(L), pack_on=_p(pack_on), pack_tg=_p(pack_tg), obs=_p(obs),
                     obs_sb=obs.stride(0), obs_st=obs.stride(1), h0_on=_p(h0_on), h0_tg=_p(h0_tg), q_on=_p(q_on),
                     h_on=_p(h_on), hmid_on=_p(hmid_on), q_tg=_p(q_tg), h_tg=_p(h_tg), B=B, T=T, A=A)
    fn = lib().t2o_agent_unroll_fwd

    def go(t0, t1):
        a.t0, a.t1 = int(t0), int(t1)
        _mark(timer, "begin:agent_fwd")
        check(fn(ctypes.byref(a), stream_ptr()), "agent_unroll_fwd")
        _mark(timer, "end:agent_fwd")
    if launcher:  # go(t0, t1) per step range, the arguments converted once (pipelined learner)
        return go
    go(*(steps if steps is not None else (0, T)))
    if pack_tg is not None:
        return q_on, h_on, q_tg, h_tg
    return q_on, h_on


def tape_floats(shape: NetShape, tiles):
    """Backward tape workspace (floats) for `tiles` tiles of weight-gradient records
    (16 per tile; a one-tile mixer stores just its A+3 query rows)."""
    return int(lib().t2o_bwd_tape_floats(ctypes.byref(shape.layout()), int(tiles)))


def agent_tape_tiles(B, T, A, shape: NetShape = None):
    return T * ((B * A + 15) // 16)


def mixer_tape_tiles(B, T, A, shape: NetShape):
    """Weight-gradient tape tiles per block of a mixer BPTT over B episodes x T
    steps (include/t2omca.h t2o_bwd_tape_tiles: one tile of the A+3 query rows
    per (episode, step) when they fit 16 records; tuned multi-tile mixers store
    each block's query-row records as one compact stream cut into 16-record
    tiles, t2o_mixer.hip)."""
    n = int(lib().t2o_bwd_tape_tiles(ctypes.byref(shape.layout()), int(B), int(T), int(A)))
    if n < 0:
        raise ValueError(f"mixer_tape_tiles: bad shape B={B} T={T} A={A} for a mixer of {shape.agents} agents")
    return n


def _tape(shape, tiles, tape, device):
    n = tape_floats(shape, tiles)
    if tape is None or tape.numel() < n:
        tape = torch.empty(n, device=device)
    return tape


# The tape contraction runs one workgroup per slab (split-K over the tape's
# tiles).  A backward over a small replay batch fills few slabs (the mixer BPTT
# one per 1-4 episodes, the agent BPTT one per two 16-row tiles: 8 and 16 at
# configs[0]'s 32 episodes), so its contraction would stream the whole tape
# through those few workgroups; it gets at least CONTRACT_MIN_WG instead, the
# extra slabs zeroed first (they receive no BPTT flush; the contraction writes
# everything else of a slab itself).
CONTRACT_MIN_WG = 256


def mixer_work_floats(shape: NetShape, B, T):
    """Workspace floats of a decoupled multi-tile mixer backward (0 when it does not
    run decoupled at this batch: t2o_mixer_split)."""
    L = shape.layout()
    if int(lib().t2o_mixer_split(ctypes.byref(L), int(B))) != 1:
        return 0
    return max(0, int(lib().t2o_mixer_bwd_work_floats(ctypes.byref(L), int(B), int(T))))


def mixer_slab_count(B):
    """Slabs a mixer backward over B episodes needs (its BPTT's + the widened contraction's)."""
    return max(int(lib().t2o_mixer_bwd_max_slabs(B)), CONTRACT_MIN_WG)


def agent_slab_count(B, A):
    """Slabs an agent backward over B episodes of A agents needs."""
    return max(int(lib().t2o_agent_bwd_max_slabs(B, A)), CONTRACT_MIN_WG)


class DeferredContraction:
    """A backward call's weight-gradient tape, not yet contracted: call it (on the
    stream that should run the contraction + slab sum) for the compact gradient
    block, or hand two of them to tape_contract_pair."""

    def __init__(self, shape, pack, tape, tiles, slabs, nslab, timer, tag, fmt):
        self.shape, self.pack, self.tape, self.tiles = shape, pack, tape, tiles
        self.slabs, self.nslab, self.timer, self.tag, self.fmt = slabs, nslab, timer, tag, fmt

    def widen(self):
        """Raise the contraction's workgroup count to CONTRACT_MIN_WG where the slab
        buffer holds them (tuned layouts): zero the slabs past the BPTT's on the
        current stream.  Idempotent."""
        L = self.shape.layout()
        cap = self.slabs.numel() // L.grad_total
        nc = min(max(self.nslab, CONTRACT_MIN_WG), cap)
        if L.generic or nc <= self.nslab:
            return
        self.slabs[self.nslab * L.grad_total:nc * L.grad_total].zero_()
        self.nslab = nc

    def __call__(self):
        self.widen()
        return tape_contract(self.shape, self.pack, self.tape, self.tiles, self.slabs, self.nslab, self.timer,
                             self.tag, self.fmt)


def agent_unroll_bwd(shape: NetShape, pack, obs, h_seq, h0=None, gq=None, gchosen=None, actions=None,
                     gh=None, want_gh0=False, slabs=None, timer=None, hmid=None, tape=None, defer_contract=False,
                     steps=None, gcarry=None, launcher=False):
    """BPTT of agent_unroll_fwd over the first T = len(grads) steps.

    obs [B, >=T, A, nF]; h_seq [B, Ts>=T, A, E] (forward output); gq [B,T,A,NA],
    gchosen [B,T,A] + actions (int64 [B, >=T, A], a-stride 1), gh [B,T,A,E].
    Returns (gpack, gh0) with gpack the compact weight-gradient block (with
    defer_contract, a DeferredContraction instead).  steps=(t_lo, t_hi): only
    steps t_hi - 1 .. t_lo (t2o_agent_bwd_args.t_lo / t_hi; ranges from the last down
    on the same slabs / tape, gcarry [B*A, E] between them); the contraction is
    then always deferred (call it after the range that ends at step 0)."""
    _dev(pack, obs, h_seq, h0, gq, gchosen, actions, gh)
    B, _, A, _ = obs.shape
    T = next(t.shape[1] for t in (gq, gchosen, gh) if t is not None)
    L = shape.layout()
    for t in (gq, gchosen, gh):
        assert t is None or t.is_contiguous()
    assert h_seq.is_contiguous() and h_seq.shape[1] >= T
    act_sb = act_st = 0
    if gchosen is not None:
        assert actions is not None and actions.dtype == torch.int64 and actions.stride(2) == 1
        act_sb, act_st = actions.stride(0), actions.stride(1)
    nmax = int(lib().t2o_agent_bwd_max_slabs(B, A))
    if slabs is None or slabs.numel() < nmax * L.grad_total:
        nmax = agent_slab_count(B, A)
        slabs = torch.empty(nmax * L.grad_total, device=obs.device)
    gh0 = torch.empty(B, A, shape.E, device=obs.device) if want_gh0 else None
    tiles = agent_tape_tiles(B, T, A)
    tape = _tape(shape, tiles, tape, obs.device)
    nslab = ctypes.c_int32(0)
    a = AgentBwdArgs(L=ctypes.pointer(L), pack=_p(pack), obs=_p(obs), obs_sb=obs.stride(0), obs_st=obs.stride(1),
                     h0=_p(h0), h_seq=_p(h_seq), hmid=_p(hmid), h_ts=h_seq.shape[1], gq=_p(gq), gchosen=_p(gchosen),
                     actions=_p(actions), act_sb=act_sb, act_st=act_st, gh=_p(gh), gslabs=_p(slabs), max_slabs=nmax,
                     nslab=ctypes.pointer(nslab), tape=_p(tape), gh0=_p(gh0), gcarry=_p(gcarry), B=B, T=T, A=A)
    fn = lib().t2o_agent_unroll_bwd
    fmt = int(lib().t2o_agent_bwd_tape_format(ctypes.byref(L), int(hmid is not None)))

    def go(t_lo, t_hi):
        a.t_lo, a.t_hi = int(t_lo), int(t_hi)
        _mark(timer, "begin:agent_bwd")
        check(fn(ctypes.byref(a), stream_ptr()), "agent_unroll_bwd")
        _mark(timer, "end:agent_bwd")
        return DeferredContraction(shape, pack, tape, tiles, slabs, nslab.value, timer, "agent_dw", fmt)
    if launcher:  # go(t_lo, t_hi) per step range -> the (deferred) contraction
        return go, gh0
    dc = go(*(steps if steps is not None else (0, T)))
    return (dc if defer_contract or steps is not None else dc()), gh0


def _mstrides(t):
    return (t.stride(0), t.stride(1)) if t is not None else (0, 0)


def mixer_unroll_fwd(shape: NetShape, pack_on, states, hid_on, *, qmode_on=0, qv_on=None, q_on=None,
                     actions=None, avail=None, hw0_on=None, T_on=None,
                     pack_tg=None, hid_tg=None, qmode_tg=2, qv_tg=None, q_tg=None, hw0_tg=None,
                     T_tg=None, want_xout=True, timer=None, phase=0, steps=None, outs=None, launcher=False):
    """Mixer unroll (see include/t2omca.h).  states [B, >=T, n_ent*F];
    hid_* [B, >=T, A, E] (contiguous inner [A, E]); q_on/q_tg [B, q_ts, A, NA]
    contiguous; actions int64 [B, >=T, A]; avail int32 [B, >=T, A, NA].
    Returns dict of outputs per network: y [B,T], hw [B,T,3,E], qv [B,T,A], xout.
    phase 1 / 2 (a decoupled mixer, t2o_mixer_fwd_args.phase): the recurrence
    over steps=(t0, t1) / the parallel rows, into the given outs=(o_on, o_tg)."""
    _dev(pack_on, states, hid_on, qv_on, q_on, hw0_on, pack_tg, hid_tg, qv_tg, q_tg, hw0_tg)
    B = states.shape[0]
    A, E = hid_on.shape[2], shape.E
    if A != shape.agents:
        raise ValueError(f"mixer_unroll_fwd: hidden states carry {A} agents, the mixer was built for {shape.agents}")
    L = shape.layout()
    dev = states.device
    T_on = T_on or (qv_on.shape[1] if qv_on is not None else hid_on.shape[1])
    assert hid_on.stride(3) == 1 and hid_on.stride(2) == E and states.stride(2) == 1
    if hid_tg is not None:
        assert hid_tg.stride(0) == hid_on.stride(0) and hid_tg.stride(1) == hid_on.stride(1)
    q_ts = q_on.shape[1] if q_on is not None else 0
    for q in (q_on, q_tg):
        assert q is None or (q.is_contiguous() and q.shape[1] == q_ts)
    if actions is not None:
        assert actions.dtype == torch.int64 and actions.stride(2) == 1
    if avail is not None:
        assert avail.dtype == torch.int32 and avail.stride(3) == 1 and avail.stride(2) == avail.shape[3]

    def alloc(T, bwd):
        # xout / xmid only feed the backward: the target network skips them
        return dict(y=torch.empty(B, T, device=dev), hw=torch.empty(B, T, 3, E, device=dev),
                    qv=torch.empty(B, T, A, device=dev),
                    xout=torch.empty(B, T, A + 3, E, device=dev) if bwd else None,
                    xmid=torch.empty(B, T, shape.D - 1, A + 3, E, device=dev) if (bwd and shape.D > 1) else None)

    # a multi-tile mixer at a small batch runs decoupled (t2o_mixer_split.hip): its
    # parallel kernel reads the recurrent kernel's window rows back from xout
    split = bool(lib().t2o_mixer_split(ctypes.byref(L), B) == 1)
    given = outs
    if given is not None:
        o_on, o_tg = given
        T_tg = T_tg or (hid_tg.shape[1] if hid_tg is not None else None)
    else:
        o_on = alloc(T_on, want_xout or split)
        o_tg = None
        if pack_tg is not None:
            T_tg = T_tg or hid_tg.shape[1]
            o_tg = alloc(T_tg, False)
            if split:
                o_tg["xout"] = torch.empty(B, T_tg, A + 3, E, device=dev)
    n_actions = q_on.shape[3] if q_on is not None else 0
    act_sb, act_st = _mstrides(actions)
    av_sb, av_st = _mstrides(avail)
    g = lambda d, k: _p(d[k]) if d is not None else None  # noqa: E731
    a = MixerFwdArgs(L=ctypes.pointer(L), pack_on=_p(pack_on), pack_tg=_p(pack_tg), states=_p(states),
                     st_sb=states.stride(0), st_st=states.stride(1), hid_on=_p(hid_on), hid_tg=_p(hid_tg),
                     hid_sb=hid_on.stride(0), hid_st=hid_on.stride(1), hw0_on=_p(hw0_on), hw0_tg=_p(hw0_tg),
                     qmode_on=qmode_on, qmode_tg=qmode_tg, qv_on=_p(qv_on), qv_tg=_p(qv_tg), q_on=_p(q_on),
                     q_tg=_p(q_tg), q_ts=q_ts, n_actions=n_actions, actions=_p(actions), act_sb=act_sb,
                     act_st=act_st, avail=_p(avail), av_sb=av_sb, av_st=av_st,
                     y_on=g(o_on, "y"), hw_on=g(o_on, "hw"), qvo_on=g(o_on, "qv"), xout_on=g(o_on, "xout"),
                     xmid_on=g(o_on, "xmid"), y_tg=g(o_tg, "y"), hw_tg=g(o_tg, "hw"), qvo_tg=g(o_tg, "qv"),
                     xout_tg=g(o_tg, "xout"), xmid_tg=g(o_tg, "xmid"), B=B, T_on=T_on, T_tg=T_tg or 0)
    fn = lib().t2o_mixer_unroll_fwd

    def go(phase, t0=0, t1=0):
        a.phase, a.t0, a.t1 = int(phase), int(t0), int(t1)
        _mark(timer, "begin:mixer_fwd")
        check(fn(ctypes.byref(a), stream_ptr()), "mixer_unroll_fwd")
        _mark(timer, "end:mixer_fwd")
    if launcher:  # go(phase, t0, t1) per phase / step range (pipelined learner)
        return go
    go(int(phase), *(steps if steps is not None else (0, 0)))
    return (o_on, o_tg) if pack_tg is not None else o_on


def tape_contract(shape: NetShape, pack, tape, tiles, slabs, nslab, timer=None, tag="dw", fmt=0):
    """Fill the M/N/W1/W2 regions of the backward's slabs from its tape (pack =
    the pack the backward used; fmt = the tape's record format,
    t2o_agent_bwd_tape_format), then sum the slabs.  Returns the compact
    gradient block (on the current stream)."""
    L = shape.layout()
    _mark(timer, "begin:" + tag)
    a = TapeArgs(L=ctypes.pointer(L), pack=_p(pack), tape=_p(tape), tiles=int(tiles), gslabs=_p(slabs),
                 nslab=int(nslab), rec_format=int(fmt))
    check(lib().t2o_bwd_tape_contract(ctypes.byref(a), None, stream_ptr()), "bwd_tape_contract")
    _mark(timer, "end:" + tag)
    gpack = torch.empty(L.grad_total, device=slabs.device)
    reduce_slabs(slabs, nslab, gpack)
    return gpack


def tape_contract_pair(dm: DeferredContraction, da: DeferredContraction, timer=None):
    """Both backwards' tape contractions in one launch (t2o_bwd_tape_contract with two tapes;
    dm the mixer's, da the agent's), then each slab sum.  Returns (gpack_m, gpack_a)."""
    Lm, La = dm.shape.layout(), da.shape.layout()
    dm.widen()
    da.widen()
    _mark(timer, "begin:dw_pair")
    am = TapeArgs(L=ctypes.pointer(Lm), pack=_p(dm.pack), tape=_p(dm.tape), tiles=int(dm.tiles), gslabs=_p(dm.slabs),
                  nslab=int(dm.nslab), rec_format=0)
    aa = TapeArgs(L=ctypes.pointer(La), pack=_p(da.pack), tape=_p(da.tape), tiles=int(da.tiles), gslabs=_p(da.slabs),
                  nslab=int(da.nslab), rec_format=int(da.fmt))
    check(lib().t2o_bwd_tape_contract(ctypes.byref(am), ctypes.byref(aa), stream_ptr()), "bwd_tape_contract (pair)")
    _mark(timer, "end:dw_pair")
    out = []
    for d, L in ((dm, Lm), (da, La)):
        g = torch.empty(L.grad_total, device=d.slabs.device)
        reduce_slabs(d.slabs, d.nslab, g)
        out.append(g)
    return out[0], out[1]


def mixer_unroll_bwd(shape: NetShape, pack, states, hid, fwd, gy, hw0=None, ghw_ext=None,
                     want_ghw0=False, slabs=None, timer=None, tape=None, defer_contract=False, work=None,
                     phase=0, steps=None, carry=None, outs=None, launcher=False):
    """BPTT of mixer_unroll_fwd (one network, `fwd` = its output dict).
    Returns (gpack, gqv [B,T,A], ghid [B,T,A,E], ghw0 or None).  With
    defer_contract the first item is instead a zero-argument callable that runs
    the tape contraction + slab sum (on whatever stream is current when called)
    and returns gpack.  work: optional float buffer for the decoupled multi-tile
    mixer (t2o_mixer_bwd_work_floats; allocated here when needed and not given).
    phase 1 / 2 (a decoupled mixer, t2o_mixer_bwd_args.phase): the parallel
    part / the recurrence over steps=(t_lo, t_hi) (ranges from the last down,
    carry [B, 3, E] between them) into outs=(gqv, ghid), with the same slabs,
    tape and work every call; the contraction is then always deferred."""
    _dev(pack, states, hid, gy, hw0, ghw_ext)
    B, T = gy.shape
    A, E = hid.shape[2], shape.E
    if A != shape.agents:
        raise ValueError(f"mixer_unroll_bwd: hidden states carry {A} agents, the mixer was built for {shape.agents}")
    L = shape.layout()
    dev = gy.device
    assert gy.is_contiguous() and fwd["xout"] is not None
    nmax = int(lib().t2o_mixer_bwd_max_slabs(B))
    if slabs is None or slabs.numel() < nmax * L.grad_total:
        nmax = mixer_slab_count(B)
        slabs = torch.empty(nmax * L.grad_total, device=dev)
    if outs is not None:
        gqv, ghid = outs
    else:
        gqv = torch.empty(B, T, A, device=dev)
        ghid = torch.empty(B, T, A, E, device=dev)
    ghw0 = torch.empty(B, 3, E, device=dev) if want_ghw0 else None
    tiles = mixer_tape_tiles(B, T, A, shape)
    tape = _tape(shape, tiles, tape, dev)
    nslab = ctypes.c_int32(0)
    nwork = mixer_work_floats(shape, B, T)
    if nwork and (work is None or work.numel() < nwork):
        work = torch.empty(nwork, device=dev)
    a = MixerBwdArgs(L=ctypes.pointer(L), pack=_p(pack), states=_p(states), st_sb=states.stride(0),
                     st_st=states.stride(1), hid=_p(hid), hid_sb=hid.stride(0), hid_st=hid.stride(1), hw0=_p(hw0),
                     qv=_p(fwd["qv"]), hw=_p(fwd["hw"]), xout=_p(fwd["xout"]), xmid=_p(fwd.get("xmid")), gy=_p(gy),
                     ghw_ext=_p(ghw_ext), gqv=_p(gqv), ghid=_p(ghid), ghw0=_p(ghw0), gslabs=_p(slabs), max_slabs=nmax,
                     nslab=ctypes.pointer(nslab), tape=_p(tape), work=_p(work) if nwork else None, work_floats=nwork,
                     ghw_carry=_p(carry), B=B, T=T)
    fn = lib().t2o_mixer_unroll_bwd

    def go(phase, t_lo=0, t_hi=0):
        a.phase, a.t_lo, a.t_hi = int(phase), int(t_lo), int(t_hi)
        _mark(timer, "begin:mixer_bwd")
        check(fn(ctypes.byref(a), stream_ptr()), "mixer_unroll_bwd")
        _mark(timer, "end:mixer_bwd")
        return DeferredContraction(shape, pack, tape, tiles, slabs, nslab.value, timer, "mixer_dw", 0)
    if launcher:  # go(phase, t_lo, t_hi) per phase / step range -> the (deferred) contraction
        return go
    contract = go(int(phase), *(steps if steps is not None else (0, 0)))
    return (contract if defer_contract or phase else contract()), gqv, ghid, ghw0


# TD loss mask element types (include/t2omca.h T2O_DT_*)
_MASK_DT = {torch.float32: 0, torch.uint8: 1, torch.bool: 1, torch.int32: 2, torch.int64: 3}


def _mask_dtype(t):
    if t is None:
        return 0
    if t.dtype not in _MASK_DT:
        raise TypeError(f"td_loss: unsupported mask dtype {t.dtype}")
    return _MASK_DT[t.dtype]


TD_ALGOS = {"auto": 0, "sequential": 1, "wave": 2}  # include/t2omca.h T2O_TD_*


def td_loss(qtot, qtot_tgt, reward, terminated=None, filled=None, per_weight=None, gamma=0.99,
            td_lambda=0.6, mask_sum=0.0, algo="auto", mask_sum_acc=None):
    """TD(λ) targets / loss / grads / priorities (PyMARL2 NQLearner contract).
    qtot [B,T], qtot_tgt [B,T+1]; reward [B, >=T] float view; terminated / filled
    [B, >=T] views in float32, uint8/bool, int32 or int64 (read in place).
    algo: "sequential" (the reference's backward order, one thread per episode),
    "wave" (one wave per episode, suffix scan) or "auto" (the library default).
    mask_sum_acc: optional 1-float device tensor that receives += Σ mask.
    Returns dict(gq [B,T], targets [B,T], prio [B], loss [2])."""
    _dev(qtot, qtot_tgt, reward, per_weight, mask_sum_acc)
    for m in (terminated, filled):  # any mask dtype of _MASK_DT, device-resident
        if m is not None and not m.is_cuda:
            raise RuntimeError("t2omca_amd ops need HIP-device tensors (no CPU fallback)")
        _mask_dtype(m)
    B, T = qtot.shape
    dev = qtot.device
    assert qtot.is_contiguous() and qtot_tgt.is_contiguous() and qtot_tgt.shape[1] == T + 1
    out = dict(gq=torch.empty(B, T, device=dev), targets=torch.empty(B, T, device=dev),
               prio=torch.empty(B, device=dev), loss=torch.empty(2, device=dev))
    rs, ts, fs = _mstrides(reward), _mstrides(terminated), _mstrides(filled)
    a = TDArgs(qtot=_p(qtot), qtot_tgt=_p(qtot_tgt), reward=_p(reward), rw_sb=rs[0], rw_st=rs[1],
               term=_p(terminated), tm_sb=ts[0], tm_st=ts[1], filled=_p(filled), fl_sb=fs[0], fl_st=fs[1],
               per_weight=_p(per_weight), gq=_p(out["gq"]), targets=_p(out["targets"]), prio=_p(out["prio"]),
               loss=_p(out["loss"]), mask_sum_acc=_p(mask_sum_acc), gamma=float(gamma), td_lambda=float(td_lambda),
               mask_sum=float(mask_sum), term_dtype=_mask_dtype(terminated), filled_dtype=_mask_dtype(filled),
               algo=TD_ALGOS[algo], B=B, T=T)
    check(lib().t2o_td_loss(ctypes.byref(a), stream_ptr()), "td_loss")
    return out


def adam_step(params, grads, exp_avg, exp_avg_sq, step, *, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
              weight_decay=0.0, max_grad_norm=10.0, workspace=None, grad_div=None, grad_norm_out=None):
    """In-place clip_grad_norm_ + Adam on flat fp32 buffers (grads divided by the
    device scalar grad_div first, if given)."""
    _dev(params, grads, exp_avg, exp_avg_sq, workspace, grad_div, grad_norm_out)
    n = params.numel()
    if workspace is None:
        workspace = torch.empty(int(lib().t2o_adam_workspace_floats()), device=params.device)
    check(lib().t2o_adam_step(ptr(params), ptr(grads), ptr(exp_avg), ptr(exp_avg_sq), ptr(workspace), n,
                              float(lr), float(betas[0]), float(betas[1]), float(eps),
                              float(weight_decay), float(max_grad_norm), int(step), ptr(grad_div),
                              ptr(grad_norm_out),
                              stream_ptr()), "adam_step")


def select_actions(q, avail, epsilon=0.0, seed=0, counter=0, out=None):
    """ε-greedy actions (include/t2omca.h t2o_select_actions): q f32 [..., NA] and
    avail i32 [..., NA], dense; returns int64 [...] (or writes `out`)."""
    _dev(q)
    if avail.dtype != torch.int32 or not avail.is_cuda:
        raise TypeError("avail must be an int32 HIP-device tensor")
    NA = q.shape[-1]
    assert q.is_contiguous() and avail.is_contiguous() and avail.shape == q.shape
    rows = q.numel() // NA
    if out is None:
        out = torch.empty(q.shape[:-1], dtype=torch.int64, device=q.device)
    assert out.is_contiguous() and out.numel() == rows and out.dtype == torch.int64
    check(lib().t2o_select_actions(ptr(q), ptr(avail), ptr(out), rows, NA, float(epsilon),
                                   ctypes.c_uint64(int(seed) & ((1 << 64) - 1)), int(counter), stream_ptr()),
          "select_actions")
    return out


def obs_expand(wire, snap_n, snap, out=None, out64=None):
    """Dense normalised obs from the compact wire format (SURVEY.md §8 f3,
    include/t2omca.h t2o_obs_expand).  wire int32 [B, T1, A, 4] (episode / step
    strides free, agent rows dense), snap_n int64 [B], snap f64 [B, 2, 9A];
    returns f32 [B, T1, A, 9A] (or writes `out`, any episode / step strides with
    dense steps); out64 optionally receives the fp64 values (dense)."""
    for t in (wire, snap_n, snap, out, out64):
        if t is not None and not t.is_cuda:
            raise RuntimeError("obs_expand needs HIP-device tensors (no CPU fallback)")
    if wire.dtype != torch.int32 or snap_n.dtype != torch.int64 or snap.dtype != torch.float64:
        raise TypeError("obs_expand: wire int32, snap_n int64, snap float64")
    B, T1, A, four = wire.shape
    assert four == 4 and wire.stride(3) == 1 and wire.stride(2) == 4
    assert snap_n.shape == (B,) and snap.shape == (B, 2, 9 * A) and snap.is_contiguous() and snap_n.is_contiguous()
    if out is None:
        out = torch.empty(B, T1, A, 9 * A, device=wire.device)
    assert out.dtype == torch.float32 and out.shape == (B, T1, A, 9 * A)
    assert out.stride(3) == 1 and out.stride(2) == 9 * A
    if out64 is not None:
        assert out64.dtype == torch.float64 and out64.shape == out.shape and out64.is_contiguous()
    check(lib().t2o_obs_expand(ptr(wire), wire.stride(0), wire.stride(1), ptr(snap_n), ptr(snap), ptr(out),
                               out.stride(0), out.stride(1), ptr(out64), B, T1, A, stream_ptr(wire.device)),
          "obs_expand")
    return out
