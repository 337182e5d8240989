"""Thin torch-tensor wrappers over the C-ABI entry points (include/t2omca.h).

Every function checks device/dtype/contiguity on the host, then launches on
the current HIP stream.  There is no CPU path: CPU tensors raise.
"""
import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr

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

    def layout(self):
        return _layout_cached(self)

    @property
    def n_params(self):
        return int(lib().t2o_param_count(self.kind, self.E, self.H, self.D, self.F, self.NA, self.FF))


_LAYOUTS = {}


def _layout_cached(s):
    L = _LAYOUTS.get(s)
    if L is None:
        L = _lib.make_layout(s.kind, s.E, s.H, s.D, s.F, s.NA, s.FF, s.n_ent)
        _LAYOUTS[s] = L
    return L


def pack_params(shape: NetShape, params: torch.Tensor, out: torch.Tensor = None):
    """params (flat, reference state_dict order) -> folded kernel pack."""
    _dev(params)
    L = shape.layout()
    assert params.numel() == shape.n_params and params.is_contiguous()
    if out is None:
        out = torch.empty(L.total, device=params.device, dtype=torch.float32)
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


def agent_unroll_fwd(shape: NetShape, pack_on, obs, h0_on=None, pack_tg=None, h0_tg=None):
    """Unroll the agent over obs [B, T, A, n_ent*F] (any stride over B, T; inner
    [A, n_ent*F] contiguous).  Returns (q_on, h_on[, q_tg, h_tg]) with
    q [B, T, A, NA], h [B, T, A, E]."""
    _dev(pack_on, obs, h0_on, pack_tg, h0_tg)
    B, T, A, nf = obs.shape
    assert obs.dtype == torch.float32 and nf == shape.n_ent * shape.F
    assert obs.stride(3) == 1 and obs.stride(2) == nf, "obs rows must be contiguous per timestep"
    L = shape.layout()
    dev = obs.device
    q_on = torch.empty(B, T, A, shape.NA, device=dev)
    h_on = torch.empty(B, T, A, shape.E, device=dev)
    q_tg = h_tg = None
    if pack_tg is not None:
        q_tg = torch.empty_like(q_on)
        h_tg = torch.empty_like(h_on)
    for h0 in (h0_on, h0_tg):
        if h0 is not None:
            assert h0.is_contiguous() and h0.numel() == B * A * shape.E
    check(lib().t2o_agent_unroll_fwd(ctypes.byref(L), ptr(pack_on), ptr(pack_tg), ptr(obs),
                                     obs.stride(0), obs.stride(1), ptr(h0_on), ptr(h0_tg),
                                     ptr(q_on), ptr(h_on), ptr(q_tg), ptr(h_tg), B, T, A,
                                     stream_ptr()), "agent_unroll_fwd")
    if pack_tg is not None:
        return q_on, h_on, q_tg, h_tg
    return q_on, h_on


def agent_unroll_bwd(shape: NetShape, pack, obs, h_seq, h0=None, gq=None, gchosen=None, actions=None,
                     gh=None, want_gh0=False, slabs=None):
    """BPTT of agent_unroll_fwd over the first T = len(grads) steps.

    obs [B, >=T, A, nF]; h_seq [B, Ts>=T, A, E] (forward output); gq [B,T,A,NA],
    gchosen [B,T,A] + actions (int64 [B, >=T, A], a-stride 1), gh [B,T,A,E].
    Returns (gpack, gh0) with gpack the compact weight-gradient block."""
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
        slabs = torch.empty(nmax * L.grad_total, device=obs.device)
    gh0 = torch.empty(B, A, shape.E, device=obs.device) if want_gh0 else None
    nslab = ctypes.c_int(0)
    check(lib().t2o_agent_unroll_bwd(ctypes.byref(L), ptr(pack), ptr(obs), obs.stride(0), obs.stride(1),
                                     ptr(h0), ptr(h_seq), h_seq.shape[1], ptr(gq), ptr(gchosen),
                                     ptr(actions), act_sb, act_st, ptr(gh), ptr(slabs), nmax,
                                     ctypes.byref(nslab), ptr(gh0), B, T, A, stream_ptr()),
          "agent_unroll_bwd")
    gpack = torch.empty(L.grad_total, device=obs.device)
    reduce_slabs(slabs, nslab.value, gpack)
    return gpack, gh0
