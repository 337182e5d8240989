"""ctypes binding of the C-ABI library (include/t2omca.h).

The library is the product: there is no CPU or eager-PyTorch fallback.  If
libt2omca.so is missing, importing the compute entry points raises.
"""
import ctypes
import os

import torch

from .build import LIB

MAX_DEPTH = 4
ABI_VERSION = 6  # include/t2omca.h T2O_ABI_VERSION this binding mirrors
_I64x = ctypes.c_int64 * MAX_DEPTH


class Layout(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_int32) for n in ("kind", "E", "H", "D", "F", "NA", "FF", "n_ent", "prec",
                                                "generic")] +
                [(n, ctypes.c_int64) for n in ("WeT", "We", "be", "Wo", "bo", "WoT")] +
                [(n, _I64x) for n in ("M", "MT", "N", "NT", "bu", "g1", "n1", "W1", "W1T", "c1",
                                      "W2", "W2T", "c2", "g2", "n2")] +
                [(n, ctypes.c_int64) for n in ("fwd_total", "total", "grad_total", "vec_lo", "pack_floats")] +
                [("n_agents", ctypes.c_int32), ("pos_func", ctypes.c_int32), ("pos_beta", ctypes.c_float),
                 ("reserved_", ctypes.c_int32)])


_P, _I32, _I64, _F = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
_LP = ctypes.POINTER(Layout)


def _fields(spec):
    """'name:type, ...' (types P pointer, I int32, J int64, F float, L layout*) -> ctypes _fields_."""
    ty = {"P": _P, "I": _I32, "J": _I64, "F": _F, "L": _LP, "IP": ctypes.POINTER(ctypes.c_int32)}
    out = []
    for item in spec.split(","):
        n, t = item.strip().split(":")
        out.append((n, ty[t]))
    return out


class _Args(ctypes.Structure):
    """Argument structs of include/t2omca.h: fields by name (unset pointers NULL, ints 0)."""

    def __init__(self, **kw):
        super().__init__()
        for k, v in kw.items():
            setattr(self, k, v)

    def __setattr__(self, k, v):
        if k not in self._names:
            raise AttributeError(f"{type(self).__name__} has no field {k!r}")
        super().__setattr__(k, v)


def _args_class(name, which, spec):
    f = _fields(spec)
    return type(name, (_Args,), {"_fields_": f, "_names": {n for n, _ in f}, "WHICH": which})


# field order and types exactly as include/t2omca.h declares them (t2o_args_sizeof checks the size)
AgentFwdArgs = _args_class("AgentFwdArgs", 0, """L:L, pack_on:P, pack_tg:P, obs:P, obs_sb:J, obs_st:J, h0_on:P,
    h0_tg:P, q_on:P, h_on:P, hmid_on:P, q_tg:P, h_tg:P, hmid_tg:P, B:I, T:I, A:I, t0:I, t1:I""")
AgentBwdArgs = _args_class("AgentBwdArgs", 1, """L:L, pack:P, obs:P, obs_sb:J, obs_st:J, h0:P, h_seq:P, hmid:P,
    h_ts:I, gq:P, gchosen:P, actions:P, act_sb:J, act_st:J, gh:P, gslabs:P, max_slabs:I, nslab:IP, tape:P, gh0:P,
    gcarry:P, B:I, T:I, A:I, t_lo:I, t_hi:I""")
MixerFwdArgs = _args_class("MixerFwdArgs", 2, """L:L, pack_on:P, pack_tg:P, states:P, st_sb:J, st_st:J, hid_on:P,
    hid_tg:P, hid_sb:J, hid_st:J, hw0_on:P, hw0_tg:P, qmode_on:I, qmode_tg:I, qv_on:P, qv_tg:P, q_on:P, q_tg:P,
    q_ts:I, n_actions:I, actions:P, act_sb:J, act_st:J, avail:P, av_sb:J, av_st:J, y_on:P, hw_on:P, qvo_on:P,
    xout_on:P, xmid_on:P, y_tg:P, hw_tg:P, qvo_tg:P, xout_tg:P, xmid_tg:P, B:I, T_on:I, T_tg:I, phase:I, t0:I,
    t1:I""")
MixerBwdArgs = _args_class("MixerBwdArgs", 3, """L:L, pack:P, states:P, st_sb:J, st_st:J, hid:P, hid_sb:J,
    hid_st:J, hw0:P, qv:P, hw:P, xout:P, xmid:P, gy:P, ghw_ext:P, gqv:P, ghid:P, ghw0:P, gslabs:P, max_slabs:I,
    nslab:IP, tape:P, work:P, work_floats:J, ghw_carry:P, B:I, T:I, phase:I, t_lo:I, t_hi:I""")
TapeArgs = _args_class("TapeArgs", 4, "L:L, pack:P, tape:P, tiles:J, gslabs:P, nslab:I, rec_format:I")
TDArgs = _args_class("TDArgs", 5, """qtot:P, qtot_tgt:P, reward:P, rw_sb:J, rw_st:J, term:P, tm_sb:J, tm_st:J,
    filled:P, fl_sb:J, fl_st:J, per_weight:P, gq:P, targets:P, prio:P, loss:P, mask_sum_acc:P, gamma:F,
    td_lambda:F, mask_sum:F, term_dtype:I, filled_dtype:I, algo:I, B:I, T:I""")
ARGS_STRUCTS = (AgentFwdArgs, AgentBwdArgs, MixerFwdArgs, MixerBwdArgs, TapeArgs, TDArgs)


# mixer head positivity functions (include/t2omca.h T2O_POS_*; n_transf_mixer.py:95-103)
POS_FUNCS = {"abs": 0, "softplus": 1, "quadratic": 2}  # anything else: identity (3)
LAYOUT_FORCE_GENERIC = 1


EXPORTS = {
    # name: (restype, argtypes)
    "t2o_layout_init": (ctypes.c_int, [ctypes.POINTER(Layout)] + [ctypes.c_int] * 9),
    "t2o_layout_init_ex": (ctypes.c_int, [ctypes.POINTER(Layout)] + [ctypes.c_int] * 11 + [ctypes.c_float,
                                                                                       ctypes.c_int]),
    "t2o_param_count": (ctypes.c_int64, [ctypes.c_int] * 7),
    "t2o_layout_sizeof": (ctypes.c_int, []),
    "t2o_layout_instance": (ctypes.c_int, [ctypes.POINTER(Layout)]),
    "t2o_pack_params": (ctypes.c_int, [ctypes.POINTER(Layout), ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p]),
    "t2o_unpack_grads": (ctypes.c_int, [ctypes.POINTER(Layout), ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "t2o_reduce_slabs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "t2o_agent_unroll_fwd": (ctypes.c_int, [ctypes.POINTER(AgentFwdArgs), ctypes.c_void_p]),
    "t2o_agent_unroll_bwd": (ctypes.c_int, [ctypes.POINTER(AgentBwdArgs), ctypes.c_void_p]),
    "t2o_agent_bwd_max_slabs": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "t2o_mixer_unroll_fwd": (ctypes.c_int, [ctypes.POINTER(MixerFwdArgs), ctypes.c_void_p]),
    "t2o_mixer_unroll_bwd": (ctypes.c_int, [ctypes.POINTER(MixerBwdArgs), ctypes.c_void_p]),
    "t2o_mixer_bwd_work_floats": (ctypes.c_int64, [ctypes.POINTER(Layout), ctypes.c_int, ctypes.c_int]),
    "t2o_mixer_split": (ctypes.c_int, [ctypes.POINTER(Layout), ctypes.c_int]),
    "t2o_mixer_bwd_max_slabs": (ctypes.c_int, [ctypes.c_int]),
    "t2o_bwd_tape_floats": (ctypes.c_int64, [ctypes.POINTER(Layout), ctypes.c_int64]),
    "t2o_bwd_tape_tiles": (ctypes.c_int64, [ctypes.POINTER(Layout), ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "t2o_bwd_tape_contract": (ctypes.c_int, [ctypes.POINTER(TapeArgs), ctypes.POINTER(TapeArgs), ctypes.c_void_p]),
    "t2o_agent_bwd_tape_format": (ctypes.c_int, [ctypes.POINTER(Layout), ctypes.c_int]),
    "t2o_agent_bwd_ranges": (ctypes.c_int, [ctypes.POINTER(Layout), ctypes.c_int]),
    "t2o_td_loss": (ctypes.c_int, [ctypes.POINTER(TDArgs), ctypes.c_void_p]),
    "t2o_args_sizeof": (ctypes.c_int, [ctypes.c_int]),
    "t2o_abi_version": (ctypes.c_int, []),
    "t2o_adam_step": (ctypes.c_int, [ctypes.c_void_p] * 5 + [ctypes.c_int64] + [ctypes.c_double] * 3 +
                      [ctypes.c_float] * 3 + [ctypes.c_int64] + [ctypes.c_void_p] * 3),
    "t2o_adam_workspace_floats": (ctypes.c_int, []),
    "t2o_probe_lane_ops": (ctypes.c_int, [ctypes.c_void_p] * 3),
    "t2o_probe_scatter_ops": (ctypes.c_int, [ctypes.c_void_p] * 3),
    "t2o_probe_xdl_hazards": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "t2o_probe_posf": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "t2o_bf_swz": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "t2o_env_run": (ctypes.c_int, [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int64] +
                    [ctypes.c_int] * 6 + [ctypes.c_uint64, ctypes.c_void_p]),
    "t2o_env_run_ex": (ctypes.c_int, [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p,
                                                                                ctypes.c_int64] +
                       [ctypes.c_int] * 6 + [ctypes.c_uint64, ctypes.c_void_p]),
    "t2o_obs_expand": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_void_p]),
    "t2o_per_workspace_doubles": (ctypes.c_int64, [ctypes.c_int64]),
    "t2o_per_sample": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                      ctypes.c_uint64, ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "t2o_per_update": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_float, ctypes.c_float,
                                                              ctypes.c_void_p, ctypes.c_void_p]),
    "t2o_gather_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]),
    "t2o_select_actions": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                                                 ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p]),
}

# exports only tests / tools call (never on the product path), and the newest
# reporting export: an older build loaded under A/B timing (T2O_LIB) may lack them
_DIAGNOSTIC = {"t2o_bf_swz", "t2o_probe_lane_ops", "t2o_probe_scatter_ops", "t2o_probe_posf", "t2o_probe_xdl_hazards",
               "t2o_layout_instance",
               "t2o_abi_version"}

_lib = None


def lib():
    """Load libt2omca.so (raises if it has not been built).  T2O_LIB overrides the
    path (A/B timing of two builds on one box)."""
    global _lib
    if _lib is None:
        path = os.environ.get("T2O_LIB", LIB)
        if not os.path.exists(path):
            raise RuntimeError(f"t2omca_amd: {path} not built; run `python -m t2omca_amd.build` "
                               "(there is no CPU fallback)")
        h = ctypes.CDLL(path)
        for name, (res, args) in EXPORTS.items():
            if name in _DIAGNOSTIC and path != LIB and not hasattr(h, name):
                continue  # an older build under A/B (T2O_LIB) may lack a diagnostic export
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if hasattr(h, "t2o_abi_version") and h.t2o_abi_version() != ABI_VERSION and path == LIB:
            raise RuntimeError(f"t2omca_amd: {path} has C-ABI version {h.t2o_abi_version()}, this binding "
                               f"mirrors include/t2omca.h version {ABI_VERSION}; rebuild the library")
        for cls in ARGS_STRUCTS:  # the mirrors of the argument structs must match the library's
            if h.t2o_args_sizeof(cls.WHICH) != ctypes.sizeof(cls):
                raise RuntimeError(f"t2omca_amd: {cls.__name__} is {ctypes.sizeof(cls)} bytes here, "
                                   f"{h.t2o_args_sizeof(cls.WHICH)} in {path}; rebuild the library")
        _lib = h
    return _lib


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"t2omca_amd: {what} failed with status {rc}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def force_generic():
    """T2O_GENERIC=1 lays every network out for the runtime-shaped kernels, tuned
    shapes included (cross-checks of the generic path against the tuned one)."""
    return os.environ.get("T2O_GENERIC", "0") == "1"


def make_layout(kind, E, H, D, F, NA, FF, n_ent, prec=0, n_agents=0, pos_func=0, pos_beta=1.0, flags=None):
    if flags is None:
        flags = LAYOUT_FORCE_GENERIC if force_generic() else 0
    L = Layout()
    check(lib().t2o_layout_init_ex(ctypes.byref(L), kind, E, H, D, F, NA, FF, n_ent, prec, n_agents, pos_func,
                                   float(pos_beta), flags), "t2o_layout_init_ex")
    return L
