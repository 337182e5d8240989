"""Shared helpers for the -m gpu parity tests (GPU kernels vs the CPU oracle)."""
import os

import numpy as np
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# golden fixtures of the tuned kernel shapes (make_golden.CONFIGS); the EXTENDED
# ones (other shapes / options) are exercised by tests/test_gpu_generic.py
TUNED_TAGS = ("a3_e16_h2_d1", "a8_e32_h3_d2", "a16_e32_h3_d2")


def tuned_fixtures(kind, tags=TUNED_TAGS):
    return [os.path.join(GOLD, f"{kind}_{t}.npz") for t in tags]


def flat_from_npz(z):
    """Reference-order flat parameter vector from a golden fixture."""
    keys = [k for k in z.files if k.startswith("param/")]
    return torch.cat([torch.from_numpy(z[k]).reshape(-1).float() for k in keys])


def flat_from_dict(p):
    return torch.cat([v.reshape(-1).float() for v in p.values()])


def normwise(a, b):
    """max|a-b| / max|b|  (the parity metric of SURVEY.md §8 c)."""
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("gpu-marked test needs a HIP device")
    from t2omca_amd import _lib
    _lib.lib()


# A tie the GPU resolved the other way must lie within rounding of 0: its fp64
# pre-activation within TIE_ULPS fp32 ulps (2^-24 relative) of the row's rounding
# scale Σ_e |W1[j,e] x_e| + |c1[j]|, and a run may override at most TIE_MAX_OVERRIDES
# of them — a kernel bug at the ReLU boundary (>= for >, a bias offset) would
# need many, or larger, flips to be fitted away.
TIE_ULPS = 16
TIE_MAX_OVERRIDES = 4


class _TieInfo(dict):
    """The tie report; prints without the per-tie branch list and the ReLU hook."""

    def __repr__(self):
        return repr({k: v for k, v in self.items() if k not in ("branches", "relu")})


def oracle_td_tie_aware(pa, pm, cfg, batch, w, gpu_grad=None, margin=1e-6, pa_tgt=None, pm_tgt=None, strict=True,
                        **kw):
    """The fp64 oracle's TD update (oracle/ref_learner.td_forward) with a tie-aware
    FFN ReLU (oracle/ref_model.TieAwareRelu).  A kept FFN pre-activation within
    `margin` of 0 is a tie: fp32 arithmetic in any summation order may put it on the
    other side of 0 than fp64 does, and the backward of that one record then differs
    by its whole upstream gradient.  For every tie the backward branch
    is chosen to match the GPU result `gpu_grad` (greedy over the ties, on the L2
    distance; the forward is unchanged, both branches agree there to < margin).
    The target networks are pa_tgt / pm_tgt (default: the online parameters).
    Returns (prio, extras, ref_grad, info) with info = dict(ties=..., overridden=...,
    err_fp64_branches=normwise error with fp64's own branches, branches=the chosen
    backward branch per tie, relu=the TieAwareRelu with every tie's value and place)."""
    from oracle import ref_learner, ref_model
    cpu = {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu()) for k, v in batch.items()}
    pa_g = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
    pm_g = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
    relu = ref_model.TieAwareRelu(margin)
    loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, pa if pa_tgt is None else pa_tgt,
                                            pm if pm_tgt is None else pm_tgt, cpu, cfg, per_weight=w.cpu().double(),
                                            relu=relu, **kw)
    params = list(pa_g.values()) + list(pm_g.values())

    def grads():
        gs = torch.autograd.grad(loss, params, retain_graph=True)
        return torch.cat([g.reshape(-1) for g in gs])

    ref_g = grads()
    info = _TieInfo(ties=len(relu.ties), overridden=0, margin=margin, branches=relu.branches(), relu=relu)
    if gpu_grad is None or not relu.ties:
        info["err_fp64_branches"] = None if gpu_grad is None else normwise(gpu_grad, ref_g)
        return prio.detach(), ex, ref_g, info
    gg = gpu_grad.detach().cpu().double().reshape(-1)
    info["err_fp64_branches"] = normwise(gg, ref_g)
    on = relu.branches()
    dist = float((gg - ref_g).norm())
    for _ in range(2):  # greedy passes until no flip helps
        improved = False
        for i in range(len(on)):
            trial = list(on)
            trial[i] = not trial[i]
            relu.set_branches(trial)
            g2 = grads()
            d2 = float((gg - g2).norm())
            if d2 < dist:
                on, ref_g, dist, improved = trial, g2, d2, True
            else:
                relu.set_branches(on)
        if not improved:
            break
    fp64 = [v > 0 for _, _, v in relu.ties]
    flips = [(v, sc) for (_, _, v), sc, a, b in zip(relu.ties, relu.scales, on, fp64) if a != b]
    info["branches"] = list(on)
    info["overridden"] = len(flips)
    info["overridden_values"] = [f"{v:.1e}" for v, _ in flips]
    # |pre-activation| in fp32 ulps of its rounding scale
    info["overridden_ulps"] = [round(abs(v) / (2.0 ** -24 * sc), 2) if sc > 0 else None for v, sc in flips]
    if not strict:  # (diagnostics report, tests assert)
        return prio.detach(), ex, ref_g, info
    assert len(flips) <= TIE_MAX_OVERRIDES, ("too many ReLU ties resolved against fp64", info)
    assert all(u is not None and u <= TIE_ULPS for u in info["overridden_ulps"]), \
        ("an overridden ReLU tie is not within rounding of 0", info)
    return prio.detach(), ex, ref_g, info
