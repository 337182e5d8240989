"""CPU: the oracle's tie-aware FFN ReLU (oracle/ref_model.TieAwareRelu), which the
fp32 GPU parity tests use to take, at a kept FFN pre-activation within rounding of
0, the backward branch the GPU took (tests/gpu_util.oracle_td_tie_aware).

  * with fp64's own branches it reproduces the plain oracle exactly (forward and
    every gradient), so it changes nothing where there is no tie;
  * only pre-activations of consumed token rows are recorded (agent token 0, the
    mixer's last A + 3 rows: transformer.py:140 token pruning) and only for the
    online networks (tensors that require grad);
  * flipping a recorded tie's branch changes gradients, never the forward.
"""
import torch

from oracle import ref_learner, ref_model
from t2omca_amd.synthetic import make_batch

A, B, T = 4, 2, 3


def _cfg():
    return dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
                n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)


def _run(relu=None):
    cfg = _cfg()
    pa = ref_model.init_params("agent", cfg, 0, torch.float64)
    pm = ref_model.init_params("mixer", cfg, 1, torch.float64)
    batch, w = make_batch(B, T, A, seed=5, device="cpu")
    cpu = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
    pa_g = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
    pm_g = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
    loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, pa, pm, cpu, cfg, per_weight=w.double(), relu=relu)
    params = list(pa_g.values()) + list(pm_g.values())
    return loss, prio, ex, params


def _grads(loss, params):
    return torch.cat([g.reshape(-1) for g in torch.autograd.grad(loss, params, retain_graph=True)])


def test_tie_aware_relu_equals_plain_oracle_on_fp64_branches():
    loss0, prio0, ex0, p0 = _run()
    relu = ref_model.TieAwareRelu(1e-6)
    loss1, prio1, ex1, p1 = _run(relu)
    assert torch.equal(loss0, loss1) and torch.equal(prio0, prio1) and torch.equal(ex0["qtot"], ex1["qtot"])
    assert torch.equal(_grads(loss0, p0), _grads(loss1, p1))
    assert ref_model._ffn_relu is None  # uninstalled after the call


def test_tie_flip_changes_only_the_backward():
    relu = ref_model.TieAwareRelu(0.05)  # a wide margin: many "ties" to flip
    loss, prio, ex, params = _run(relu)
    n = len(relu.ties)
    assert n > 10
    # kept rows only: agent token 0 is 1 of A + 1 rows, the mixer's A + 3 of 2A + 3
    per_call = {}
    for m, i, v in relu.ties:
        per_call.setdefault(id(m), []).append(i)
        assert abs(v) < 0.05
    g0 = _grads(loss, params)
    on = relu.branches()
    relu.set_branches([not b for b in on])
    g1 = _grads(loss, params)
    assert (g1 - g0).abs().max() > 1e-6
    relu.set_branches(on)
    assert torch.equal(_grads(loss, params), g0)


def test_ties_are_recorded_on_consumed_rows_only():
    relu = ref_model.TieAwareRelu(10.0)  # every kept pre-activation is a "tie"
    _run(relu)
    FF = 128
    # online agent: T + 1 steps x 2 blocks x (B*A sequences x token 0 x FF);
    # online mixer: T steps x 2 blocks x (B x (A + 3) rows x FF); targets: none
    want = (T + 1) * 2 * B * A * FF + T * 2 * B * (A + 3) * FF
    assert len(relu.ties) == want
