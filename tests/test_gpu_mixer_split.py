"""GPU: the decoupled multi-tile mixer (t2o_mixer_split.hip) against t2o_mixer.hip's
one-wave kernels on the same inputs (T2O_MIXER_SPLIT=1 / 0 in one process).

The forward computes every query row with the same code on the same key block —
only which kernel, and which lane of a 16-row tile, holds the row changes — and MFMA
output columns are independent, so y, hyper tokens, qvals, final rows and block
inputs are bit-identical.  The backward sums the key gradients in another order
(the rows before the window, then the window's), so dL/dqvals (the head's backward,
no key sum) are bit-identical and the key-token / weight gradients agree to
rounding.  Parity with the reference itself: every multi-tile TD-update test of
tests/test_gpu_configs.py / test_gpu_runtime_shapes.py runs this path (their
batches are small) against the fp64 oracle."""
import os

import pytest
import torch

from tests.gpu_util import normwise, require_gpu

pytestmark = pytest.mark.gpu


def _setup(A, B, T, precision, seed=5):
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args, make_batch
    torch.manual_seed(seed)
    args = make_args(A, device="cuda")
    agent, mixer = TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()
    learner = TDLearner(agent, mixer, precision=precision, priorities_to_cpu=False)
    batch, w = make_batch(B, T, A, seed=seed)
    return learner, batch, w


def _with_split(flag, fn):
    old = os.environ.get("T2O_MIXER_SPLIT")
    os.environ["T2O_MIXER_SPLIT"] = flag
    try:
        return fn()
    finally:
        if old is None:
            del os.environ["T2O_MIXER_SPLIT"]
        else:
            os.environ["T2O_MIXER_SPLIT"] = old


@pytest.mark.parametrize("A,precision", [(16, "bf16"), (16, "fp32"), (20, "bf16"), (40, "fp32"), (64, "bf16")])
def test_split_mixer_equals_one_wave_kernels(A, precision):
    require_gpu()
    from t2omca_amd import ops
    B, T = 5, 9
    learner, batch, w = _setup(A, B, T, precision)
    sm, sa = learner.sm, learner.sa
    assert int(ops.lib().t2o_mixer_split(ops.ctypes.byref(sm.layout()), B)) in (0, 1)
    ops.pack_params(sa, learner.params[:learner.na], learner.pack_a)
    ops.pack_params(sm, learner.params[learner.na:], learner.pack_m)
    obs, state = batch["obs"], batch["state"]
    act = batch["actions"][..., 0].contiguous()
    avail = batch["avail_actions"].int()
    q_on, h_on, q_tg, h_tg = ops.agent_unroll_fwd(sa, learner.pack_a, obs, pack_tg=learner.pack_a)
    gy = torch.randn(B, T, device="cuda", generator=torch.Generator("cuda").manual_seed(1))

    def run():
        o_on, o_tg = ops.mixer_unroll_fwd(sm, learner.pack_m, state, h_on, qmode_on=1, q_on=q_on, actions=act,
                                          avail=avail, T_on=T, pack_tg=learner.pack_m, hid_tg=h_tg, qmode_tg=2,
                                          q_tg=q_tg, T_tg=T + 1)
        gpack, gqv, ghid, ghw0 = ops.mixer_unroll_bwd(sm, learner.pack_m, state, h_on, o_on, gy, want_ghw0=True)
        torch.cuda.synchronize()
        return o_on, o_tg, gpack, gqv, ghid, ghw0

    on1, tg1, gp1, gqv1, gh1, gw1 = _with_split("1", run)
    on0, tg0, gp0, gqv0, gh0, gw0 = _with_split("0", run)
    for k in ("y", "hw", "qv", "xout", "xmid"):
        assert torch.equal(on1[k], on0[k]), ("online", k)
    for k in ("y", "hw", "qv"):
        assert torch.equal(tg1[k], tg0[k]), ("target", k)
    assert torch.equal(gqv1, gqv0)
    errs = {"ghid": normwise(gh1, gh0), "ghw0": normwise(gw1, gw0), "grads": normwise(gp1, gp0)}
    print(f"A={A} {precision} split vs one-wave backward:", {k: f"{v:.1e}" for k, v in errs.items()})
    bar = 1e-5 if precision == "fp32" else 2e-3
    assert max(errs.values()) < bar, errs


def test_split_learner_update_is_reproducible_and_close():
    """Two TD updates at 16 AGVs through the learner: split vs one-wave within
    rounding (gradients 1e-5, post-Adam parameters 5e-5), and the split path
    bit-reproducible run to run."""
    require_gpu()
    A, B, T = 16, 4, 12

    def run():
        learner, batch, w = _setup(A, B, T, "fp32", seed=7)
        for u in range(2):
            learner.train(batch, 0, u, per_weight=w)
        torch.cuda.synchronize()
        return learner.params.clone(), (learner.grad[:-1] / learner.grad[-1]).clone()

    p1, g1 = _with_split("1", run)
    p1b, g1b = _with_split("1", run)
    p0, g0 = _with_split("0", run)
    assert torch.equal(p1, p1b) and torch.equal(g1, g1b)
    print(f"split vs one-wave: grads {normwise(g1, g0):.1e}, params {normwise(p1, p0):.1e}")
    # (Adam's m / sqrt(v) turns gradient rounding on near-zero entries into steps of
    # up to lr: the parameters after two updates sit 6.5e-6 apart for 1.8e-7 in the grads)
    assert normwise(g1, g0) < 1e-5 and normwise(p1, p0) < 5e-5


@pytest.mark.parametrize("A,precision,ranges", [(16, "fp32", 4), (16, "bf16", 7), (20, "fp32", 3)])
def test_pipelined_update_matches_sequential(A, precision, ranges):
    """TDLearner's pipelined mode (agent and decoupled-mixer recurrences in step ranges
    on two streams: h, the hyper tokens and their grads carried between ranges through
    memory) against the same update with one launch per recurrence.  Forward outputs are
    bit-identical (the same per-step code); the weight gradients are flushed per range,
    so they agree to rounding; run to run the pipelined update is bit-reproducible."""
    require_gpu()
    from t2omca_amd.learner import TDLearner
    B, T = 4, 13

    def run(pipeline):
        learner, batch, w = _setup(A, B, T, precision, seed=9)
        learner = TDLearner(learner.agent, learner.mixer, precision=precision, priorities_to_cpu=False,
                            pipeline=pipeline, pipeline_ranges=ranges)
        assert learner._pipelined(B) == (pipeline is True)
        infos = [learner.train(batch, 0, u, per_weight=w) for u in range(2)]
        torch.cuda.synchronize()
        return (infos[0]["qtot"].clone(), infos[0]["td_errors_abs"].clone(),
                (learner.grad[:-1] / learner.grad[-1]).clone(), learner.params.clone())

    q1, p1, g1, w1 = run(True)
    q1b, p1b, g1b, w1b = run(True)
    q0, p0, g0, w0 = run(False)
    assert torch.equal(q1, q0) and torch.equal(p1, p0), "forward / priorities of the first update"
    assert torch.equal(g1, g1b) and torch.equal(w1, w1b), "pipelined update not reproducible"
    errs = {"grads": normwise(g1, g0), "params": normwise(w1, w0)}
    print(f"A={A} {precision} ranges={ranges} pipelined vs sequential:", {k: f"{v:.1e}" for k, v in errs.items()})
    bar = (1e-5, 5e-5) if precision == "fp32" else (2e-3, 5e-3)
    assert errs["grads"] < bar[0] and errs["params"] < bar[1], errs


def test_pipeline_falls_back_when_agent_bwd_cannot_take_ranges():
    """T2O_AGENT_BWD=single selects the one-wave agent BPTT, which takes only the
    whole unroll (t2o_agent_bwd_ranges = 0): pipeline='auto' must then run the
    sequential update (the same result as pipeline=False), and pipeline=True must
    refuse rather than fail part way through the update."""
    require_gpu()
    from t2omca_amd import ops
    from t2omca_amd.learner import TDLearner
    A, B, T = 16, 4, 9
    old = os.environ.get("T2O_AGENT_BWD")
    os.environ["T2O_AGENT_BWD"] = "single"
    try:
        base, batch, w = _setup(A, B, T, "bf16", seed=9)
        assert int(ops.lib().t2o_agent_bwd_ranges(ops.ctypes.byref(base.sa.layout()), 1)) == 0
        outs = []
        for pipeline in ("auto", False):
            learner = TDLearner(base.agent, base.mixer, precision="bf16", priorities_to_cpu=False, pipeline=pipeline)
            snap = learner.params.clone()
            assert not learner._pipelined(B)
            info = learner.train(batch, 0, 0, per_weight=w)
            torch.cuda.synchronize()
            outs.append((learner.grad.clone(), info["td_errors_abs"].clone()))
            learner.params.copy_(snap)
            learner._params_written()
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
        forced = TDLearner(base.agent, base.mixer, precision="bf16", priorities_to_cpu=False, pipeline=True)
        with pytest.raises(RuntimeError, match="pipeline=True"):
            forced.train(batch, 0, 0, per_weight=w)
    finally:
        if old is None:
            del os.environ["T2O_AGENT_BWD"]
        else:
            os.environ["T2O_AGENT_BWD"] = old
    with_ranges = TDLearner(base.agent, base.mixer, precision="bf16", priorities_to_cpu=False)
    assert int(ops.lib().t2o_agent_bwd_ranges(ops.ctypes.byref(with_ranges.sa.layout()), 1)) == 1
    assert with_ranges._pipelined(B)
