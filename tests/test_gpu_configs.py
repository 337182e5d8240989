"""GPU parity at every BASELINE.json config's real shape (BASELINE.json "configs",
SURVEY.md §8 scenario mapping), on an episode slice the fp64 CPU oracle finishes
in seconds:

  configs[0]/[1]  16 AGVs, T = 150 (default scenario): the agent + mixer forward
                  unroll (configs[1]'s inference workload) and the full TD update
                  (configs[0]'s), 4 episodes, each in fp32 AND bf16;
  configs[2]      8 AGVs, T = 60 (the headline): the full TD update in fp32 AND in
                  bf16 (configs[2] is quoted in bf16), 16 episodes, plus the bf16
                  agent Q error at every t up to t = 59;
  configs[3]      64 AGVs, T = 60: the full TD update, 2 episodes (chunked online-
                  softmax agent, five-tile mixer with weights through L2), fp32 AND
                  bf16;
  configs[4]      the vectorised env, 16 AGVs x 2 MEC servers, a full 150-step
                  episode, bit-exact against the numpy restatement for 6 envs.

Oracle: oracle/ref_learner.td_forward in fp64 (pinned to the reference modules'
goldens by tests/test_oracle_golden.py; TD semantics parity-unpinned).
Bars (normwise max|Δ| / max|ref|):
  fp32   Q_tot, targets, priorities <= 1e-5; parameter gradients <= 3e-5 against the
         tie-aware oracle (below);
  bf16   Q_tot, targets, priorities <= 2e-2; gradients <= 6e-2; agent Q at every
         t <= 4e-2 (bf16 MFMA operands, fp32 accumulation / LayerNorm / softmax /
         recurrent state).  Measured on the box (profiles/r3_a/pytest.log), bf16:
           configs[2] A=8  T=60:  Q_tot 1.2e-2, grads 7.2e-3; agent Q 3.4e-3 at t=0,
                                  1.7e-2 at t=30, 2.3e-2 at t=59, 2.6e-2 max;
           configs[0] A=16 T=150: Q_tot 1.1e-2, grads 1.1e-2; agent Q 3.9e-3 at t=0,
                                  2.0e-2 at t=75, 1.7e-2 at t=149, 2.5e-2 max;
           configs[1] A=16 T=150 forward: Q_tot 1.4e-2, hyper tokens 3.9e-3; agent
                                  Q 1.3e-2 overall, 2.1e-2 at t=149;
           configs[3] A=64 T=60:  Q_tot 1.1e-2, grads 5.5e-3; agent Q 4.0e-3 at t=0,
                                  1.8e-2 at t=59, 2.0e-2 max.
         (the rounding of the recurrent input to bf16 operands compounds over the
         unroll and then saturates; SURVEY §8c's all-bf16 probe: 4.5e-2).
The fp32 gradient check and ReLU ties: an FFN pre-activation within fp32 rounding
of 0 can take the other ReLU branch than in fp64 whatever the summation order, and
that one record's whole upstream gradient (not a rounding-sized amount) then enters
dW1 and, through the recurrence, every earlier step.  With ~2M ReLU evaluations per
update at configs[2]'s slice that happens about once per run.  The oracle's FFN ReLU
is therefore tie-aware (tests/gpu_util.oracle_td_tie_aware): at every kept
pre-activation within 1e-6 of 0 its backward takes the branch the GPU result agrees
with, and the test prints how many there were.  Measured (profiles/r4_a/pytest.log):
configs[2] 7 ties, 1 overridden (a pre-activation of -9.7e-9): gradient error
5.97e-5 with fp64's branches, 6.3e-7 tie-aware; configs[0] 15 ties / 3 overridden,
4.7e-6 -> 3.6e-6; configs[3] 8 / 2, 7.3e-7 -> 7.2e-7.  Q_tot, targets and
priorities (forward quantities) are not affected (2e-7 - 6e-7).
"""
import dataclasses

import pytest
import torch

from oracle import ref_learner, ref_model
from tests.gpu_util import normwise, oracle_td_tie_aware, require_gpu

pytestmark = pytest.mark.gpu

TOL = {"fp32": dict(q=1e-5, g=3e-5, qt=1e-5), "bf16": dict(q=2e-2, g=6e-2, qt=4e-2)}


def _cfg(A):
    return dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
                n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)


def _modules(A, seed=0):
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args
    torch.manual_seed(seed)
    args = make_args(A)
    return TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()


_ORACLE = {}


def _oracle(A, B, T, seed):
    """The fp64 oracle's TD update on the seeded modules + batch, computed once per
    shape and shared by the fp32 and bf16 runs (the oracle is the slow half)."""
    key = (A, B, T, seed)
    if key not in _ORACLE:
        from t2omca_amd.synthetic import make_batch
        agent, mixer = _modules(A)
        pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
        pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
        batch, w = make_batch(B, T, A, seed=seed)
        cpu = {k: (v.cpu().double() if v.is_floating_point() else v.cpu()) for k, v in batch.items()}
        pa_g = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
        pm_g = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
        loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, pa, pm, cpu, _cfg(A), per_weight=w.cpu().double())
        loss.backward()
        ref_g = torch.cat([v.grad.reshape(-1) for v in list(pa_g.values()) + list(pm_g.values())])
        _ORACLE[key] = (prio.detach(), {k: v.detach() if torch.is_tensor(v) else v for k, v in ex.items()}, ref_g)
    return _ORACLE[key]


RELU_MARGIN = 1e-6


def _td_vs_oracle(A, B, T, precision, seed=3):
    """GPU TD update vs the fp64 oracle.  fp32 also reports the gradient error
    against the tie-aware oracle (tests/gpu_util.oracle_td_tie_aware: at a kept FFN
    pre-activation within RELU_MARGIN of 0 the oracle's backward takes the branch the
    GPU result agrees with) as errs["grad_tie_aware"], with the tie counts."""
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    agent, mixer = _modules(A)
    learner = TDLearner(agent, mixer, precision=precision)
    batch, w = make_batch(B, T, A, seed=seed)
    info = learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    g = (learner.grad[:-1] / learner.grad[-1]).cpu()
    prio, ex, ref_g = _oracle(A, B, T, seed)
    errs = dict(qtot=normwise(info["qtot"], ex["qtot"]), targets=normwise(info["targets"], ex["targets"]),
                prio=normwise(info["td_errors_abs"], prio), grad=normwise(g, ref_g))
    if precision == "fp32":
        pa = {k: v.detach().cpu().double() for k, v in _modules(A)[0].state_dict().items()}
        pm = {k: v.detach().cpu().double() for k, v in _modules(A)[1].state_dict().items()}
        _, _, ref_t, ties = oracle_td_tie_aware(pa, pm, _cfg(A), batch, w, g, margin=RELU_MARGIN)
        errs["grad_tie_aware"] = normwise(g, ref_t)
        print(f"A={A} B={B} T={T} relu ties", ties)
    return errs, learner, batch, ex


def _agent_q_per_t(learner, batch, ex, precision, label):
    """Agent Q error at every step (the bf16 drift grows with t): the
    online network's unroll with the learner's own pack vs the oracle's mac_out."""
    from t2omca_amd import ops
    q, _ = ops.agent_unroll_fwd(learner.sa, learner.pack_a, batch["obs"])
    torch.cuda.synchronize()
    ref_q = ex["mac_out"]
    per_t = [normwise(q[:, t], ref_q[:, t]) for t in range(q.shape[1])]
    T = q.shape[1] - 1
    print(precision, label, "agent Q normwise error t=0/mid/T-1/T:",
          [f"{per_t[t]:.2e}" for t in (0, T // 2, T - 1, T)], f"max {max(per_t):.2e}")
    assert per_t[T - 1] < TOL[precision]["qt"] and max(per_t) < TOL[precision]["qt"], max(per_t)
    return per_t


def _check(errs, precision):
    tol = TOL[precision]
    print(precision, {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["qtot"] < tol["q"] and errs["targets"] < tol["q"] and errs["prio"] < tol["q"], errs
    # fp32: against the tie-aware oracle (_td_vs_oracle); bf16: plain
    assert errs.get("grad_tie_aware", errs["grad"]) < tol["g"], errs


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_config2_headline_td_update_T60(precision):
    """configs[2]: 8 AGVs x 4 MEC, T = 60, a 16-episode slice of the 1024-episode batch."""
    require_gpu()
    errs, learner, batch, ex = _td_vs_oracle(8, 16, 60, precision)
    _check(errs, precision)
    _agent_q_per_t(learner, batch, ex, precision, "configs[2]")


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_config1_forward_A16_T150(precision):
    """configs[1]: agent + mixer forward only (inference over a replay batch), 16 AGVs, T = 150.
    bf16 bar: TOL["bf16"]["q"] on Q_tot / hyper tokens, ["qt"] on the agent Q / h."""
    require_gpu()
    from t2omca_amd import ops
    from t2omca_amd.synthetic import make_batch
    A, B, T = 16, 4, 150
    agent, mixer = _modules(A)
    pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
    pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
    batch, _ = make_batch(B, T, A, seed=4)
    prec = 1 if precision == "bf16" else 0
    sa, sm = dataclasses.replace(agent.shape, prec=prec), dataclasses.replace(mixer.shape, prec=prec)
    pack_a = ops.pack_params(sa, torch.cat([p.detach().reshape(-1) for p in agent.parameters()]))
    pack_m = ops.pack_params(sm, torch.cat([p.detach().reshape(-1) for p in mixer.parameters()]))
    q, h = ops.agent_unroll_fwd(sa, pack_a, batch["obs"])
    act = batch["actions"][..., 0]
    o = ops.mixer_unroll_fwd(sm, pack_m, batch["state"], h, qmode_on=1, q_on=q, actions=act, T_on=T,
                             want_xout=False)
    torch.cuda.synchronize()
    key = ("fwd", A, B, T)
    if key not in _ORACLE:
        cfg = _cfg(A)
        obs = batch["obs"].cpu().double()
        ref_q, ref_h = ref_model.agent_unroll(pa, obs, torch.zeros(B, A, 32, dtype=torch.float64), cfg=cfg)
        chosen = torch.gather(ref_q[:, :-1], 3, act[:, :-1].cpu().unsqueeze(3)).squeeze(3)
        ref_y, ref_hw = ref_model.mixer_unroll(pm, chosen, ref_h[:, :-1], batch["state"][:, :-1].cpu().double(),
                                               torch.zeros(B, 3, 32, dtype=torch.float64), cfg=cfg)
        _ORACLE[key] = (ref_q, ref_h, ref_y, ref_hw)
    ref_q, ref_h, ref_y, ref_hw = _ORACLE[key]
    errs = dict(q=normwise(q, ref_q), h=normwise(h, ref_h), y=normwise(o["y"], ref_y), hw=normwise(o["hw"], ref_hw))
    per_t = [normwise(q[:, t], ref_q[:, t]) for t in range(q.shape[1])]
    print(f"configs[1] forward {precision}", {k: f"{v:.2e}" for k, v in errs.items()},
          f"agent Q t=0/75/149/150: {[f'{per_t[t]:.2e}' for t in (0, 75, 149, 150)]}")
    if precision == "fp32":
        assert max(errs.values()) < 1e-5, errs
    else:
        tol = TOL["bf16"]
        assert errs["y"] < tol["q"] and errs["hw"] < tol["q"], errs
        assert errs["q"] < tol["qt"] and errs["h"] < tol["qt"], errs


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_config0_td_update_A16_T150(precision):
    """configs[0]: the default scenario's TD update, 16 AGVs, T = 150, 4 episodes.
    bf16 runs the 16-entity agent BPTT with the full (format-0) tape and the
    two-tile mixer BPTT with transposed weight reads (the 16-AGV bench path)."""
    require_gpu()
    errs, learner, batch, ex = _td_vs_oracle(16, 4, 150, precision)
    _check(errs, precision)
    if precision == "bf16":
        _agent_q_per_t(learner, batch, ex, precision, "configs[0]")


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_config3_td_update_A64_T60(precision):
    """configs[3]: 64 AGVs x 16 MEC, T = 60, 2 episodes (of the 512 per GPU).  bf16
    runs the chunked online-softmax agent and the five-tile, L2-weight mixer (the
    64-AGV bench path)."""
    require_gpu()
    errs, learner, batch, ex = _td_vs_oracle(64, 2, 60, precision)
    _check(errs, precision)
    if precision == "bf16":
        _agent_q_per_t(learner, batch, ex, precision, "configs[3]")


def test_config4_env_full_episode_A16_M2_T150():
    """configs[4]: the vectorised env over a whole 150-step episode, bit-exact."""
    require_gpu()
    from tests.test_gpu_env import _rollout_vs_oracle
    _rollout_vs_oracle(NE=6, M=2, A=16, T=150, eps=1, seed=21)


def test_bf16_mode_is_the_learner_precision():
    """The bf16 learner really runs the prec-1 kernels (pack carries the bf16 image)."""
    require_gpu()
    agent, mixer = _modules(8)
    from t2omca_amd.learner import TDLearner
    lr = TDLearner(agent, mixer, precision="bf16")
    assert lr.sa.prec == 1 and lr.sm.prec == 1
    assert lr.pack_a.numel() == dataclasses.replace(agent.shape, prec=1).layout().pack_floats
