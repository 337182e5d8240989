"""GPU: parity on the grid the bench times.

The oracle tests (test_gpu_configs.py, test_gpu_runtime_shapes.py) run 2-16
episodes; bench.py times 1024 (configs[2]), and the configs[3]-shape / 16-AGV lines
512 and 1024.  Those grids run other launch geometries (256 BPTT slabs, a full wave
per SIMD, the one-wave multi-tile mixer instead of the decoupled one), so they are
checked here at full size through properties that need no fp64 run of the whole
batch (per_run.py:224-238 is the caller: one learner.train per replay batch):

  * episodes are independent and every forward kernel computes a row with the same
    code whatever the batch, so Q_tot, the TD(lambda) targets and the priorities of
    every slice equal, BIT FOR BIT, those rows of the full-batch update;
  * the raw gradient (learner.grad[:-1], before the division by the Σ mask in the
    Adam kernel) is a sum over episodes, so the full batch's equals the sum of the
    slices' up to fp32 summation order (≤ 1e-6 normwise, both precisions: the bf16
    operands of an episode are the same in both runs), and the Σ mask slots add up
    exactly;
  * one slice of the same batch matches the fp64 oracle (the fp32 bar 1e-5 / 3e-5
    tie-aware, bf16 2e-2 / 6e-2 as test_gpu_configs.py).

Masks are ragged (episodes end early: terminated at their last step, filled 0
after), as a PyMARL replay batch is.  The slices run the same kernel families as the
full batch: the decoupled mixer (T2O_MIXER_SPLIT, chosen at <= 256 episodes) is
switched off for them, since it sums the key gradients in another order (it has its
own cross-check, test_gpu_mixer_split.py)."""
import os

import pytest
import torch

from tests.gpu_util import normwise, oracle_td_tie_aware, require_gpu

pytestmark = pytest.mark.gpu

TOL = {"fp32": dict(q=1e-5, g=3e-5), "bf16": dict(q=2e-2, g=6e-2)}
GRAD_SUM_BAR = 1e-6


def _cfg(A):
    return dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
                n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)


def _ragged(batch, seed):
    """Half the episodes end early at a random step L in [T/3, T): terminated at L,
    filled 0 after it."""
    B, T1 = batch["filled"].shape[:2]
    T = T1 - 1
    g = torch.Generator(device="cpu").manual_seed(seed)
    ends = torch.randint(T // 3, T, (B,), generator=g)
    early = torch.rand(B, generator=g) < 0.5
    term = torch.zeros(B, T1, 1, dtype=torch.uint8)
    filled = torch.ones(B, T1, 1, dtype=torch.int64)
    for b in torch.nonzero(early).flatten().tolist():
        L = int(ends[b])
        term[b, L, 0] = 1
        filled[b, L + 1:, 0] = 0
    dev = batch["filled"].device
    batch["terminated"] = term.to(dev)
    batch["filled"] = filled.to(dev)
    return batch


class _Split:
    def __init__(self, flag):
        self.flag, self.old = flag, None

    def __enter__(self):
        self.old = os.environ.get("T2O_MIXER_SPLIT")
        os.environ["T2O_MIXER_SPLIT"] = self.flag

    def __exit__(self, *exc):
        if self.old is None:
            del os.environ["T2O_MIXER_SPLIT"]
        else:
            os.environ["T2O_MIXER_SPLIT"] = self.old


def _run(A, B, T, precision, S, n_oracle):
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args, make_batch
    torch.manual_seed(7)
    args = make_args(A)
    agent, mixer = TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()
    pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
    pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
    learner = TDLearner(agent, mixer, precision=precision, priorities_to_cpu=False)
    batch, w = make_batch(B, T, A, seed=21)
    batch = _ragged(batch, 22)
    snap = (learner.params.clone(), learner.exp_avg.clone(), learner.exp_avg_sq.clone(), learner.step_count)

    def restore():
        learner.params.copy_(snap[0])
        learner.exp_avg.copy_(snap[1])
        learner.exp_avg_sq.copy_(snap[2])
        learner.step_count = snap[3]
        learner._params_written()

    def update(b0, b1):
        sub = {k: v[b0:b1] for k, v in batch.items()}
        info = learner.train(sub, 0, 0, per_weight=w[b0:b1])
        torch.cuda.synchronize()
        out = (learner.grad.clone(), info["qtot"].clone(), info["targets"].clone(), info["td_errors_abs"].clone())
        restore()
        return out

    g_full, q_full, t_full, p_full = update(0, B)
    assert torch.isfinite(g_full).all() and torch.isfinite(q_full).all()
    g_sum = torch.zeros_like(g_full, dtype=torch.float64)
    mismatched = []
    with _Split("0"):
        for b0 in range(0, B, S):
            g, q, t, p = update(b0, b0 + S)
            g_sum += g.double()
            for name, a, ref in (("qtot", q, q_full[b0:b0 + S]), ("targets", t, t_full[b0:b0 + S]),
                                 ("prio", p, p_full[b0:b0 + S])):
                if not torch.equal(a, ref):
                    mismatched.append((b0, name, int((a != ref).sum())))
        g_o, q_o, t_o, p_o = update(0, n_oracle)
    err_sum = normwise(g_full[:-1], g_sum[:-1])
    print(f"A={A} B={B} T={T} {precision}: {B // S} slices of {S}; slices differing from the full batch "
          f"{mismatched[:6]}; Σ-of-slices raw gradient vs full {err_sum:.2e}; Σ mask {float(g_full[-1]):.0f} "
          f"vs {float(g_sum[-1]):.0f}")
    assert not mismatched, mismatched
    assert float(g_full[-1]) == float(g_sum[-1])
    assert err_sum < GRAD_SUM_BAR, err_sum
    # one slice against the fp64 oracle
    sub = {k: v[:n_oracle] for k, v in batch.items()}
    g = (g_o[:-1] / g_o[-1]).cpu()
    prio, ex, ref_g, ties = oracle_td_tie_aware(pa, pm, _cfg(A), sub, w[:n_oracle],
                                                g if precision == "fp32" else None)
    errs = dict(qtot=normwise(q_o, ex["qtot"]), targets=normwise(t_o, ex["targets"]), prio=normwise(p_o, prio),
                grad=normwise(g, ref_g))
    print(f"  slice of {n_oracle} vs the fp64 oracle:", {k: f"{v:.2e}" for k, v in errs.items()}, "relu ties", ties)
    tol = TOL[precision]
    assert errs["qtot"] < tol["q"] and errs["targets"] < tol["q"] and errs["prio"] < tol["q"], errs
    assert errs["grad"] < tol["g"], errs


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_config2_full_grid_1024x60(precision):
    """configs[2], the headline grid: 8 AGVs, 1024 episodes x T = 60."""
    require_gpu()
    _run(8, 1024, 60, precision, S=16, n_oracle=4)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_config3_shape_full_grid_A64_512x60(precision):
    """configs[3]-shape, one GPU's share: 64 AGVs, 512 episodes x T = 60 (the one-wave
    five-tile mixer with L2 weights, the chunked agent)."""
    require_gpu()
    _run(64, 512, 60, precision, S=32, n_oracle=2)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_A16_full_grid_1024x150(precision):
    """The reference's default scenario (16 AGVs) at a full replay grid, 1024 x T = 150."""
    require_gpu()
    _run(16, 1024, 150, precision, S=64, n_oracle=2)
