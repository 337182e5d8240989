"""GPU: the runtime-entity MFMA instances (csrc/t2o_dispatch.hpp) — the default
network of every BASELINE config (emb 32, 3 heads, depth 2, ff_hidden_mult 4) at an
AGV count without an exact instance (environment_multi_mec.py:9-11 takes any
agv_num; transf_agent.py:9-48 / n_transf_mixer.py:13-50 any n_agents).  Each
instance is compiled for a capacity class and reads the real count at run time:

  agent   8 / 16 entities in registers (padding entities score -inf), 64 streamed in
          8-entity chunks (a partial last chunk masked);
  mixer   8 and 13 agents: one 16-row query tile, the two-wave pipelined BPTT;
          16 / 32 / 64: the multi-tile kernels (query tiles past A + 3 skipped,
          padding keys -inf).

The cases below put every class on both sides of its boundaries (A = 2 ... 63).
The runtime mixer instances also compute every qmix_pos_func (softplus with beta,
quadratic, identity; n_transf_mixer.py:95-103), so those heads run on MFMA kernels
at every AGV count; at 8 AGVs (the headline) a non-abs head runs the exact instance
with the head as a run-time parameter.
Checked against the reference modules' goldens (5 and 32 AGVs, per-step forward +
autograd through the drop-in modules) and against the fp64 oracle's full TD update
(oracle/ref_learner; TD semantics parity-unpinned).

Bars (normwise max|Δ| / max|ref|): fp32 forward quantities (Q_tot,
targets, priorities) <= 1e-5, gradients <= 3e-5; bf16 <= 2e-2 / 6e-2 (bf16 MFMA
operands, fp32 accumulation / LayerNorm / softmax / recurrent state), as the exact
instances (tests/test_gpu_configs.py).  The fp32 cases compare against a tie-aware
oracle (tests/gpu_util.oracle_td_tie_aware): a kept FFN pre-activation within 1e-6
of 0 can take the other ReLU branch in fp32 than in fp64 whatever the summation
order — seed 3 at 40 AGVs has one 1.8e-8 from 0, and with fp64's branch its
gradient error is 1e-3 (profiles/r3_rt2/) — so the oracle's backward takes, at
each such record only, the branch the GPU result agrees with, and the test prints
how many records that was.  Measured on the box
(profiles/r3_rt2/pytest.log), fp32: Q_tot <= 1.1e-6, gradients <= 1.2e-6 (A = 63)
and <= 3.6e-7 elsewhere; bf16: Q_tot <= 1.0e-2, gradients <= 1.4e-2.
"""
import os

import pytest

from tests.gpu_util import require_gpu
from tests.test_gpu_generic import GOLD, _cfg_of, _td, agent_module_check, mixer_module_check

pytestmark = pytest.mark.gpu

# (A, B, T): every capacity class, padded and full, of both networks
FP32_CASES = [(2, 4, 6), (5, 4, 6), (12, 4, 6), (13, 3, 5), (14, 3, 5), (20, 2, 5), (32, 2, 4), (40, 2, 4),
              (63, 2, 3)]
BF16_CASES = [(5, 4, 6), (12, 4, 6), (20, 2, 5), (40, 2, 4)]


@pytest.fixture(autouse=True)
def _tuned(monkeypatch):
    monkeypatch.setenv("T2O_GENERIC", "0")


@pytest.mark.parametrize("A,B,T", FP32_CASES, ids=lambda v: str(v))
def test_runtime_instance_td_update_fp32(A, B, T):
    require_gpu()
    learner, _ = _td(dict(_cfg_of(A), tag=f"A{A}"), B, T)
    assert learner.sa.instance == "runtime" and learner.sm.instance == "runtime"


@pytest.mark.parametrize("A,B,T", BF16_CASES, ids=lambda v: str(v))
def test_runtime_instance_td_update_bf16(A, B, T):
    require_gpu()
    learner, _ = _td(dict(_cfg_of(A), tag=f"A{A}"), B, T, precision="bf16", tol=(2e-2, 6e-2))
    assert learner.sa.instance == "runtime" and learner.sm.instance == "runtime"


@pytest.mark.parametrize("name", ["a5_e32_h3_d2", "a32_e32_h3_d2"])
def test_runtime_instance_modules_vs_reference_goldens(name):
    """The drop-in modules (reference signatures, one step per call + autograd) on
    the runtime instances, against the reference modules' own outputs."""
    require_gpu()
    assert agent_module_check(os.path.join(GOLD, f"agent_{name}.npz")) == "runtime"
    assert mixer_module_check(os.path.join(GOLD, f"mixer_{name}.npz")) == "runtime"


@pytest.mark.parametrize("name", ["a8_softplus", "a8_quadratic", "a8_identity"])
def test_mixer_heads_vs_reference_goldens(name):
    """Every non-abs qmix_pos_func against the reference module's own outputs and
    autograd (n_transf_mixer.py:95-103).  At 8 AGVs these run the exact 8-AGV mixer
    instance with the head as a run-time parameter (t2o_dispatch.hpp mode 2)."""
    require_gpu()
    assert mixer_module_check(os.path.join(GOLD, f"mixer_{name}.npz")) == "exact"


# 8 AGVs: the exact instance with a run-time head; 7 / 12 / 5: the runtime-entity
# instances of capacity 8 and 13 (counts and head both run-time)
@pytest.mark.parametrize("A,B,T,head,beta,precision,inst", [(8, 4, 6, "softplus", 0.5, "fp32", "exact"),
                                                            (7, 4, 6, "softplus", 0.5, "fp32", "runtime"),
                                                            (12, 3, 5, "quadratic", 1.0, "fp32", "runtime"),
                                                            (5, 4, 6, "identity", 1.0, "fp32", "runtime"),
                                                            (8, 4, 6, "quadratic", 1.0, "fp32", "exact"),
                                                            (8, 4, 6, "softplus", 2.0, "bf16", "exact"),
                                                            (7, 4, 6, "softplus", 2.0, "bf16", "runtime")])
def test_mixer_heads_td_update(A, B, T, head, beta, precision, inst):
    require_gpu()
    cfg = dict(_cfg_of(A, qmix_pos_func=head, qmix_pos_func_beta=beta), tag=f"A{A}-{head}")
    tol = (2e-2, 6e-2) if precision == "bf16" else None
    learner, _ = _td(cfg, B, T, precision=precision, tol=tol)
    assert learner.sm.instance == inst
