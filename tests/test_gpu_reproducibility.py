"""GPU: the TD update is reproducible run to run.  Two learners that start from the
same parameters and see the same batch must agree to summation-order rounding.
They are not bit-identical: the waves of a workgroup add their vector grads into the
workgroup's slab with float atomics, and the TD loss sums with float atomics, so
the order of fp32 additions varies (measured: 1 ulp of a 2^18-sized raw gradient).
A race, an uninitialised slab entry or a wave-placement bug would show up as an
O(1) difference.  Bars (normwise max|Δ| / max|ref|): fp32 1e-6; bf16 1e-4, since a
one-ulp fp32 difference can flip the bf16 rounding of an MFMA operand.  The batches
cover the mixer BPTT pipeline with 4, 2 and 1 episode pairs per workgroup, and the
one-wave mixer BPTT at 16 AGVs."""
import pytest
import torch

from tests.gpu_util import normwise, require_gpu
from tests.test_gpu_learner import _setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("A,B,T,precision", [(8, 64, 12, "bf16"), (8, 6, 7, "fp32"), (8, 7, 5, "bf16"),
                                             (16, 4, 6, "bf16")])
def test_td_update_reproducible_across_runs(A, B, T, precision):
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    batch, w = make_batch(B, T, A, seed=11)
    runs = []
    for _ in range(2):
        agent, mixer, _, _ = _setup(A, seed=5)
        learner = TDLearner(agent, mixer, precision=precision, priorities_to_cpu=False)
        info = None
        for step in range(2):  # the second update starts from the first's Adam state
            info = learner.train(batch, 0, step, per_weight=w)
        torch.cuda.synchronize()
        runs.append((learner.grad.clone(), info["td_errors_abs"].clone(), learner.params.clone()))
    for name, a, b in zip(("grad", "priorities", "params"), *runs):
        assert torch.isfinite(a).all(), name
        err = normwise(a.double().cpu(), b.double().cpu())
        print(f"A={A} B={B} T={T} {precision} {name}: normwise {err:.2e}")
        assert err <= (1e-6 if precision == "fp32" else 1e-4), (name, err)
