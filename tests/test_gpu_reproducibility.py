"""GPU: the TD update is bit-reproducible run to run on the tuned kernels.  Two
learners that start from the same parameters and see the same batch must produce
IDENTICAL gradients, priorities and post-Adam parameters (torch.equal), over two
updates (the second starts from the first's Adam state):

  * the BPTT kernels' end-of-kernel slab flushes run wave by wave in a fixed order
    (t2o_common.hpp flush_in_wave_order), so every slab element receives its fp32
    addends in the same order;
  * the tape contractions write their slab regions with plain stores, the slab sum
    (t2o_reduce_slabs), the unfold and the Adam step reduce in a fixed order;
  * the TD loss kernel's float atomics (t2o_learner.hip) add only the reported loss
    value and the 0/1 mask count (exact in fp32), neither of which enters a gradient.

A race, an uninitialised slab entry or a wave-placement bug would show up too.  The
batches cover the mixer BPTT pipeline with 4, 2 and 1 episode pairs per workgroup,
the one-wave mixer BPTT at 16 AGVs, the chunked 64-entity agent, and runtime-entity
instances (12 and 40 AGVs)."""
import pytest
import torch

from tests.gpu_util import require_gpu
from tests.test_gpu_learner import _setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("A,B,T,precision", [(8, 64, 12, "bf16"), (8, 6, 7, "fp32"), (8, 7, 5, "bf16"),
                                             (16, 4, 6, "bf16"), (64, 2, 3, "bf16"), (12, 5, 4, "bf16"),
                                             (40, 2, 3, "fp32")])
def test_td_update_bit_reproducible_across_runs(A, B, T, precision):
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    batch, w = make_batch(B, T, A, seed=11)
    runs = []
    for _ in range(2):
        agent, mixer, _, _ = _setup(A, seed=5)
        learner = TDLearner(agent, mixer, precision=precision, priorities_to_cpu=False)
        assert learner.sa.instance != "generic" and learner.sm.instance != "generic"
        info = None
        for step in range(2):  # the second update starts from the first's Adam state
            info = learner.train(batch, 0, step, per_weight=w)
        torch.cuda.synchronize()
        runs.append((learner.grad.clone(), info["td_errors_abs"].clone(), learner.params.clone()))
    for name, a, b in zip(("grad", "priorities", "params"), *runs):
        assert torch.isfinite(a).all(), name
        ndiff = int((a != b).sum())
        print(f"A={A} B={B} T={T} {precision} {name}: {ndiff} differing elements of {a.numel()}")
        if ndiff and name == "grad":  # where they sit: [agent params | mixer params | Σ mask]
            idx = torch.nonzero(a != b).flatten().cpu()
            print(f"  differing indices {int(idx.min())}..{int(idx.max())} (agent params {learner.na}, "
                  f"mixer {learner.nm}); first {idx[:8].tolist()}; max |diff| {float((a - b).abs().max()):.3g}")
        assert torch.equal(a, b), (name, ndiff)


@pytest.mark.parametrize("A,B,T,precision", [(8, 64, 12, "bf16"), (8, 6, 7, "fp32"), (16, 4, 6, "bf16"),
                                             (64, 2, 3, "bf16"), (5, 3, 4, "fp32")])
def test_paired_contraction_equals_separate_launches(A, B, T, precision):
    """t2o_bwd_tape_contract with two tapes (both in one grid, TDLearner(contract="pair"))
    gives exactly the gradients of the two separate contractions (contract="side",
    the learner's default: the mixer's on the side stream):
    every workgroup runs the same code on the same tiles into the same slab."""
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    batch, w = make_batch(B, T, A, seed=12)
    out = {}
    for mode in ("pair", "side"):
        agent, mixer, _, _ = _setup(A, seed=6)
        # (both sequential: the pipelined update, which small multi-tile batches run by
        # default, flushes per step range and never takes contract="pair")
        learner = TDLearner(agent, mixer, precision=precision, priorities_to_cpu=False, contract=mode,
                            pipeline=False)
        info = learner.train(batch, 0, 0, per_weight=w)
        torch.cuda.synchronize()
        out[mode] = (learner.grad.clone(), info["td_errors_abs"].clone(), learner.params.clone())
    for name, a, b in zip(("grad", "priorities", "params"), out["pair"], out["side"]):
        assert torch.equal(a, b), (name, int((a != b).sum()))
