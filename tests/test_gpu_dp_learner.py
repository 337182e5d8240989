"""GPU, data parallel on the PRODUCT learner: two ranks (gloo, both on cuda:0, spawned
before any GPU call in the children) each run TDLearner.train on their episode shard;
every update's post-Adam parameters equal a single-rank full-batch TDLearner update
from the same state (<= 1e-6 normwise), and the ranks stay identical.

Each update is compared from the replicas' own state (parameters, target network,
Adam moments; gradients and post-Adam parameters <= 1e-6), then the two
trajectories are run freely (<= 1e-4): over several updates they differ by gradient
summation order (~1e-7), and once the parameters differ, an FFN pre-activation
within that distance of 0 can take the other ReLU branch and move one unit's
gradients by O(1) — profiles/r4_elu/diag_dp_*.log show it: after two updates
1.2e-7 apart, the third update's gradients of one mixer FFN unit differ by 1.3e-4
normwise, with the first two updates' gradients 1.1e-7 apart.

The ranks deliberately build their modules from different seeds: the learner's
rank-0 broadcast (distributed.broadcast_state) must make the replicas identical
before the first update.  Masks are ragged (a terminated step, unfilled tail), so
the shards carry different Σ mask and only the all-reduced [grad, Σ mask] buffer
gives the full-batch normalisation (learner.py step 7).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from tests.gpu_util import normwise, require_gpu

pytestmark = pytest.mark.gpu
B, T, UPDATES = 6, 7, 3


def _batch(device, A):
    from t2omca_amd.synthetic import make_batch
    batch, w = make_batch(B, T, A, seed=11, device=device)
    batch["terminated"][1, 3] = 1  # ragged masks: the shards' Σ mask differ
    batch["filled"][4, 5:] = 0
    return batch, w


def _learner(seed, device, A, pg=None):
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args
    torch.manual_seed(seed)
    args = make_args(A, device=str(device))
    agent = TransformerAgent(None, args).to(device)
    mixer = TransformerMixer(args).to(device)
    return TDLearner(agent, mixer, process_group=pg, target_update_interval=2)


def _worker(rank, world, port, out, A):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from t2omca_amd.distributed import shard_bounds
        learner = _learner(100 + rank, dev, A)  # different init per rank: the broadcast must fix it
        batch, w = _batch(dev, A)
        lo, hi = shard_bounds(B, rank, world)
        shard = {k: v[lo:hi] for k, v in batch.items()}

        def state(grad):
            return torch.stack([learner.params, learner.target_params, learner.exp_avg,
                                learner.exp_avg_sq, grad]).detach().cpu().clone()

        hist = [state(torch.zeros_like(learner.params))]
        for u in range(UPDATES):
            learner.train(shard, 0, u, per_weight=w[lo:hi])
            torch.cuda.synchronize()
            hist.append(state(learner.grad[:-1] / learner.grad[-1]))  # the all-reduced, Σmask-normalised grad
        out.put((rank, torch.stack(hist).numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("A", [8, 16])
def test_dp_two_ranks_equal_full_batch_learner(A):
    """A = 8: the one-tile mixer, sequential update.  A = 16: the decoupled two-tile
    mixer at these small shards, so both ranks and the full-batch learner run the
    PIPELINED update (step ranges on two streams, learner._pipelined), whose
    mixer-half all-reduce is issued on the side stream after the per-range flushes."""
    require_gpu()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, A)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    r0, r1 = torch.from_numpy(res[0]), torch.from_numpy(res[1])  # [update, (params, target, m, v, grad), n]
    # replicas are identical from the start (rank 0's init) and stay identical
    assert torch.equal(r0, r1)
    dev = torch.device("cuda", 0)
    full = _learner(100, dev, A)  # rank 0's init
    if A == 16:
        assert full._pipelined(B) and full._pipelined(B // 2)
    batch, w = _batch(dev, A)
    assert torch.equal(full.params.cpu(), r0[0, 0])
    for u in range(UPDATES):
        # the full-batch update from the replicas' state before update u
        for buf, k in ((full.params, 0), (full.target_params, 1), (full.exp_avg, 2), (full.exp_avg_sq, 3)):
            buf.copy_(r0[u, k].to(dev))
        full._params_written()
        full._pack_targets()
        full.train(batch, 0, u, per_weight=w)
        torch.cuda.synchronize()
        gerr = normwise(r0[u + 1, 4], (full.grad[:-1] / full.grad[-1]).cpu())
        err = normwise(r0[u + 1, 0], full.params.cpu())
        print(f"update {u} from the replicas' state: grad {gerr:.2e}, params {err:.2e}")
        assert gerr < 1e-6, (u, gerr)
        assert err < 1e-6, (u, err)
    # ... and the two trajectories run freely: they separate only by summation
    # order, plus at most an O(1) move of one FFN unit's gradient once a ReLU tie
    # flips (the third update: 4.6e-5 on the parameters, tools/diag_dp_adam.py
    # names the pre-activation, profiles/r5_split/diag_dp.log); a systematic DP error
    # (Σ mask or Adam state handled per rank) moves every parameter by ~lr
    free = _learner(100, dev, A)
    for u in range(UPDATES):
        free.train(batch, 0, u, per_weight=w)
        torch.cuda.synchronize()
        err = normwise(r0[u + 1, 0], free.params.cpu())
        print(f"update {u} free-running: params {err:.2e}")
        assert err < 1e-4, (u, err)
