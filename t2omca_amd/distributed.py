"""Data parallelism for the TD update (one process per GPU, RCCL over xGMI).

Episodes of a replay batch are independent (the recurrence is over t inside
an episode), so each rank trains on its own episode shard and the only
collective is ONE all-reduce per update of a flat fp32 buffer
[Σ_shard grad (un-normalised) ..., Σ_shard mask].  Dividing by the summed
mask afterwards (inside the Adam kernel, t2o_adam_step's grad_div) makes the
DP update equal to the full-batch update:

    loss = Σ_b w_b Σ_t ½ td² m / Σ_all m   ->   grad = Σ_r g_r / Σ_r M_r

At E = 32 that buffer is 84,007 floats (336 KB), latency-bound over xGMI.  The
default learner path (``TDLearner(contract="side")``, learner.py step 6) issues
it in TWO halves on two streams: the mixer half [mixer grads, Σ mask] from the
side stream as soon as the mixer's tape contraction and unfold finish there, the
agent half [agent grads] from the main stream after the agent's; the main stream
waits for both before Adam.  (``contract="pair"`` contracts both tapes in one
launch after the agent BPTT and issues the whole buffer as one all-reduce.)
Neither half runs under a BPTT kernel: those hold every SIMD (the agent BPTT
one 503-register wave per SIMD), and an RCCL kernel, like any kernel issued on
another stream, needs a wave slot — the round-3 trace shows a side-stream copy
issued at the agent BPTT's start waiting until its end
(profiles/r3_f5/prof/timeline.txt); the mixer half runs as that BPTT drains.

Replicas start identical and stay identical: the learner broadcasts its
parameters, target parameters and Adam moments from rank 0 when it is built
and after every checkpoint load (``broadcast_state``); after that every rank
applies the same all-reduced gradient with the same Adam arithmetic.
"""
import torch.distributed as dist


def world_size(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def rank(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group)
    return 0


def allreduce_grad_and_mask(buf, group=None):
    """In-place SUM all-reduce of [grad..., mask_sum]; returns buf."""
    if world_size(group) > 1:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def allreduce_async(buf, group=None):
    """Start an in-place SUM all-reduce of `buf` ordered after the work already
    queued on the CURRENT stream; returns a handle for ``wait_all`` (None
    without a process group)."""
    if world_size(group) > 1:
        return dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group, async_op=True)
    return None


def wait_all(works):
    """Make the current stream wait for every started all-reduce."""
    for w in works:
        if w is not None:
            w.wait()


def broadcast_state(tensors, group=None, src=0):
    """Overwrite every rank's copy of `tensors` (flat device buffers) with rank
    `src`'s, in place.  One broadcast per tensor; a no-op without a process group."""
    if world_size(group) > 1:
        gsrc = src if group is None else dist.get_global_rank(group, src)
        for t in tensors:
            dist.broadcast(t, gsrc, group=group)


def shard_bounds(n, rank, world):
    """Contiguous episode shard [lo, hi) of rank (weak scaling uses a full batch per rank)."""
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def rank_seed(seed, rank):
    """Per-rank seed for the env / rollout / PER streams, so data-parallel ranks
    collect and sample different episodes (rank 0 keeps `seed` itself)."""
    return int(seed) + 0x9E3779B9 * int(rank)
