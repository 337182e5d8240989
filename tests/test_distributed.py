"""CPU, world_size 2 (gloo): the data-parallel gradient reduction of the TD update equals the
single-process full-batch gradient (the math t2omca_amd.learner relies on under RCCL)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_learner, ref_model

A, B, T = 3, 6, 4


def _cfg():
    return dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=16, heads=2, depth=1, ff_hidden_mult=4,
                n_actions=5, state_entity_feats=8, mixer_emb=16, mixer_heads=2, mixer_depth=1)


def _setup():
    cfg = _cfg()
    pa = ref_model.init_params("agent", cfg, 0, torch.float64)
    pm = ref_model.init_params("mixer", cfg, 1, torch.float64)
    from t2omca_amd.synthetic import make_batch
    batch, w = make_batch(B, T, A, seed=5, device="cpu")
    batch = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
    batch["terminated"][1, 2] = 1  # ragged masks: shards have different Σ mask
    batch["filled"][4, 3:] = 0
    return cfg, pa, pm, batch, w.double()


def _grads(cfg, pa, pm, batch, w):
    pa = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
    pm = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
    loss, _, _ = ref_learner.td_forward(pa, pm, {k: v.detach() for k, v in pa.items()},
                                        {k: v.detach() for k, v in pm.items()}, batch, cfg, per_weight=w)
    term = batch["terminated"][:, :-1, 0].float()
    mask = batch["filled"][:, :-1, 0].float()
    mask[:, 1:] = mask[:, 1:] * (1 - term[:, :-1])
    msum = mask.sum()
    (loss * msum).backward()  # un-normalised shard gradient, as the GPU learner produces it
    g = torch.cat([v.grad.reshape(-1) for v in list(pa.values()) + list(pm.values())])
    return g, msum


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from t2omca_amd.distributed import allreduce_grad_and_mask, shard_bounds
    cfg, pa, pm, batch, w = _setup()
    lo, hi = shard_bounds(B, rank, world)
    shard = {k: v[lo:hi] for k, v in batch.items()}
    g, msum = _grads(cfg, pa, pm, shard, w[lo:hi])
    buf = torch.cat([g, msum.reshape(1)])
    allreduce_grad_and_mask(buf)
    if rank == 0:
        out.put((buf[:-1] / buf[-1]).numpy())
    dist.destroy_process_group()


def test_dp_gradient_equals_full_batch():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    dp = torch.from_numpy(q.get(timeout=120))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg, pa, pm, batch, w = _setup()
    g, msum = _grads(cfg, pa, pm, batch, w)
    full = g / msum
    assert torch.allclose(dp, full, rtol=1e-10, atol=1e-12)


def test_shard_bounds_cover_batch():
    from t2omca_amd.distributed import shard_bounds
    for n in (1, 7, 1024):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = shard_bounds(n, r, world)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))
