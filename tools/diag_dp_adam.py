"""Diagnostic (not a test): the DP learner scenario of tests/test_gpu_dp_learner.py run as two
free trajectories (two gloo ranks on their shards vs one full-batch learner), printing per update
the normwise distance of the all-reduced gradient to the full-batch gradient and, at the
parameters whose post-Adam values differ most, both gradients and Adam's second moment.

Then, at the update whose gradients differ most, it names the cause: the fp64 oracle's TD update
(tests/gpu_util.oracle_td_tie_aware) is run from EACH trajectory's own state before that update
and matched to that trajectory's GPU gradient, choosing the backward branch of every FFN
pre-activation within 1e-6 of 0 (a "tie").  It prints every tie (network, block call, episode /
token / FFN unit, its fp64 value under both states, its distance to 0 in fp32 ulps of the row's
rounding scale) with the branch each trajectory's gradient takes, and the parameters of the unit
whose tie resolves differently.  A DP error would instead leave both GPU gradients far from the
tie-aware oracle.

Run on the GPU box:  python tools/diag_dp_adam.py   (T2O_LIB selects the library build)."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_dp_learner import A, B, UPDATES, _batch, _learner  # noqa: E402


def _state(learner):
    return torch.stack([learner.params, learner.target_params, learner.exp_avg,
                        learner.exp_avg_sq]).detach().cpu().clone()


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from t2omca_amd.distributed import shard_bounds
        learner = _learner(100 + rank, dev)
        batch, w = _batch(dev)
        lo, hi = shard_bounds(B, rank, world)
        shard = {k: v[lo:hi] for k, v in batch.items()}
        st, gs = [_state(learner)], []
        for u in range(UPDATES):
            learner.train(shard, 0, u, per_weight=w[lo:hi])
            torch.cuda.synchronize()
            st.append(_state(learner))
            gs.append((learner.grad[:-1] / learner.grad[-1]).detach().cpu().clone())
        out.put((rank, torch.stack(st), torch.stack(gs)))
    finally:
        dist.destroy_process_group()


def _dicts(learner, flat):
    """Reference-keyed fp64 parameter dicts (agent, mixer) from a flat [agent | mixer] vector."""
    out, off = [], 0
    for m in (learner.agent, learner.mixer):
        d = {}
        for k, p in m.named_parameters():
            d[k] = flat[off:off + p.numel()].view_as(p.detach().cpu()).double().clone()
            off += p.numel()
        out.append(d)
    return out


def _param_name(learner, i):
    off = 0
    for net, m in (("agent", learner.agent), ("mixer", learner.mixer)):
        for k, p in m.named_parameters():
            if i < off + p.numel():
                j = i - off
                return f"{net}.{k}[{tuple(int(v) for v in torch.unravel_index(torch.tensor(j), p.shape))}]"
            off += p.numel()
    return "?"


def _where(w):
    call, shape, i = w
    idx = tuple(int(v) for v in torch.unravel_index(torch.tensor(i), shape))
    net = "agent" if shape[1] == A + 1 else "mixer"  # [b·A, 1 + n_ent, FF] vs [b, 2A + 3, FF]
    return f"call {call:3d} {net} ff shape {tuple(shape)} (row, token, unit) {idx}", net, idx[-1]


def main():
    from tests.gpu_util import normwise, oracle_td_tie_aware
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, st, gs = q.get(timeout=240)
        res[r] = (st, gs)
    for p in procs:
        p.join(timeout=60)
    assert torch.equal(res[0][0], res[1][0]), "replicas differ"
    dst, dgs = res[0]
    dev = torch.device("cuda", 0)
    full = _learner(100, dev)
    batch, w = _batch(dev)
    fst, fgs = [_state(full)], []
    for u in range(UPDATES):
        full.train(batch, 0, u, per_weight=w)
        torch.cuda.synchronize()
        fst.append(_state(full))
        fgs.append((full.grad[:-1] / full.grad[-1]).detach().cpu().clone())
    fst, fgs = torch.stack(fst), torch.stack(fgs)
    gerrs = []
    for u in range(UPDATES):
        gerr = normwise(dgs[u], fgs[u])
        gerrs.append(gerr)
        d = (dst[u + 1, 0] - fst[u + 1, 0]).abs()
        print(f"update {u}: state before it {normwise(dst[u, 0], fst[u, 0]):.2e} apart; grad normwise {gerr:.2e}, "
              f"post-Adam params normwise {normwise(dst[u + 1, 0], fst[u + 1, 0]):.2e}")
        for i in torch.topk(d, 3).indices.tolist():
            print(f"   param {i} {_param_name(full, i)}: |dp| {float(d[i]):.3e} grad dp {float(dgs[u][i]):+.3e} "
                  f"full {float(fgs[u][i]):+.3e} v {float(fst[u + 1, 3][i]):.3e}")
    u = max(range(UPDATES), key=lambda k: gerrs[k])
    gd = (dgs[u] - fgs[u]).abs()
    big = (gd > 1e-3 * gd.max()).nonzero().reshape(-1).tolist()
    print(f"\nupdate {u}: gradients {gerrs[u]:.2e} apart; {len(big)} parameters within 1e-3 of the largest "
          f"difference, {big[0]}..{big[-1]}: {_param_name(full, big[0])} .. {_param_name(full, big[-1])}")
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
               n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)
    reps = {}
    for name, st, g in (("DP", dst, dgs), ("full", fst, fgs)):
        pa, pm = _dicts(full, st[u, 0])
        ta, tm = _dicts(full, st[u, 1])
        _, _, ref, info = oracle_td_tie_aware(pa, pm, cfg, batch, w, g[u], margin=1e-6, pa_tgt=ta, pm_tgt=tm,
                                              strict=False)
        reps[name] = (info, ref)
        print(f"{name} trajectory: GPU grad vs the tie-aware fp64 oracle from its own state "
              f"{normwise(g[u], ref):.2e} (with fp64's own branches {info['err_fp64_branches']:.2e}); {info}")
    (di, dref), (fi, fref) = reps["DP"], reps["full"]
    print(f"cross-check: DP GPU grad vs the full-state oracle {normwise(dgs[u], fref):.2e}, "
          f"full GPU grad vs the DP-state oracle {normwise(fgs[u], dref):.2e}")
    rd, rf = di["relu"], fi["relu"]
    print(f"\nties (|fp64 pre-activation| < 1e-6 in a consumed row of an online network): {len(rd.ties)} from the DP "
          f"state, {len(rf.ties)} from the full-batch state")
    fmap = {wh: (v, sc, b) for wh, (_, _, v), sc, b in zip(rf.where, rf.ties, rf.scales, fi["branches"])}
    for wh, (_, _, v), sc, bd in zip(rd.where, rd.ties, rd.scales, di["branches"]):
        desc, net, unit = _where(wh)
        vf, scf, bf = fmap.get(wh, (float("nan"), sc, None))
        flag = "  <-- resolved differently" if bf is not None and bd != bf else ""
        print(f"  {desc}: fp64 value DP state {v:+.3e} / full state {vf:+.3e} "
              f"({abs(v) / (2.0 ** -24 * sc):.1f} ulps of its scale {sc:.3f}); branch DP "
              f"{'on' if bd else 'off'}, full {'on' if bf else 'off' if bf is not None else '-'}{flag}")
        if flag:
            print(f"      -> {net} FFN unit {unit}: its ff.0 row / bias and ff.2 column are the gradients that move")


if __name__ == "__main__":
    main()
