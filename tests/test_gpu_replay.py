"""GPU: device-resident prioritized replay vs the numpy oracle
(oracle/ref_replay.py): stratified proportional sampling indices and IS
weights, priority updates with max tracking, ring-buffer insert with wrap, the
episode gather, and one full rollout -> insert -> sample -> train ->
update_priorities cycle on the device."""
import types

import numpy as np
import pytest
import torch

from oracle import ref_replay
from tests.gpu_util import require_gpu

pytestmark = pytest.mark.gpu


def _buffer(n_ep=40, T1=5, A=3, cap=32, alpha=0.6, beta=0.4, t_max=1000, seed=7):
    from t2omca_amd.replay import PrioritizedReplayBuffer
    g = torch.Generator(device="cuda").manual_seed(1)
    batch = {"obs": torch.randn(n_ep, T1, A, 9 * A, device="cuda", generator=g),
             "actions": torch.randint(0, 5, (n_ep, T1, A, 1), device="cuda", generator=g),
             "terminated": torch.zeros(n_ep, T1, 1, dtype=torch.uint8, device="cuda")}
    return PrioritizedReplayBuffer(batch, cap, T1, alpha, beta, t_max, seed=seed), batch


def test_sample_matches_oracle():
    require_gpu()
    buf, batch = _buffer()
    buf.insert_episode_batch({k: v[:20] for k, v in batch.items()})
    g = np.random.default_rng(3)
    pri = g.uniform(0.01, 5.0, 20)
    buf.update_priorities(list(range(20)), pri.tolist())
    for t in (0, 500):
        idx, w = buf.sample_indices(8, t)
        ref_idx, ref_w = ref_replay.sample(pri ** 0.6, 8, 0.4 + t * 0.6 / 1000, 7, buf._draws - 1)
        assert np.array_equal(idx.cpu().numpy(), ref_idx)
        assert np.allclose(w.cpu().numpy(), ref_w, rtol=1e-5)


def test_update_priorities_and_max():
    require_gpu()
    buf, batch = _buffer()
    buf.insert_episode_batch({k: v[:10] for k, v in batch.items()})
    assert torch.allclose(buf.p[:10].cpu(), torch.ones(10))
    idx = torch.tensor([1, 4, 7], device="cuda")
    pr = torch.tensor([0.5, 3.0, 2.0], device="cuda")
    buf.update_priorities(idx, pr)
    ref_p, ref_max = ref_replay.update(np.ones(10), 1.0, [1, 4, 7], [0.5, 3.0, 2.0], 0.6)
    assert np.allclose(buf.p[:10].cpu().numpy(), ref_p, rtol=1e-6)
    assert abs(float(buf.max_priority) - ref_max) < 1e-6
    buf.insert_episode_batch({k: v[10:12] for k, v in batch.items()})  # new episodes at max priority
    assert np.allclose(buf.p[10:12].cpu().numpy(), 3.0 ** 0.6, rtol=1e-6)


def test_update_priorities_add_equals_adding_first():
    """update_priorities(idx, td, add=1e-6) (the driver's `+ 1e-6` inside the kernel)
    writes exactly what update_priorities(idx, td + 1e-6) does."""
    require_gpu()
    out = []
    for fused in (False, True):
        buf, batch = _buffer()
        buf.insert_episode_batch({k: v[:10] for k, v in batch.items()})
        idx = torch.tensor([0, 3, 9], device="cuda")
        td = torch.tensor([2.5e-7, 0.125, 7.0], device="cuda")
        if fused:
            buf.update_priorities(idx, td, add=1e-6)
        else:
            buf.update_priorities(idx, td + 1e-6)
        out.append((buf.p.clone(), buf.max_priority.clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_ring_insert_and_gather():
    require_gpu()
    buf, batch = _buffer(cap=32)
    buf.insert_episode_batch({k: v[:30] for k, v in batch.items()})
    buf.insert_episode_batch({k: v[30:40] for k, v in batch.items()})  # wraps: slots 30, 31, 0..7
    assert buf.episodes_in_buffer == 32 and buf.buffer_index == 8
    slot_of = {30: 30, 31: 31}
    slot_of.update({32 + i: i for i in range(8)})
    idx = torch.tensor([0, 5, 30, 31, 12], device="cuda")
    got = buf.gather(idx)
    src = [32, 37, 30, 31, 12]
    for k in batch:
        assert torch.equal(got[k], batch[k][src])


def test_rollout_insert_sample_train_cycle():
    require_gpu()
    from t2omca_amd.env import VecEnv
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.replay import PrioritizedReplayBuffer
    from t2omca_amd.runner import RolloutRunner
    from t2omca_amd.synthetic import make_args
    A, M, n, T = 8, 4, 6, 5
    torch.manual_seed(0)
    agent = TransformerAgent(None, make_args(A)).cuda()
    mixer = TransformerMixer(make_args(A)).cuda()
    runner = RolloutRunner(agent, VecEnv(n, mec_num=M, agv_num=A, episode_limit=T, seed=5))
    learner = TDLearner(agent, mixer, priorities_to_cpu=False)
    batch = runner.run()
    buf = PrioritizedReplayBuffer(batch, 16, T + 1, 0.6, 0.4, 10000)
    buf.insert_episode_batch(batch)
    batch = runner.run()
    buf.insert_episode_batch(batch)
    sample, idx, w = buf.sample(4, runner.t_env)
    info = learner.train(sample, runner.t_env, 0, per_weight=w)
    buf.update_priorities(idx, info["td_errors_abs"].flatten() + 1e-6)
    torch.cuda.synchronize()
    p = buf.p[:buf.episodes_in_buffer].cpu()
    assert torch.isfinite(p).all() and bool((p > 0).all())
    expect = (info["td_errors_abs"].flatten().cpu() + 1e-6) ** 0.6
    assert torch.allclose(p[idx.cpu()], expect, rtol=1e-5) or len(set(idx.tolist())) < 4


def test_reference_driver_loop_runs_unchanged():
    """per_run.py:212-238's training loop, statement for statement, on the device
    runner / buffer / learner (priorities to the host as the reference buffer wants)."""
    require_gpu()
    from t2omca_amd.env import VecEnv
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.replay import PrioritizedReplayBuffer
    from t2omca_amd.runner import RolloutRunner
    from t2omca_amd.synthetic import make_args
    A, T, batch_size, batch_size_run = 3, 4, 4, 4
    args = types.SimpleNamespace(device=torch.device("cuda", torch.cuda.current_device()), t_max=3 * batch_size_run * T)
    torch.manual_seed(0)
    mac_agent = TransformerAgent(None, make_args(A)).cuda()
    learner = TDLearner(mac_agent, TransformerMixer(make_args(A)).cuda())
    runner = RolloutRunner(mac_agent, VecEnv(batch_size_run, mec_num=2, agv_num=A, episode_limit=T, seed=1))
    buffer = PrioritizedReplayBuffer(runner.run(), 16, T + 1, 0.6, 0.4, args.t_max)
    episode, trained = 0, 0
    while runner.t_env <= args.t_max:
        with torch.no_grad():
            episode_batch = runner.run(test_mode=False)
            buffer.insert_episode_batch(episode_batch)
        if buffer.can_sample(batch_size):
            episode_sample, idx, weights = buffer.sample(batch_size, runner.t_env)
            max_ep_t = episode_sample.max_t_filled()
            episode_sample = episode_sample[:, :max_ep_t]
            if episode_sample.device != args.device:
                episode_sample.to(args.device)
            info = learner.train(episode_sample, runner.t_env, episode, weights)
            del episode_sample
            new_priorities = info["td_errors_abs"].flatten() + 1e-6
            buffer.update_priorities(idx, new_priorities.numpy().tolist())
            trained += 1
        episode += batch_size_run
    torch.cuda.synchronize()
    assert trained >= 2 and max_ep_t == T + 1
    assert torch.isfinite(learner.params).all()
    assert bool((buffer.p[:buffer.episodes_in_buffer] > 0).all())
