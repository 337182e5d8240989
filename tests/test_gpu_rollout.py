"""GPU: ε-greedy action selection and the closed-loop rollout.

* t2o_select_actions vs the numpy oracle (oracle/ref_mac.py), exactly, for
  greedy, mixed and fully random selection, with tied and masked Q values;
* RolloutRunner plumbing: the batch it writes equals a fresh VecEnv replayed
  with the recorded actions (obs / state / avail bit-exact, rewards equal), the
  greedy actions equal the masked argmax of an agent unroll over the recorded
  observations (hidden state carried step by step = the unroll), and every
  selected action was available;
* the rollout batch (time-major storage, strided views) feeds TDLearner.train,
  which matches the CPU oracle TD update on it.
"""
import numpy as np
import pytest
import torch

from oracle import ref_learner, ref_mac
from tests.gpu_util import normwise, require_gpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("eps", [0.0, 0.3, 1.0])
def test_select_actions_matches_oracle(eps):
    require_gpu()
    from t2omca_amd import ops
    g = torch.Generator().manual_seed(5)
    rows, na = 4096, 5
    q = torch.randint(-3, 4, (rows, na), generator=g).float()  # many ties
    avail = (torch.rand(rows, na, generator=g) < 0.6).int()
    avail[:, 0] = 1  # the no-offload action is always available (environment_multi_mec.py:61-74)
    avail[::7] = 0
    avail[::7, 3] = 1  # rows with a single available action
    act = ops.select_actions(q.cuda(), avail.cuda(), eps, seed=99, counter=17).cpu().numpy()
    ref = ref_mac.select_actions(q.numpy(), avail.numpy(), eps, 99, 17)
    assert np.array_equal(act, ref)
    assert (avail.numpy()[np.arange(rows), act] != 0).all()
    if eps == 1.0:  # uniform over the available actions
        full = avail.numpy().sum(1) == na
        counts = np.bincount(act[full], minlength=na)
        assert counts.min() > 0.8 * full.sum() / na


def _agent(A, seed=0):
    from t2omca_amd.modules import TransformerAgent
    from t2omca_amd.synthetic import make_args
    torch.manual_seed(seed)
    return TransformerAgent(None, make_args(A)).cuda()


@pytest.mark.parametrize("A,M,n,T,prec", [(3, 2, 5, 4, "fp32"), (8, 4, 6, 6, "fp32"), (8, 4, 6, 6, "bf16"),
                                          (16, 2, 9, 5, "bf16")])
def test_rollout_matches_env_replay_and_agent_unroll(A, M, n, T, prec):
    """The runner's per-step agent launches equal one unroll over the recorded obs
    (fp32, and the bf16 agent step of RolloutRunner(precision="bf16"))."""
    require_gpu()
    from t2omca_amd import ops
    from t2omca_amd.env import VecEnv
    from t2omca_amd.runner import RolloutRunner
    agent = _agent(A)
    env = VecEnv(n, mec_num=M, agv_num=A, episode_limit=T, seed=11)
    runner = RolloutRunner(agent, env, seed=3, precision=prec)
    batch = runner.run(test_mode=True)
    ret = runner.last_returns
    torch.cuda.synchronize()
    # replay the recorded actions on a fresh env
    env2 = VecEnv(n, mec_num=M, agv_num=A, episode_limit=T, seed=11)
    st, av, ob = env2.reset()
    assert torch.equal(ob, batch["obs"][:, 0]) and torch.equal(st, batch["state"][:, 0])
    assert torch.equal(av, batch["avail_actions"][:, 0])
    ret2 = torch.zeros_like(ret)
    for t in range(T):
        acts = batch["actions"][:, t, :, 0].contiguous()
        taken = torch.gather(batch["avail_actions"][:, t], 2, acts.unsqueeze(2))
        assert bool((taken != 0).all())
        r, _, _, st, av, ob = env2.step(acts)
        assert torch.equal(ob, batch["obs"][:, t + 1]) and torch.equal(st, batch["state"][:, t + 1])
        assert torch.equal(av, batch["avail_actions"][:, t + 1])
        assert torch.equal(r.float(), batch["reward"][:, t, 0])
        ret2 += r
    assert torch.equal(ret, ret2)
    assert int(batch["terminated"].sum()) == 0 and bool((batch["filled"] == 1).all())
    # greedy actions = masked argmax of the unrolled agent's Q on the recorded observations
    flat = torch.cat([p.detach().reshape(-1) for p in agent.parameters()])
    pack = ops.pack_params(runner.shape, flat)
    q, _ = ops.agent_unroll_fwd(runner.shape, pack, batch["obs"])
    masked = q.masked_fill(batch["avail_actions"] == 0, -float("inf"))
    assert torch.equal(masked.argmax(-1), batch["actions"][..., 0])
    if prec == "bf16":  # the bf16 step against fp32 operands on the same observations
        q32, _ = ops.agent_unroll_fwd(agent.shape, ops.pack_params(agent.shape, flat), batch["obs"])
        err = float((q - q32).abs().max() / q32.abs().max())
        print(f"bf16 rollout agent step: Q normwise {err:.2e} vs fp32")
        assert err < 2e-2


def test_rollout_batch_feeds_learner():
    require_gpu()
    from t2omca_amd.env import VecEnv
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerMixer
    from t2omca_amd.runner import RolloutRunner
    from t2omca_amd.synthetic import make_args
    A, M, n, T = 8, 4, 4, 5
    agent = _agent(A, seed=1)
    mixer = TransformerMixer(make_args(A)).cuda()
    pa = {k: v.detach().cpu().double() for k, v in agent.state_dict().items()}
    pm = {k: v.detach().cpu().double() for k, v in mixer.state_dict().items()}
    env = VecEnv(n, mec_num=M, agv_num=A, episode_limit=T, seed=2)
    runner = RolloutRunner(agent, env, seed=4, epsilon_start=0.5)
    batch = runner.run()
    learner = TDLearner(agent, mixer)
    w = torch.linspace(0.5, 1.0, n, device="cuda")
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
               n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)
    cpu = {k: v.cpu().contiguous() for k, v in batch.items()}

    def oracle(dtype):
        cast = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in cpu.items()}
        pa_g = {k: v.to(dtype).clone().requires_grad_(True) for k, v in pa.items()}
        pm_g = {k: v.to(dtype).clone().requires_grad_(True) for k, v in pm.items()}
        loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, {k: v.to(dtype) for k, v in pa.items()},
                                                {k: v.to(dtype) for k, v in pm.items()}, cast, cfg,
                                                per_weight=w.cpu().to(dtype))
        loss.backward()
        return prio, ex, torch.cat([v.grad.reshape(-1) for v in list(pa_g.values()) + list(pm_g.values())])

    prio, ex, ref_g = oracle(torch.float64)
    _, _, ref_g32 = oracle(torch.float32)
    info = learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    assert normwise(info["qtot"], ex["qtot"]) < 1e-5
    assert normwise(info["td_errors_abs"], prio) < 1e-5
    g = (learner.grad[:-1] / learner.grad[-1]).cpu()
    # env rewards are O(100), so the loss gradient sums large terms of both signs:
    # the bar is fp32 arithmetic itself on the same batch (the fp32 oracle's error
    # against fp64), with the synthetic-data bar as the floor
    bar = max(3e-5, 3 * normwise(ref_g32, ref_g))
    assert normwise(g, ref_g) < bar
