#!/usr/bin/env python3
"""Benchmark: agent-transitions/sec of a full TD update (fwd + bwd + Adam).

BASELINE.json metric, configs[2]: 8 AGVs x 4 MEC servers, replay batch 1024
episodes x T = 60, emb 32 / 3 heads / depth 2 (SURVEY.md §8 defaults), one
TD update = t2omca_amd.learner.TDLearner.train on a synthetic batch resident
in HBM (t2omca_amd.synthetic, SURVEY.md §8 d).  One agent-transition = one
(episode, timestep, agent) of the sampled batch, so an update is B*T*A.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N` with N > 1 from a plain process starts the N ranks itself
(torch.distributed.run on 127.0.0.1, one process per GPU, RCCL); under a
launcher (WORLD_SIZE set) each process is one rank.

Data parallel (weak scaling): every rank trains on its own 1024-episode shard
and the flat gradient (+ Σ mask) is all-reduced over RCCL once per update.
Rank 0 prints ONE JSON line.  Per-kernel times come from HIP events recorded
on the launch stream inside the timed region; the CPU baseline is the
oracle's PyTorch-CPU TD update (oracle/ref_learner.py) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_FP32_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 matrix = vector peak (dense)
PEAK_BF16_TFLOPS = 2500.0    # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (not the 2:1-sparsity figure)
PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E spec peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # untimed; the GPU's clocks ramp over the first ~10 updates (per-update period
    # 2.74 -> 2.43 ms at configs[2], profiles/r3_f3/NOTE.txt)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--batch", type=int, default=None,
                    help="episodes per GPU (default: 1024 train = configs[2]; 128 forward = configs[1])")
    ap.add_argument("--T", type=int, default=None,
                    help="episode length (default: 60 train = configs[2]; 150 forward / rollout, the default "
                         "scenario of configs[1] / configs[4])")
    ap.add_argument("--agents", type=int, default=None, help="AGVs (default: 8 train; 16 forward / rollout)")
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default="bf16",
                    help="MFMA operand precision (BASELINE configs[2] is quoted in bf16; accumulation, "
                         "LayerNorm, softmax, recurrent state, TD targets and Adam stay fp32 either way)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=16, help="episodes in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--mode", choices=("train", "forward", "rollout", "expand", "dropin", "loop"), default="train",
                    help="train: the TD update (the BASELINE metric); forward: online agent + mixer "
                         "unroll only (configs[1], inference over a replay batch); rollout: closed-loop "
                         "env step + agent step + ε-greedy over --envs envs per GPU (configs[4]); dropin: "
                         "per-call cost of the drop-in modules' per-step forward; loop: the driver's whole "
                         "cycle (per_run.py:212-238): rollout of --envs envs -> insert -> PER sample -> "
                         "TD update -> update_priorities, --updates-per-rollout updates of --batch episodes")
    ap.add_argument("--updates-per-rollout", type=int, default=8,
                    help="loop mode: learner updates per rollout (default 8 x 1024 episodes = the 8192 "
                         "episodes each rollout collects)")
    ap.add_argument("--envs", type=int, default=8192, help="rollout mode: envs per GPU")
    ap.add_argument("--compact-obs", action="store_true",
                    help="rollout mode: store obs in the compact wire format (SURVEY.md §8 f3)")
    ap.add_argument("--no-cpu-configs0", action="store_true",
                    help="skip the configs[0]-shape (16 AGVs, T=150) CPU-baseline figure")
    ap.add_argument("--mecs", type=int, default=2, help="rollout mode: MEC servers")
    ap.add_argument("--rollout-precision", choices=("fp32", "bf16"), default="fp32",
                    help="rollout / loop modes: the agent step's MFMA operands (fp32 = the reference's precision)")
    ap.add_argument("--qmix-pos-func", choices=("abs", "softplus", "quadratic", "identity"), default="abs",
                    help="the mixer head's positivity function (n_transf_mixer.py:95-103); at 8 AGVs every "
                         "head runs the exact MFMA mixer instance (softplus / quadratic / identity with a run-time "
                         "head), at other AGV counts the runtime-entity instance of the count's capacity class "
                         "(ops.NetShape.instance; the bench line's config.kernels says which)")
    ap.add_argument("--contract", choices=("pair", "side"), default="side",
                    help="weight-gradient tape contractions: side (default) = the mixer's on a side stream "
                         "issued before the agent BPTT; pair = both in one launch after the agent BPTT")
    ap.add_argument("--td-algo", choices=("auto", "sequential", "wave"), default="auto",
                    help="TD(lambda) target kernel (t2o_td_args.algo): the sequential per-episode recursion "
                         "or the one-wave-per-episode suffix scan; auto = the library default")
    ap.add_argument("--priorities", choices=("device", "cpu"), default="device",
                    help="where each update's |TD errors| go: device (consumed by the device-resident "
                         "PrioritizedReplayBuffer, t2omca_amd/replay.py) or cpu (the reference driver's "
                         "host-side buffer contract: one device->host copy and sync per update)")
    ap.add_argument("--serial", action="store_true",
                    help="no side-stream overlap: every kernel's HIP-event time is its isolated cost")
    ap.add_argument("--kernel-timer-every", type=int, default=5,
                    help="bracket the kernels with HIP events on every k-th timed step (the per-kernel "
                         "times and the roofline come from those steps; the events cost ~40 us per "
                         "instrumented update, so every step would inflate ms_per_step ~1.5%%, every 5th "
                         "~0.3%%; 0: never)")
    ap.add_argument("--no-fp32-companion", dest="fp32_companion", action="store_false",
                    help="skip the fp32-precision companion timing of the same workload (bf16 runs)")
    ap.add_argument("--no-config-companions", dest="config_companions", action="store_false",
                    help="skip the fp32 16-AGV TD update (1024 episodes x T=150) timed beside the "
                         "headline (N=1, configs[2] runs only)")
    ap.add_argument("--print-workload-tag", action="store_true",
                    help="print the tag that keys profiles/hbm_traffic.json for these args and exit")
    a = ap.parse_args()
    # per-mode defaults: each mode's BASELINE config (SURVEY.md §8 scenario mapping)
    scen = a.mode in ("forward", "rollout", "dropin", "loop")
    if a.agents is None:
        a.agents = 16 if scen else 8
    if a.T is None:
        a.T = 150 if scen else 60
    if a.batch is None:
        a.batch = 128 if a.mode == "forward" else 1024
    return a


def workload_tag(args):
    if args.mode == "rollout":
        return rollout_tag(args)
    return f"b{args.batch}_t{args.T}_a{args.agents}_{args.dtype}"


def train_config_name(A, B, T):
    """Which BASELINE config a TD-update run is (the learner's shapes depend on the
    AGV count only: entities = agents, state = 8 features per AGV)."""
    if (A, B, T) == (8, 1024, 60):
        return "configs[2]"
    if A == 64:
        return "configs[3]-shape (64 AGVs, per-GPU shard)"
    if B == 32:
        return "configs[0]-shape (batch 32)"
    return "configs[2]-style"


class KernelTimer:
    """HIP events around each phase of TDLearner.train (same stream as the launches)."""

    def __init__(self):
        self.events = []
        self.updates = 0  # instrumented updates (a pipelined update times each step range of a kernel)

    def __call__(self, name):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.events.append((name, ev))

    def durations(self):
        out = {}
        for (n0, e0), (n1, e1) in zip(self.events, self.events[1:]):
            if n0.startswith("begin:") and n1 == "end:" + n0[6:]:
                out.setdefault(n0[6:], []).append(e0.elapsed_time(e1))
        return out


def traffic_for(kernel, tag):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/hbm_traffic.json: rocprofv3 FETCH_SIZE / WRITE_SIZE passes, corrected
    as MI355X_MICROARCH.md prescribes, by tools/pmc_traffic.py), or None when that
    summary was taken on another workload."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "hbm_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != tag:
        return None
    k = d.get("kernels", {}).get(kernel)
    return None if k is None else k.get("hbm_bytes")


def _cpu_rate(A, T, B, threads, seconds):
    """min-of-N time of the oracle's CPU TD update on B episodes with `threads` threads."""
    from oracle import ref_learner, ref_model
    from t2omca_amd.synthetic import make_batch
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
               n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)
    batch, w = make_batch(B, T, A, seed=7, device="cpu")
    learner = ref_learner.RefLearner(ref_model.init_params("agent", cfg, 0), ref_model.init_params("mixer", cfg, 1),
                                     cfg)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        learner.train(batch, 0, 0, per_weight=w)  # warm-up
        times = []
        t_start = time.perf_counter()
        while len(times) < 3 or (time.perf_counter() - t_start < seconds and len(times) < 20):
            t0 = time.perf_counter()
            learner.train(batch, 0, 0, per_weight=w)
            times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    return B * T * A / min(times), len(times)


def host_cpus():
    """The host cores this process may really run on: its CPU affinity set, capped
    by a cgroup CPU quota (v2 cpu.max, v1 cpu.cfs_quota_us) and, when no quota is
    visible, by OMP_NUM_THREADS (the GPU box sets it to the box's CPU share: its
    affinity set spans the whole machine).  Oversubscribing the share is not a
    baseline: 256 torch threads on a 16-CPU share ran the rollout's CPU path at
    11 agent-transitions/s (profiles/r3_c/rollout.json) against 2.3 K/s on 8."""
    import math
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = math.ceil(int(q) / int(per))
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f1, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f2:
                q, per = int(f1.read()), int(f2.read())
                if q > 0:
                    quota = math.ceil(q / per)
        except (OSError, ValueError):
            pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    usable = min(affinity, quota) if quota else (min(affinity, omp) if omp else affinity)
    return {"usable": max(1, usable), "affinity": affinity, "cgroup_quota": quota, "omp_num_threads": omp}


def cpu_baseline(args):
    """The oracle's PyTorch-CPU TD update (oracle/ref_learner.py, reference op order,
    fp32) on a bounded sample of the same workload, on this host's cores.
    BASELINE.md: torch.set_num_threads(n) with n = the host cores available —
    len(os.sched_getaffinity(0)), capped by the CPU share the process really has
    (host_cpus: on the GPU box the affinity set is the whole 256-core machine but
    the share is 16).  Beside it: one thread, and configs[0]'s own shape (16 AGVs,
    T = 150) at n threads."""
    hc = host_cpus()
    n_thr = hc["usable"]
    A, T, B = args.agents, args.T, args.cpu_sample
    sec = args.cpu_seconds
    rate, n = _cpu_rate(A, T, B, n_thr, sec)
    out = {"value": rate, "unit": "agent-transitions/s", "cores": n_thr, "kind": "port",
           "sample": f"{B} episodes x T={T} x A={A} (one TD update = {B * T * A} agent-transitions), "
                     f"min of {n} updates after 1 warm-up, torch CPU fp32, torch.set_num_threads({n_thr}): "
                     f"the host cores available (sched_getaffinity {hc['affinity']}, cgroup quota "
                     f"{hc['cgroup_quota']}, OMP_NUM_THREADS {hc['omp_num_threads']})",
           "affinity_cores": hc["affinity"], "host_cpus": hc}
    b1 = max(1, B // 4)
    rate1, n1 = _cpu_rate(A, T, b1, 1, sec / 3)
    out["single_thread"] = {"value": rate1, "unit": "agent-transitions/s", "cores": 1,
                            "sample": f"{b1} episodes x T={T} x A={A}, min of {n1} updates after 1 warm-up"}
    if not args.no_cpu_configs0:
        b0 = 2
        r0, n0 = _cpu_rate(16, 150, b0, n_thr, sec / 2)
        out["configs0"] = {"value": r0, "unit": "agent-transitions/s", "cores": n_thr,
                           "sample": f"configs[0]'s shape (16 AGVs, T=150; the config quotes 32 episodes): "
                                     f"{b0} episodes, min of {n0} updates after 1 warm-up, {n_thr} threads"}
    return out


def _cpu_rollout_rate(A, M, T, n_env, threads, seconds):
    """The CPU path configs[4] replaces, on a sample of n_env envs: per timestep the
    agent forward on torch CPU (oracle/ref_model.agent_forward, transf_agent.py:54-76)
    for all n_env x A agents, ε-greedy (oracle/ref_mac), then each env's worker step
    (oracle/ref_env.RefEnv.worker_step = env.step + get_state + get_avail_actions +
    get_obs, parallel_runner.py:239-256, environment_multi_mec.py:309-366) in one
    process.  Returns agent-transitions/s over whole steps until `seconds` elapse."""
    import numpy as np
    from oracle import ref_mac, ref_model
    from oracle.ref_env import RefEnv
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
               n_actions=5)
    p = ref_model.init_params("agent", cfg, 0)
    envs = [RefEnv(M, A, T, 1, e) for e in range(n_env)]
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        obs = np.stack([e.worker_reset()[2] for e in envs])
        avail = np.stack([e.get_avail_actions() for e in envs])
        h = torch.zeros(n_env, A, 32)
        steps, t0 = 0, time.perf_counter()
        while steps < T and (steps < 3 or time.perf_counter() - t0 < seconds):
            with torch.no_grad():
                q, h = ref_model.agent_forward(p, torch.as_tensor(obs, dtype=torch.float32), h, n_entities=A,
                                               feat_dim=9, emb=32, heads=3, depth=2)
            act = ref_mac.select_actions(q.reshape(-1, 5).numpy(), avail.reshape(-1, 5), 0.05, 3, steps)
            act = act.reshape(n_env, A)
            res = [e.worker_step(act[i]) for i, e in enumerate(envs)]
            obs = np.stack([r[5] for r in res])
            avail = np.stack([np.asarray(r[4]) for r in res])
            steps += 1
        el = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return n_env * A * steps / el, steps


def rollout_bench(args, world, rank, dev):
    """configs[4]: every rank steps its own shard of envs (no collective)."""
    from t2omca_amd.env import VecEnv
    from t2omca_amd.modules import TransformerAgent
    from t2omca_amd.perfmodel import agent_row_step_flops, env_step_bytes, ref_order_network_flops
    from t2omca_amd.runner import RolloutRunner
    from t2omca_amd.synthetic import make_args
    A, T, n = args.agents, args.T, args.envs
    torch.manual_seed(0)
    agent = TransformerAgent(None, make_args(A, device=str(dev))).to(dev)
    env = VecEnv(n, mec_num=args.mecs, agv_num=A, episode_limit=T, seed=1, device=dev, wire=args.compact_obs)
    runner = RolloutRunner(agent, env, seed=0, compact_obs=args.compact_obs, precision=args.rollout_precision)
    for _ in range(args.warmup):
        runner.run(new_buffers=False)
    timer = KernelTimer()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        # HIP events around every 10th timestep's launches on every 2nd rollout
        runner.timer = timer if args.kernel_timer_every > 0 and i % args.kernel_timer_every == 0 else None
        runner.run(new_buffers=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    runner.timer = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    env_steps = world * n * T * args.steps
    kern = {k: sum(v) / len(v) for k, v in timer.durations().items()}
    # the rollout's two hot kernels and their bounds: the env step (HBM: SURVEY §8(d)'s
    # bytes per agent-step x n x A per launch) and the one-step agent forward (MFMA:
    # §8(d)'s F_agent per sequence x n x A); the dominant one carries `roofline`
    env_bytes = env_step_bytes(A) * n * A
    agent_flops = agent_row_step_flops(n=A) * n * A  # what the agent kernel executes per launch
    agent_peak = PEAK_BF16_TFLOPS if args.rollout_precision == "bf16" else PEAK_FP32_TFLOPS
    agent_ref_flops = ref_order_network_flops(A)[0] * n * A
    rl = {}
    if "env_step" in kern:
        ach = env_bytes / (kern["env_step"] * 1e-3) / 1e9
        rl["env_step"] = {"bound": "hbm", "kernel": "env_step", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                          "frac": ach / PEAK_HBM_GBS, "traffic": traffic_for("env_step", rollout_tag(args)),
                          "algorithmic_bytes_per_launch": env_bytes, "avg_launch_ms": kern["env_step"],
                          "basis": "SURVEY.md §8(d): (16+4+64+4 + 9A*4) B per agent-step (perfmodel.env_step_bytes)"}
    if "agent_fwd" in kern:
        ach = agent_flops / (kern["agent_fwd"] * 1e-3) / 1e12
        rl["agent_fwd"] = {"bound": "mfma", "kernel": "agent_fwd", "achieved": ach, "peak": agent_peak,
                           "unit": "TFLOP/s", "frac": ach / agent_peak,
                           "traffic": traffic_for("agent_fwd", rollout_tag(args)),
                           "algorithmic_flops_per_launch": agent_flops, "avg_launch_ms": kern["agent_fwd"],
                           "basis": "executed algorithm (perfmodel.agent_row_step_flops: folded projections, "
                                    f"observation-space attention, token 0 only) vs the {args.rollout_precision} "
                                    "MFMA peak (the rollout agent's operand precision)",
                           "reference_order": {"flops_per_launch": agent_ref_flops,
                                               "achieved": agent_ref_flops / (kern["agent_fwd"] * 1e-3) / 1e12,
                                               "note": "SURVEY.md §8(d) F_agent: the reference association order "
                                                       "counts more work than the kernel issues, so it is not "
                                                       "priced against the peak"}}
    dom = max(rl, key=lambda k: rl[k]["avg_launch_ms"]) if rl else None
    out = {"metric": "agent-transitions/sec for closed-loop rollout (env step + agent step + eps-greedy)",
           "value": env_steps * A / elapsed, "unit": "agent-transitions/s", "env_steps_per_s": env_steps / elapsed,
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": f"{args.rollout_precision} agent, fp64 env", "data": "simulated (VecEnv, env_spec stand-ins)",
           "config": {"workload": f"configs[4]: {n} envs/GPU x {A} AGVs x {args.mecs} MEC, episode {T} steps, "
                                  "one rollout per step" + (", compact obs wire format" if args.compact_obs else ""),
                      "global_envs": n * world, "agents": A, "compact_obs": bool(args.compact_obs)},
           "roofline": rl.get(dom), "roofline_other": {k: v for k, v in rl.items() if k != dom},
           "kernels_ms": {k: round(v, 4) for k, v in sorted(kern.items())},
           "per_env_step_ms": elapsed / args.steps / T * 1e3}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        hc = host_cpus()
        ne = 8
        r, st = _cpu_rollout_rate(A, args.mecs, T, ne, hc["usable"], args.cpu_seconds)
        out["cpu_baseline"] = {"value": r, "unit": "agent-transitions/s", "cores": hc["usable"], "kind": "port",
                               "sample": f"{ne} envs x {A} AGVs x {args.mecs} MEC, {st} steps of one episode: "
                                         f"agent forward on torch CPU ({hc['usable']} threads: the host cores "
                                         f"available, see host_cpus), eps-greedy and the numpy env "
                                         f"(oracle/ref_env, environment_multi_mec.py:309-366) serially in one "
                                         f"process (the reference runs one process per env, "
                                         f"parallel_runner.py:18-32)", "affinity_cores": hc["affinity"],
                               "host_cpus": hc}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _cpu_loop_rate(A, M, T, ne, threads):
    """The CPU path of the driver's cycle on a sample (per_run.py:212-238 with
    parallel_runner.py:102-221): one rollout of `ne` envs (torch-CPU agent forward,
    ε-greedy, the numpy env's worker step; as _cpu_rollout_rate), the episodes as an
    EpisodeBatch-shaped dict, then one TD update (oracle/ref_learner, fp32, Adam) on
    those same `ne` episodes — so, as in the GPU loop's default, every collected
    episode is learned from once.  Returns (learned agent-transitions/s, env
    steps/s, rollout s, train s)."""
    import numpy as np
    from oracle import ref_learner, ref_mac, ref_model
    from oracle.ref_env import RefEnv
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2, ff_hidden_mult=4,
               n_actions=5, state_entity_feats=8, mixer_emb=32, mixer_heads=3, mixer_depth=2)
    pa, pm = ref_model.init_params("agent", cfg, 0), ref_model.init_params("mixer", cfg, 1)
    learner = ref_learner.RefLearner(pa, pm, cfg)
    envs = [RefEnv(M, A, T, 1, e) for e in range(ne)]
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        t0 = time.perf_counter()
        st, av, ob = zip(*[e.worker_reset() for e in envs])
        obs = [np.stack(ob)]
        state = [np.stack(st)]
        avail = [np.stack([np.asarray(a) for a in av])]
        acts, rews = [], []
        h = torch.zeros(ne, A, 32)
        for t in range(T + 1):
            with torch.no_grad():
                q, h = ref_model.agent_forward(learner.pa, torch.as_tensor(obs[-1], dtype=torch.float32), h,
                                               n_entities=A, feat_dim=9, emb=32, heads=3, depth=2)
            act = ref_mac.select_actions(q.reshape(-1, 5).numpy(), avail[-1].reshape(-1, 5), 0.05, 3, t)
            acts.append(act.reshape(ne, A))
            if t == T:
                break
            res = [e.worker_step(acts[-1][i]) for i, e in enumerate(envs)]
            rews.append([r[0] for r in res])
            state.append(np.stack([r[3] for r in res]))
            avail.append(np.stack([np.asarray(r[4]) for r in res]))
            obs.append(np.stack([r[5] for r in res]))
        t1 = time.perf_counter()
        tm = lambda xs, dt: torch.as_tensor(np.stack(xs, 1), dtype=dt)  # noqa: E731
        batch = {"obs": tm(obs, torch.float32), "state": tm(state, torch.float32),
                 "avail_actions": tm(avail, torch.int64), "actions": tm(acts, torch.int64)[..., None],
                 "reward": torch.cat([tm(rews, torch.float32), torch.zeros(ne, 1)], 1)[..., None],
                 "terminated": torch.zeros(ne, T + 1, 1), "filled": torch.ones(ne, T + 1, 1)}
        learner.train(batch, ne * T, 0, per_weight=torch.ones(ne))
        t2 = time.perf_counter()
    finally:
        torch.set_num_threads(prev)
    return ne * T * A / (t2 - t0), ne * T / (t2 - t0), t1 - t0, t2 - t1


def loop_bench(args, world, rank, dev):
    """The driver's cycle, per_run.py:212-238, on the device, each rank on its own
    shard (no collective except the learner's gradient all-reduce):
        episode_batch = runner.run()                          (RolloutRunner, --envs envs)
        buffer.insert_episode_batch(episode_batch)
        repeat --updates-per-rollout times:
            sample, idx, w = buffer.sample(--batch, t_env); sample = sample[:, :sample.max_t_filled()]
            info = learner.train(sample, t_env, episode, w)
            buffer.update_priorities(idx, info["td_errors_abs"] + 1e-6)
    A step = one such iteration.  Phase times from HIP events on the main stream
    (every step); value = learned agent-transitions/s over all ranks."""
    from t2omca_amd.env import VecEnv
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.replay import PrioritizedReplayBuffer
    from t2omca_amd.runner import RolloutRunner
    from t2omca_amd.synthetic import make_args
    A, T, n, B, U = args.agents, args.T, args.envs, args.batch, args.updates_per_rollout
    torch.manual_seed(0)
    margs = make_args(A, device=str(dev))
    agent, mixer = TransformerAgent(None, margs).to(dev), TransformerMixer(margs).to(dev)
    learner = TDLearner(agent, mixer, precision=args.dtype, priorities_to_cpu=False, td_algo=args.td_algo)
    env = VecEnv(n, mec_num=args.mecs, agv_num=A, episode_limit=T, seed=1, device=dev, wire=args.compact_obs)
    env.get_env_info()
    runner = RolloutRunner(agent, env, seed=0, compact_obs=args.compact_obs, precision=args.rollout_precision)
    buf = None
    episode = 0
    marks = []

    def mark(tag):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((tag, ev))

    def iteration(timed):
        nonlocal buf, episode
        if timed:
            mark("rollout")
        eb = runner.run()
        if buf is None:  # capacity: two rollouts of episodes (PyMARL2 keeps buffer_size >= the runner's batch)
            buf = PrioritizedReplayBuffer(eb, 2 * n, T + 1, 0.6, 0.4, 10 ** 7, device=dev, seed=rank)
        if timed:
            mark("insert")
        buf.insert_episode_batch(eb)
        episode += n
        for _ in range(U):
            if timed:
                mark("sample")
            sample, idx, w = buf.sample(B, runner.t_env)
            sample = sample[:, :sample.max_t_filled()]
            if timed:
                mark("train")
            info = learner.train(sample, runner.t_env, episode, per_weight=w)
            if timed:
                mark("update_priorities")
            buf.update_priorities(idx, info["td_errors_abs"].flatten(), add=1e-6)
        if timed:
            mark("end")

    for _ in range(args.warmup):
        iteration(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        iteration(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    phases = {}
    for (tag, e0), (_, e1) in zip(marks, marks[1:]):
        if tag != "end":
            phases[tag] = phases.get(tag, 0.0) + e0.elapsed_time(e1)
    phases = {k: round(v / args.steps, 3) for k, v in phases.items()}  # ms per iteration
    learned = world * args.steps * U * B * T * A
    out = {"metric": "learned agent-transitions/sec of the closed driver loop (rollout -> insert -> PER sample -> "
                     "TD update -> update_priorities)",
           "value": learned / elapsed, "unit": "agent-transitions/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": f"{args.dtype} learner, {args.rollout_precision} rollout agent, fp64 env",
           "data": "simulated (VecEnv, env_spec stand-ins) + device PER replay",
           "config": {"workload": f"configs[4] feeding the learner: {n} envs/GPU x {A} AGVs x {args.mecs} MEC, "
                                  f"episode {T} steps; per rollout {U} TD updates of {B} PER-sampled episodes "
                                  f"(replay capacity {2 * n})" + (", compact obs" if args.compact_obs else ""),
                      "global_envs": n * world, "agents": A, "learner_batch": B, "updates_per_rollout": U,
                      "parallelism": f"dp{world}"},
           "env_steps_per_s": world * args.steps * n * T / elapsed,
           "collected_agent_transitions_per_s": world * args.steps * n * T * A / elapsed,
           "phase_ms_per_step": phases}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        hc = host_cpus()
        ne = 4
        r, es, t_roll, t_train = _cpu_loop_rate(A, args.mecs, T, ne, hc["usable"])
        out["cpu_baseline"] = {"value": r, "unit": "agent-transitions/s", "cores": hc["usable"], "kind": "port",
                               "env_steps_per_s": es,
                               "sample": f"one cycle on {ne} envs x {A} AGVs x {args.mecs} MEC x T={T}: rollout "
                                         f"(torch-CPU agent, eps-greedy, numpy env; {t_roll:.2f} s) then one TD "
                                         f"update on those {ne} episodes (oracle/ref_learner fp32 + Adam; "
                                         f"{t_train:.2f} s), {hc['usable']} threads (host_cpus)",
                               "host_cpus": hc}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rollout_tag(args):
    return (f"rollout_n{args.envs}_t{args.T}_a{args.agents}_m{args.mecs}" + ("_wire" if args.compact_obs else "")
            + ("_bf16" if args.rollout_precision == "bf16" else ""))


def expand_bench(args, world, rank, dev):
    """rebuild a replay batch's dense obs from the compact wire
    format (t2o_obs_expand), records from a real VecEnv rollout of B envs."""
    from t2omca_amd import ops
    from t2omca_amd.env import VecEnv
    A, T, B = args.agents, args.T, args.batch
    env = VecEnv(B, mec_num=args.mecs, agv_num=A, episode_limit=T, seed=1 + rank, device=dev, wire=True)
    env.get_env_info()
    wire = torch.empty(T + 1, B, A, 4, dtype=torch.int32, device=dev)
    env.reset(dest={"wire": wire[0]})
    snap_n, snap = env.snap_n.clone(), env.snap.clone()
    g = torch.Generator(device=dev).manual_seed(rank)
    for t in range(T):
        acts = torch.randint(0, env.n_actions, (B, A), device=dev, generator=g)
        env.step(acts, dest={"wire": wire[t + 1]})
    wire_b = wire.transpose(0, 1).contiguous()
    out = torch.empty(B, T + 1, A, 9 * A, device=dev)
    for _ in range(args.warmup):
        ops.obs_expand(wire_b, snap_n, snap, out=out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    for _ in range(args.steps):
        ops.obs_expand(wire_b, snap_n, snap, out=out)
    ev[1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev[0].elapsed_time(ev[1]) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    rows = B * (T + 1) * A
    dense_b, wire_bytes = rows * 9 * A * 4, rows * 16 + B * (8 + 2 * 9 * A * 8)
    achieved = (dense_b + wire_bytes) / (kern_ms * 1e-3) / 1e9
    res = {"metric": "agent-obs rows/sec rebuilt from the compact wire format (t2o_obs_expand)",
           "value": world * rows * args.steps / elapsed, "unit": "agent-obs rows/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64 normaliser, f32 out",
           "data": "simulated (VecEnv wire records, env_spec stand-ins)",
           "config": {"workload": f"SURVEY §8 f3: dense obs of {B} episodes x (T+1)={T + 1} x {A} AGVs "
                                  f"({args.mecs} MEC) from wire records + normaliser snapshots",
                      "global_batch": B * world, "seq_len": T, "agents": A},
           "storage": {"dense_obs_bytes": dense_b, "wire_bytes": wire_bytes, "ratio": dense_b / wire_bytes},
           "roofline": {"bound": "hbm", "kernel": "obs_expand", "achieved": achieved, "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                        "algorithmic_bytes_per_launch": dense_b + wire_bytes, "avg_launch_ms": kern_ms,
                        "note": "the per-feature normaliser is a serial fp64 chain of (T+1)*A updates "
                                "(bit-exact order), so the kernel is latency-bound below the HBM roof"}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dropin_bench(args, world, rank, dev):
    """The drop-in modules called as the reference calls them: one
    TransformerAgent.forward per env step for every env of the runner
    (parallel_runner.py:121 -> transf_agent.py:54-76) and one
    TransformerMixer.forward per step (n_transf_mixer.py:55-91), under no_grad.
    Times the cached path (the pack is rebuilt only when the weights change,
    modules._PackCache) against re-packing on every call (the round-2 behaviour:
    concatenate + pack per call), and the bare kernel launch, at the runner's
    small batch and at --envs."""
    from t2omca_amd import ops
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args
    A, E = args.agents, 32
    torch.manual_seed(0)
    margs = make_args(A, device=str(dev))
    agent, mixer = TransformerAgent(None, margs).to(dev), TransformerMixer(margs).to(dev)
    calls = max(args.steps, 1) * 20

    def per_call_ms(fn):
        for _ in range(max(args.warmup, 1) * 5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / calls * 1e3

    sizes = {}
    for n in sorted({8, args.envs}):
        g = torch.Generator(device=dev).manual_seed(n)
        obs = torch.randn(n, A, 9 * A, device=dev, generator=g)
        hid = torch.zeros(n, A, E, device=dev)
        qv = torch.randn(n, 1, A, device=dev, generator=g)
        st = torch.randn(n, 8 * A, device=dev, generator=g)
        hw = torch.zeros(n, 3, E, device=dev)
        res = {}
        with torch.no_grad():
            res["agent_cached_ms"] = per_call_ms(lambda: agent(obs, hid))
            res["agent_repack_ms"] = per_call_ms(lambda: (agent._pack_cache.invalidate(), agent(obs, hid)))
            _, _, pack = agent._pack_cache.get(agent, agent.shape)
            o4, h0 = obs.view(n, 1, A, 9 * A), hid.reshape(n * A, E)
            res["agent_kernel_only_ms"] = per_call_ms(lambda: ops.agent_unroll_fwd(agent.shape, pack, o4, h0_on=h0))
            res["mixer_cached_ms"] = per_call_ms(lambda: mixer(qv, hid, hw, st, None))
            res["mixer_repack_ms"] = per_call_ms(lambda: (mixer._pack_cache.invalidate(), mixer(qv, hid, hw, st, None)))
        sizes[str(n)] = {k: round(v, 5) for k, v in res.items()}
    big = sizes[str(args.envs)]
    out = {"metric": "agent forward calls/sec through the drop-in module (one env step of every env)",
           "value": 1e3 / big["agent_cached_ms"], "unit": "calls/s", "n_gpus": 1, "steps": calls,
           "warmup": max(args.warmup, 1) * 5, "ms_per_step": big["agent_cached_ms"], "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic (N(0,1) obs, zero hidden)",
           "config": {"workload": f"TransformerAgent.forward / TransformerMixer.forward per env step, {A} AGVs, "
                                  f"batch = envs (8: a runner's parallel envs; {args.envs}: configs[4]'s envs)",
                      "agents": A, "envs": sorted(int(k) for k in sizes)},
           "per_call_ms": sizes,
           "pack_rebuilds": {"agent": agent._pack_cache.rebuilds, "mixer": mixer._pack_cache.rebuilds}}
    if rank == 0:
        print(json.dumps(out), flush=True)


def mixer_decoupled(learner, B):
    from t2omca_amd import ops
    return int(ops.lib().t2o_mixer_split(ops.ctypes.byref(learner.sm.layout()), int(B))) == 1


def dist_info(world, rank_seconds, steps):
    """What the process group itself reports (so a SCALE line shows that RCCL saw N
    ranks, not only what WORLD_SIZE said) and every rank's ms per step."""
    ms = [t / steps * 1e3 for t in rank_seconds]
    up = dist.is_available() and dist.is_initialized()
    return {"world_size": dist.get_world_size() if up else 1, "backend": dist.get_backend() if up else None,
            "env_world_size": world, "devices_visible": torch.cuda.device_count(),
            "rank_ms_per_step": {"max": max(ms), "min": min(ms), "per_rank": [round(v, 4) for v in ms]}}


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, n, port):
    """The command that runs this bench as `n` ranks, one process per GPU, over
    torch.distributed.run on 127.0.0.1 (the driver's own N > 1 invocation)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def needs_launch(args, environ):
    """`--gpus N` (N > 1) started as a plain process: this process starts the N
    ranks itself instead of timing one GPU."""
    return args.gpus > 1 and "WORLD_SIZE" not in environ


def launch(args, argv):
    """Run the N ranks as child processes (nothing in this parent has touched the
    GPU: torch.cuda.device_count() does not initialise it on this image) and exit
    with their status.  Each child binds cuda:<LOCAL_RANK>; rank 0 prints the line."""
    import subprocess
    backend = os.environ.get("T2O_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and ndev < args.gpus:
        sys.exit(f"bench.py --gpus {args.gpus}: only {ndev} HIP devices visible (RCCL needs one GPU per rank; "
                 f"T2O_DIST_BACKEND=gloo rehearses the ranks on fewer devices)")
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    r = subprocess.run(launcher_cmd(argv, args.gpus, free_port()), env=env)
    sys.exit(r.returncode)


def main():
    args = parse()
    if args.print_workload_tag:
        print(workload_tag(args))
        return
    if needs_launch(args, os.environ):
        return launch(args, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; reporting the real world size",
              file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # T2O_DIST_BACKEND=gloo rehearses the multi-rank path on a box with fewer GPUs
    # than ranks (ranks share devices round-robin); the default is RCCL, one GPU per rank
    backend = os.environ.get("T2O_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.perfmodel import (ref_order_flops_per_transition, ref_order_kernel_flops, td_tape_bytes,
                                      td_update_bytes,
                                      td_update_flops)
    from t2omca_amd.synthetic import make_args, make_batch

    A, T, B = args.agents, args.T, args.batch
    if args.mode == "rollout":
        return rollout_bench(args, world, rank, dev)
    if args.mode == "expand":
        return expand_bench(args, world, rank, dev)
    if args.mode == "dropin":
        return dropin_bench(args, world, rank, dev)
    if args.mode == "loop":
        return loop_bench(args, world, rank, dev)
    def make_learner(precision, agents=A):
        torch.manual_seed(0)
        margs = make_args(agents, device=str(dev), qmix_pos_func=args.qmix_pos_func)
        agent = TransformerAgent(None, margs).to(dev)
        mixer = TransformerMixer(margs).to(dev)
        pipe = {"0": False, "1": True}.get(os.environ.get("T2O_PIPELINE", "auto"), "auto")
        return TDLearner(agent, mixer, target_update_interval=10 ** 9, precision=precision,
                         overlap=not args.serial, priorities_to_cpu=args.priorities == "cpu",
                         td_algo=args.td_algo, contract=args.contract, pipeline=pipe,
                         pipeline_ranges=int(os.environ.get("T2O_PIPELINE_RANGES", "6")))

    learner = make_learner(args.dtype)
    batch, w = make_batch(B, T, A, seed=1 + rank, device=dev)
    # which kernels run (include/t2omca.h t2o_layout_instance): the runtime-shaped
    # generic kernels compute in fp32 whatever precision is asked, and say so
    kernels = {"agent": learner.sa.instance, "mixer": learner.sm.instance}
    dtype = "fp32" if "generic" in kernels.values() else args.dtype
    if args.mode == "forward":
        from t2omca_amd import ops
        act = batch["actions"][..., 0]
        ops.pack_params(learner.sa, learner.params[:learner.na], learner.pack_a)
        ops.pack_params(learner.sm, learner.params[learner.na:], learner.pack_m)

        def step(i):
            q, h = ops.agent_unroll_fwd(learner.sa, learner.pack_a, batch["obs"])
            ops.mixer_unroll_fwd(learner.sm, learner.pack_m, batch["state"], h, qmode_on=1, q_on=q, actions=act,
                                 T_on=T, want_xout=False)
    else:
        # the driver's closed step (per_run.py:224-238): the update, then the sampled
        # episodes' priorities back into the replay buffer.  --priorities device: the
        # device-resident buffer's update_priorities (t2o_per_update) on the device
        # |TD errors|; cpu: the learner copies them to the host (4 KB + a sync) and the
        # host list goes through the same call.  The buffer is sized like PyMARL2's
        # default (5000 episodes); the batch's episode indices are a fixed sample.
        from t2omca_amd.replay import PrioritizedReplayBuffer
        buf = PrioritizedReplayBuffer({"filled": torch.zeros(1, T + 1, 1, device=dev)}, max(5000, B), T + 1,
                                      0.6, 0.4, 10 ** 6, device=dev, seed=rank)
        idx = torch.randperm(max(5000, B), generator=torch.Generator().manual_seed(rank))[:B].to(dev)

        def make_step(lr):
            def step(i):
                info = lr.train(batch, 0, i, per_weight=w)
                # per_run.py:237-238's `+ 1e-6`, applied inside the priority kernel
                buf.update_priorities(idx, info["td_errors_abs"].flatten(), add=1e-6)
            return step
        step = make_step(learner)

    def timed(step, timer=None, every=0):
        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            learner.timer = timer if every > 0 and i % every == 0 else None
            if learner.timer is not None:
                timer.updates += 1
            step(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        learner.timer = None
        if world > 1:
            # every rank's time (the line reports the max; the spread shows the ranks ran together)
            ts = [torch.zeros(1, device=dev) for _ in range(world)]
            dist.all_gather(ts, torch.tensor([el], device=dev))
            per_rank = [float(t) for t in ts]
            el = max(per_rank)
        else:
            per_rank = [el]
        rank_times.clear()
        rank_times.extend(per_rank)
        return el

    rank_times = []

    timer = KernelTimer()
    elapsed = timed(step, timer, args.kernel_timer_every)
    if args.mode == "forward":
        value = world * B * (T + 1) * A * args.steps / elapsed
        out = {"metric": "agent-transitions/sec for agent+mixer forward (inference over a replay batch)",
               "value": value, "unit": "agent-transitions/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": dtype,
               "data": "synthetic (SURVEY.md §8 d distributions, resident in HBM)",
               "config": {"workload": f"configs[1]-style: online agent (t=0..T) + online mixer (t<T) unroll, "
                                      f"{A} AGVs, batch {B} episodes/GPU x T={T}",
                          "global_batch": B * world, "seq_len": T, "agents": A, "kernels": kernels}}
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    transitions = world * B * T * A * args.steps
    value = transitions / elapsed
    # per update: a pipelined update (TDLearner._pipelined) runs each recurrence in
    # step ranges on two streams, so its kernels' sums overlap in time
    kern = {k: sum(v) / max(1, timer.updates) for k, v in timer.durations().items()}
    flops = td_update_flops(B, T, A)
    ref_flops = ref_order_kernel_flops(B, T, A)
    bytes_ = td_update_bytes(B, T, A, elem=2 if args.dtype == "bf16" else 4)
    tape_ = td_tape_bytes(B, T, A, elem=2 if args.dtype == "bf16" else 4)
    # dominant kernel: the longest of the four network kernels on the critical path
    # (the tape contractions are part of a backward; mixer_dw runs on a side stream)
    dom = max(ref_flops, key=lambda k: kern.get(k, 0.0))
    dom_ms = kern.get(dom, float("nan"))
    peak_tf = PEAK_BF16_TFLOPS if dtype == "bf16" else PEAK_FP32_TFLOPS
    # SURVEY.md §8(d) basis: the reference-order necessary FLOPs of the kernel's share
    achieved = ref_flops[dom] / (dom_ms * 1e-3) / 1e12
    ms_step = elapsed / args.steps * 1e3
    upd_flops = ref_order_flops_per_transition(A) * B * T * A
    dw = "dw_pair" if "dw_pair" in kern else {"agent_bwd": "agent_dw", "mixer_bwd": "mixer_dw"}.get(dom)
    out = {
        "metric": "agent-transitions/sec for TD update fwd+bwd (whole node)",
        "value": value,
        "unit": "agent-transitions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (SURVEY.md §8 d distributions, seeded per rank, resident in HBM)",
        "config": {"workload": f"{train_config_name(A, B, T)}: full TD update fwd+bwd+Adam, {A} AGVs, "
                               f"batch {B} episodes/GPU x T={T}",
                   "global_batch": B * world, "seq_len": T, "agents": A, "emb": 32, "heads": 3, "depth": 2,
                   "parallelism": f"dp{world}", "priorities": args.priorities, "kernels": kernels,
                   "mixer_head": args.qmix_pos_func,
                   # small batches: the multi-tile mixer's recurrence decoupled from its other
                   # rows (t2o_mixer_split) and the two networks' recurrences in step ranges
                   # on two streams (TDLearner._pipelined)
                   "mixer_decoupled": mixer_decoupled(learner, B), "pipelined": learner._pipelined(B)},
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": achieved, "peak": peak_tf,
                     "unit": "TFLOP/s", "frac": achieved / peak_tf, "traffic": traffic_for(dom, workload_tag(args)),
                     "basis": "SURVEY.md §8(d) reference-order necessary FLOPs of the kernel's share "
                              "(perfmodel.ref_order_kernel_flops)",
                     "algorithmic_flops_per_launch": ref_flops[dom],
                     "algorithmic_bytes_per_launch": bytes_.get(dom),
                     "tape_bytes_per_update": tape_,
                     "avg_launch_ms": dom_ms,
                     "incl_tape_contraction": None if dw is None or dw not in kern else {"contraction": dw,
                         "ms": dom_ms + kern[dw],
                         "frac": ref_flops[dom] / ((dom_ms + kern[dw]) * 1e-3) / 1e12 / peak_tf,
                         **({"note": "mixer_dw is issued on the side stream as the agent BPTT starts: its "
                                     "event span includes waiting for that kernel's waves to drain, so this "
                                     "is an upper bound (run --serial for the contraction alone)"}
                            if dw == "mixer_dw" and args.contract == "side" and not args.serial else {})},
                     "executed_algorithm": {"flops_per_launch": flops[dom],
                                            "frac": flops[dom] / (dom_ms * 1e-3) / 1e12 / peak_tf},
                     "whole_update": {"flops": upd_flops, "ms": ms_step,
                                      "achieved": upd_flops / (ms_step * 1e-3) / 1e12,
                                      "frac": upd_flops / (ms_step * 1e-3) / 1e12 / peak_tf},
                     # every network kernel on the same basis (the two BPTT kernels run within a
                     # few µs of each other, so which one is "dominant" flips between runs)
                     "per_kernel": {k: {"avg_launch_ms": kern[k],
                                        "achieved": ref_flops[k] / (kern[k] * 1e-3) / 1e12,
                                        "frac": ref_flops[k] / (kern[k] * 1e-3) / 1e12 / peak_tf}
                                    for k in sorted(ref_flops) if k in kern}},
        "kernels_ms": {k: round(v, 4) for k, v in sorted(kern.items())},
        "distributed": dist_info(world, rank_times, args.steps),
        "flops_per_transition": {"executed_algorithm": sum(flops.values()) / (B * T * A),
                                 "reference_order": ref_order_flops_per_transition(A)},
    }
    if dtype == "bf16" and args.fp32_companion:
        # the same workload at the reference's own precision (fp32 MFMA operands)
        lr32 = make_learner("fp32")
        el32 = timed(make_step(lr32))
        out["fp32_companion"] = {"value": transitions / el32, "unit": "agent-transitions/s",
                                 "ms_per_step": el32 / args.steps * 1e3, "dtype": "fp32"}
        del lr32
    if world == 1 and args.config_companions and (A, B, T) == (8, 1024, 60):
        # an fp32 16-AGV TD update (the reference's precision at the
        # 16-AGV scenario, 1024 episodes x T=150) in the same line; timed as above
        A2, B2, T2, s2 = 16, 1024, 150, 3
        lr16 = make_learner("fp32", agents=A2)
        b16, w16 = make_batch(B2, T2, A2, seed=1 + rank, device=dev)
        for i in range(1 + s2):
            if i == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            lr16.train(b16, 0, i, per_weight=w16)
        torch.cuda.synchronize()
        el16 = time.perf_counter() - t0
        out["configs"] = {"a16_fp32": {
            "workload": f"TD update fwd+bwd+Adam, {A2} AGVs, batch {B2} episodes x T={T2}, fp32 MFMA operands",
            "value": B2 * T2 * A2 * s2 / el16, "unit": "agent-transitions/s", "ms_per_step": el16 / s2 * 1e3,
            "steps": s2, "warmup": 1, "kernels": {"agent": lr16.sa.instance, "mixer": lr16.sm.instance}}}
        del lr16, b16, w16
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
