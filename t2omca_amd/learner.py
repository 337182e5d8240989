"""GPU TD update with the reference driver's learner contract.

per_run.py:224-238 calls

    info = learner.train(episode_sample, runner.t_env, episode, weights)
    buffer.update_priorities(idx, (info["td_errors_abs"].flatten() + 1e-6).numpy().tolist())

The reference's learner module is absent, so the semantics are
the PyMARL2 NQLearner ones (oracle/ref_learner.py restates them on the CPU;
parity-unpinned beyond the agent/mixer arithmetic).  One ``train`` call is a
fixed sequence of HIP launches on the current stream (no host sync until the
priorities are copied out):

  pack(online agent, online mixer)                 t2o_pack_params x2
  agent unroll fwd, online + target, t = 0..T      t2o_agent_unroll_fwd (1 launch)
  mixer unroll fwd, online (chosen Q, t < T) +
        target (double-Q, t <= T)                  t2o_mixer_unroll_fwd (1 launch)
  TD(λ) targets, loss, dL/dQtot, priorities        t2o_td_loss
  mixer BPTT -> dL/dq_chosen, dL/dhidden           t2o_mixer_unroll_bwd
  mixer tape contraction + slab sum + unfold       side stream, issued here; it
                                                   runs as the agent BPTT's waves drain
  agent BPTT, its tape contraction, slab sum,      t2o_agent_unroll_bwd, ...
  unfold into the reference parameter order        t2o_unpack_grads
  [data parallel: all_reduce of the flat grad + Σ mask over RCCL in two
   halves, the mixer's from the side stream; neither runs under a BPTT kernel,
   whose waves hold every SIMD]
  (contract="pair": both tapes in one launch after the agent BPTT, one all-reduce)
  clip_grad_norm_ + Adam                           t2o_adam_step
"""
import dataclasses
import os

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from .distributed import allreduce_async, broadcast_state, wait_all


def _bind_flat(modules, device):
    """Move the modules' parameters into one flat fp32 buffer (views)."""
    params = [p for m in modules for p in m.parameters()]
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, device=device, dtype=torch.float32)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.detach().reshape(-1))
        p.data = flat[off:off + k].view_as(p)
        off += k
    return flat


class TDLearner:
    def __init__(self, agent, mixer, *, lr=1e-3, gamma=0.99, td_lambda=0.6, grad_norm_clip=10.0,
                 target_update_interval=200, optim_betas=(0.9, 0.999), optim_eps=1e-8, weight_decay=0.0,
                 detach_mixer_hidden=False, process_group=None, priorities_to_cpu=True, precision="fp32",
                 overlap=True, td_algo="auto", contract="side", pipeline="auto", pipeline_ranges=6):
        # options first (a bad value fails here, not inside the first train())
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        if contract not in ("pair", "side"):
            raise ValueError("contract must be 'pair' or 'side'")
        if td_algo not in ops.TD_ALGOS:
            raise ValueError(f"td_algo must be one of {sorted(ops.TD_ALGOS)}, got {td_algo!r}")
        if pipeline not in ("auto", True, False) or int(pipeline_ranges) < 1:
            raise ValueError("pipeline must be 'auto', True or False and pipeline_ranges >= 1")
        if pipeline is True and (contract == "pair" or not overlap):
            raise ValueError("pipeline=True runs the mixer's contraction on the side stream: it needs "
                             "contract='side' and overlap=True")
        dev = next(agent.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("TDLearner needs the modules on a HIP device (no CPU fallback)")
        self.agent, self.mixer = agent, mixer
        # bf16: MFMA operands (weights, activations entering a matrix product) in
        # bf16; accumulation, LayerNorm, softmax, recurrent state, TD targets, grads
        # and the Adam master weights stay fp32
        prec = 1 if precision == "bf16" else 0
        self.precision = precision
        self.sa = dataclasses.replace(agent.shape, prec=prec)
        self.sm = dataclasses.replace(mixer.shape, prec=prec)
        self.na, self.nm = self.sa.n_params, self.sm.n_params
        assert self.na == sum(p.numel() for p in agent.parameters())
        assert self.nm == sum(p.numel() for p in mixer.parameters())
        self.device = dev
        self.params = _bind_flat([agent, mixer], dev)
        self.grad = torch.zeros(self.na + self.nm + 1, device=dev)  # last slot: Σ mask
        self.exp_avg = torch.zeros_like(self.params)
        self.exp_avg_sq = torch.zeros_like(self.params)
        self.target_params = self.params.clone()
        self.pg = process_group
        # data parallel: every replica starts from rank 0's parameters (ranks that
        # initialised with different seeds would otherwise drift apart silently)
        broadcast_state([self.params, self.target_params], self.pg)
        self._params_written()
        self.adam_ws = torch.empty(int(ops.lib().t2o_adam_workspace_floats()), device=dev)
        self.grad_norm = torch.zeros(1, device=dev)
        self.lr, self.betas, self.eps, self.wd = lr, optim_betas, optim_eps, weight_decay
        self.gamma, self.td_lambda, self.clip = gamma, td_lambda, grad_norm_clip
        self.target_update_interval = target_update_interval
        self.detach_mixer_hidden = detach_mixer_hidden
        self.priorities_to_cpu = priorities_to_cpu
        self.overlap = overlap  # mixer tape contraction on a side stream beside the agent BPTT
        self.td_algo = td_algo  # ops.TD_ALGOS
        # "side" (default): the mixer's tape contraction on the side stream, issued
        # before the agent BPTT — it cannot run beside the BPTT (whose waves hold
        # every SIMD) but its workgroups take the CUs the BPTT's last waves free;
        # "pair": both contractions in one launch after the agent BPTT, measured
        # 15 us slower per update (profiles/r4_b/: 2.455 vs 2.438 ms)
        self.contract = contract
        # small replay batches: the agent and the (decoupled) mixer recurrences run
        # side by side on two streams in step ranges (_pipelined).  "auto": wherever
        # the layout and batch allow it (never with contract="pair", which contracts
        # both tapes in one launch after the agent BPTT); True: required — train()
        # raises when the update cannot be pipelined; False: never
        self.pipeline, self.pipeline_ranges = pipeline, int(pipeline_ranges)
        self.step_count = 0
        self.last_target_update_episode = 0
        self.timer = None   # optional callable(tag) recording HIP events around the big kernels
        self.pack_a = torch.empty(self.sa.layout().pack_floats, device=dev)
        self.pack_m = torch.empty(self.sm.layout().pack_floats, device=dev)
        self.pack_at = torch.empty_like(self.pack_a)
        self.pack_mt = torch.empty_like(self.pack_m)
        self._pack_targets()
        self._slabs = {}

    # -- parameters --------------------------------------------------------
    def _params_written(self):
        """The Adam kernel and the replica broadcasts write the modules' parameters
        through raw pointers, which autograd's version counters do not see: drop the
        modules' cached kernel packs (modules._PackCache) so their next per-step
        forward re-packs."""
        for m in (self.agent, self.mixer):
            cache = getattr(m, "_pack_cache", None)
            if cache is not None:
                cache.invalidate()

    def agent_params(self, target=False):
        src = self.target_params if target else self.params
        return src[:self.na]

    def mixer_params(self, target=False):
        src = self.target_params if target else self.params
        return src[self.na:]

    def _pack_targets(self):
        ops.pack_params(self.sa, self.target_params[:self.na], self.pack_at)
        ops.pack_params(self.sm, self.target_params[self.na:], self.pack_mt)

    def update_targets(self):
        self.target_params.copy_(self.params)
        self._pack_targets()

    def _world(self):
        if self.pg is not None or (dist.is_available() and dist.is_initialized()):
            return dist.get_world_size(self.pg)
        return 1

    def _buf(self, key, shape):
        t = self._slabs.get(key)
        n = 1
        for d in shape:
            n *= d
        if t is None or t.numel() < n:
            t = torch.empty(n, device=self.device)
            self._slabs[key] = t
        return t[:n].view(shape)

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        return self._side

    def _slab(self, key, n):
        t = self._slabs.get(key)
        if t is None or t.numel() < n:
            t = torch.empty(n, device=self.device)
            self._slabs[key] = t
        return t

    # -- checkpoints (per_run.py:159-189 load, :265-279 save) -----------------
    def cuda(self):
        """per_run.py:156 calls learner.cuda(); the learner already lives on its HIP device."""
        return self

    def _optimiser_view(self):
        """A torch.optim.Adam over the modules' parameters (mac then mixer, the
        order of a PyMARL2 NQLearner's optimiser) carrying this learner's moments,
        so opt.th is a standard Adam state_dict."""
        params = list(self.agent.parameters()) + list(self.mixer.parameters())
        opt = torch.optim.Adam(params, lr=self.lr, betas=self.betas, eps=self.eps, weight_decay=self.wd)
        off = 0
        for p in params:
            k = p.numel()
            if self.step_count:
                opt.state[p] = {"step": torch.tensor(float(self.step_count)),
                                "exp_avg": self.exp_avg[off:off + k].view_as(p),
                                "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p)}
            off += k
        return opt

    def save_models(self, path):
        """PyMARL layout: {path}/agent.th, mixer.th (reference state_dict keys) and
        opt.th (torch Adam state_dict)."""
        torch.save(self.agent.state_dict(), os.path.join(path, "agent.th"))
        torch.save(self.mixer.state_dict(), os.path.join(path, "mixer.th"))
        torch.save(self._optimiser_view().state_dict(), os.path.join(path, "opt.th"))

    def load_models(self, path):
        """Inverse of save_models; also takes checkpoints written by the reference
        framework.  As PyMARL2's NQLearner does, the target agent is reloaded from
        agent.th and the target mixer is left as it is; opt.th is optional."""
        def load(name):
            return torch.load(os.path.join(path, name), map_location=self.device, weights_only=True)
        with torch.no_grad():
            self.agent.load_state_dict(load("agent.th"))  # copies into the flat-buffer views
            self.mixer.load_state_dict(load("mixer.th"))
            self.target_params[:self.na].copy_(self.params[:self.na])
        if not os.path.exists(os.path.join(path, "opt.th")):
            self._sync_replicas()
            return
        opt = self._optimiser_view()
        opt.load_state_dict(load("opt.th"))
        off, steps = 0, set()
        for p in list(self.agent.parameters()) + list(self.mixer.parameters()):
            k = p.numel()
            st = opt.state.get(p)
            if st:
                self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(float(st["step"])))
            off += k
        if len(steps) > 1:
            raise ValueError(f"opt.th: parameters carry different Adam step counts {sorted(steps)}")
        self.step_count = steps.pop() if steps else 0
        self._sync_replicas()

    def _sync_replicas(self):
        """Data parallel: rank 0's params, target params, Adam moments and step
        count on every rank (after a checkpoint load), then re-pack the targets."""
        if self._world() > 1:
            step = torch.tensor([float(self.step_count)], device=self.device)
            broadcast_state([self.params, self.target_params, self.exp_avg, self.exp_avg_sq, step], self.pg)
            self.step_count = int(step.item())
        self._params_written()
        self._pack_targets()

    # -- the TD update -------------------------------------------------------
    def _pipelined(self, B):
        """Run the update's recurrences in step ranges on two streams?  Only where the
        mixer runs decoupled (a multi-tile mixer at a small batch, t2o_mixer_split)
        and the agent BPTT is the pipelined kernel (depth 2), which take ranges."""
        if self.pipeline is False or self.contract == "pair" or self.sa.D != 2 or self.sa.generic or self.sm.generic:
            return False
        lib = ops.lib()
        if int(lib.t2o_agent_bwd_ranges(ops.ctypes.byref(self.sa.layout()), 1)) != 1:
            return False  # (e.g. T2O_AGENT_BWD=single: the one-wave BPTT takes only the whole unroll)
        return int(lib.t2o_mixer_split(ops.ctypes.byref(self.sm.layout()), int(B))) == 1

    def _ranges(self, n):
        """pipeline_ranges step ranges covering [0, n), in order."""
        k = min(self.pipeline_ranges, n)
        cuts = [round(i * n / k) for i in range(k + 1)]
        return [(cuts[i], cuts[i + 1]) for i in range(k) if cuts[i] < cuts[i + 1]]

    def train(self, batch, t_env=0, episode_num=0, per_weight=None):
        if "obs" in _keys(batch):
            obs = batch["obs"]
        else:  # compact wire-format batch: dense obs rebuilt on the device
            wire = batch["obs_wire"]
            b, T1, A = wire.shape[:3]
            obs = ops.obs_expand(wire, batch["obs_nrm_n"], batch["obs_nrm"],
                                 out=self._buf("obs", (b, T1, A, 9 * A)))
        # the mixer's tokens: the state (state_entity_mode) or every agent's obs
        # entities (n_transf_mixer.py:60-63)
        state = batch["state"] if self.mixer.custom_space else obs.flatten(2)
        actions = batch["actions"]
        avail = batch["avail_actions"]
        B, T1, A, _ = obs.shape
        T = T1 - 1
        dev = self.device
        if avail.dtype != torch.int32:
            avail = avail.int()
        act = actions[..., 0] if actions.dim() == 4 else actions
        if act.dtype != torch.int64:
            act = act.long()
        if act.stride(2) != 1:
            act = act.contiguous()
        reward = batch["reward"][:, :, 0]
        term = batch["terminated"][:, :, 0]  # uint8 / int64 as the EpisodeBatch keeps them: read in place
        filled = batch["filled"][:, :, 0] if "filled" in _keys(batch) else None
        w = None
        if per_weight is not None:
            w = torch.as_tensor(np.asarray(per_weight) if not torch.is_tensor(per_weight) else per_weight,
                                dtype=torch.float32).to(dev).reshape(B).contiguous()

        # the gradient buffer is cleared on the side stream, off the critical path
        # (after the previous update's Adam, which read it)
        main = torch.cuda.current_stream(dev)
        side = self._side_stream() if self.overlap else main
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self.grad.zero_()
            ops.pack_params(self.sm, self.params[self.na:], self.pack_m)  # beside the agent's pack + forward
            mixer_packed = side.record_event()  # (main waits for it before the mixer: grad is clear by then too)
        ops.pack_params(self.sa, self.params[:self.na], self.pack_a)
        hmid = self._buf("hmid", (B, T1, self.sa.D - 1, A, self.sa.E)) if self.sa.D > 1 else None
        piped = self._pipelined(B) and side is not main
        if self.pipeline is True and not piped:
            raise RuntimeError(f"pipeline=True, but this update cannot run in step ranges (layout instance "
                               f"{self.sa.instance}/{self.sm.instance}, {B} episodes: the mixer must run decoupled "
                               f"and the agent BPTT must be the pipelined kernel)")
        mixer_kw = dict(qmode_on=1, actions=act, avail=avail, T_on=T, pack_tg=self.pack_mt, qmode_tg=2, T_tg=T1,
                        timer=self.timer)
        if piped:
            # 1+2 in step ranges: agent range k (main) || mixer recurrence range k-1
            # (side), then every (episode, step)'s mixer rows (side)
            E = self.sa.E
            q_on, q_tg = (self._buf(k, (B, T1, A, self.sa.NA)) for k in ("q_on", "q_tg"))
            h_on, h_tg = (self._buf(k, (B, T1, A, E)) for k in ("h_on", "h_tg"))
            o_on, o_tg = ({"y": self._buf("y" + n, (B, Tn)), "hw": self._buf("hw" + n, (B, Tn, 3, E)),
                           "qv": self._buf("qv" + n, (B, Tn, A)), "xout": self._buf("xo" + n, (B, Tn, A + 3, E)),
                           "xmid": (self._buf("xm" + n, (B, Tn, self.sm.D - 1, A + 3, E)) if n == "on" else None)}
                          for n, Tn in (("on", T), ("tg", T1)))
            # (launchers: each wrapper's arguments converted once, then one C call per
            # range — the host must stay ahead of ranges of ~0.1 ms)
            agent_go = ops.agent_unroll_fwd(self.sa, self.pack_a, obs, pack_tg=self.pack_at, timer=self.timer,
                                            hmid_on=hmid, outs=(q_on, h_on, q_tg, h_tg), launcher=True)
            mixer_go = ops.mixer_unroll_fwd(self.sm, self.pack_m, state, h_on, q_on=q_on, hid_tg=h_tg, q_tg=q_tg,
                                            outs=(o_on, o_tg), launcher=True, **mixer_kw)
            for t0, t1 in self._ranges(T1):
                agent_go(t0, t1)
                agent_done = main.record_event()
                with torch.cuda.stream(side):
                    side.wait_event(agent_done)
                    mixer_go(1, t0, t1)
            with torch.cuda.stream(side):
                mixer_go(2)
            main.wait_stream(side)
        else:
            # 1. agents: online + target over t = 0..T
            q_on, h_on, q_tg, h_tg = ops.agent_unroll_fwd(self.sa, self.pack_a, obs, pack_tg=self.pack_at,
                                                          timer=self.timer, hmid_on=hmid)
            # 2. mixers: online on chosen Q (t < T), target on double-Q (t <= T)
            main.wait_event(mixer_packed)
            o_on, o_tg = ops.mixer_unroll_fwd(self.sm, self.pack_m, state, h_on, q_on=q_on, hid_tg=h_tg, q_tg=q_tg,
                                              **mixer_kw)
        # 3. TD(λ) targets / loss (un-normalised: Σ mask is applied in Adam so the
        #    data-parallel sum over ranks divides by the GLOBAL Σ mask)
        #    (Σ mask also lands in grad[-1] straight from the kernel: grad was cleared
        #    on the side stream before the mixer forward, which waited for it)
        td = ops.td_loss(o_on["y"], o_tg["y"], reward, term, filled, w, gamma=self.gamma,
                         td_lambda=self.td_lambda, mask_sum=1.0, algo=self.td_algo, mask_sum_acc=self.grad[-1:])
        # 4. mixer BPTT (its weight-grad tape is contracted after the agent BPTT)
        tape_m = self._slab("tape_m", ops.tape_floats(self.sm, ops.mixer_tape_tiles(B, T, A, self.sm)))
        tape_a = self._slab("tape_a", ops.tape_floats(self.sa, ops.agent_tape_tiles(B, T, A)))
        slabs_m = self._slab("m", ops.mixer_slab_count(B) * self.sm.layout().grad_total)
        nwork = ops.mixer_work_floats(self.sm, B, T)
        work_m = self._slab("work_m", nwork) if nwork else None
        slabs_a = self._slab("a", ops.agent_slab_count(B, A) * self.sa.layout().grad_total)
        if piped:
            # 4+5 in step ranges: the mixer's parallel part, then per range from the
            # last down its recurrence (side) || the agent BPTT of the range after (main)
            gqv, ghid = self._buf("gqv", (B, T, A)), self._buf("ghid", (B, T, A, self.sm.E))
            carry_m, carry_a = self._buf("carry_m", (B, 3, self.sm.E)), self._buf("carry_a", (B * A, self.sa.E))
            mixer_go = ops.mixer_unroll_bwd(self.sm, self.pack_m, state, h_on, o_on, td["gq"], slabs=slabs_m,
                                            timer=self.timer, tape=tape_m, work=work_m, outs=(gqv, ghid),
                                            carry=carry_m, launcher=True)
            agent_go, _ = ops.agent_unroll_bwd(self.sa, self.pack_a, obs, h_on, gchosen=gqv, actions=act,
                                               gh=None if self.detach_mixer_hidden else ghid, slabs=slabs_a,
                                               timer=self.timer, hmid=hmid, tape=tape_a, gcarry=carry_a,
                                               launcher=True)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                contract_m = mixer_go(1)
            for t_lo, t_hi in reversed(self._ranges(T)):
                with torch.cuda.stream(side):
                    mixer_go(2, t_lo, t_hi)
                    mixer_done = side.record_event()
                main.wait_event(mixer_done)
                contract_a = agent_go(t_lo, t_hi)
            with torch.cuda.stream(side):
                gm = contract_m()
                ops.unpack_grads(self.sm, self.params[self.na:], gm, self.grad[self.na:self.na + self.nm])
                work_m_ = allreduce_async(self.grad[self.na:], self.pg)
            ga = contract_a()
            ops.unpack_grads(self.sa, self.params[:self.na], ga, self.grad[:self.na])
            work_a = allreduce_async(self.grad[:self.na], self.pg)
            main.wait_stream(side)
            wait_all((work_m_, work_a))
            return self._finish(episode_num, td, {"y": o_on["y"].clone()})  # (o_on: reused buffers)
        contract_m, gqv, ghid, _ = ops.mixer_unroll_bwd(self.sm, self.pack_m, state, h_on, o_on, td["gq"],
                                                        slabs=slabs_m, timer=self.timer, tape=tape_m,
                                                        defer_contract=True, work=work_m)
        gh = None if self.detach_mixer_hidden else ghid
        if self.contract == "pair":
            # 5. agent BPTT (grads of the chosen Q and, unless detached, of the hidden
            #    states), then both tapes contracted in one launch
            contract_a, _ = ops.agent_unroll_bwd(self.sa, self.pack_a, obs, h_on, gchosen=gqv, actions=act, gh=gh,
                                                 slabs=slabs_a, timer=self.timer, hmid=hmid, tape=tape_a,
                                                 defer_contract=True)
            gm, ga = ops.tape_contract_pair(contract_m, contract_a, timer=self.timer)
            # 6. grads in reference parameter order; data parallel: one all-reduce of
            #    [agent grads, mixer grads, Σ mask] (336 KB at the default network)
            ops.unpack_grads(self.sm, self.params[self.na:], gm, self.grad[self.na:self.na + self.nm])
            ops.unpack_grads(self.sa, self.params[:self.na], ga, self.grad[:self.na])
            wait_all((allreduce_async(self.grad, self.pg),))
        else:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                gm = contract_m()
                ops.unpack_grads(self.sm, self.params[self.na:], gm, self.grad[self.na:self.na + self.nm])
                work_m = allreduce_async(self.grad[self.na:], self.pg)
            ga, _ = ops.agent_unroll_bwd(self.sa, self.pack_a, obs, h_on, gchosen=gqv, actions=act, gh=gh,
                                         slabs=slabs_a, timer=self.timer, hmid=hmid, tape=tape_a)
            ops.unpack_grads(self.sa, self.params[:self.na], ga, self.grad[:self.na])
            work_a = allreduce_async(self.grad[:self.na], self.pg)
            main.wait_stream(side)
            wait_all((work_m, work_a))
        return self._finish(episode_num, td, o_on)

    def _finish(self, episode_num, td, o_on):
        # 7. clip + Adam
        self.step_count += 1
        ops.adam_step(self.params, self.grad[:-1], self.exp_avg, self.exp_avg_sq, self.step_count, lr=self.lr,
                      betas=self.betas, eps=self.eps, weight_decay=self.wd, max_grad_norm=self.clip,
                      workspace=self.adam_ws, grad_div=self.grad[-1:], grad_norm_out=self.grad_norm)
        self._params_written()
        if (episode_num - self.last_target_update_episode) / self.target_update_interval >= 1.0:
            self.update_targets()
            self.last_target_update_episode = episode_num
        prio = td["prio"]
        info = {"td_errors_abs": prio.cpu() if self.priorities_to_cpu else prio,
                "loss_sum": td["loss"][0:1], "mask_sum": td["loss"][1:2], "grad_norm": self.grad_norm,
                "qtot": o_on["y"], "targets": td["targets"]}
        return info


def _keys(batch):
    try:
        return batch.keys()
    except AttributeError:
        return getattr(batch, "scheme", {}).keys()
