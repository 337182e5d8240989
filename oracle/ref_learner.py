"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

CPU TD update in plain PyTorch autograd — the "reference CPU path" that
bench.py times as cpu_baseline and the GPU learner is checked against.

The reference ships no learner; per_run.py:224-238 only
fixes the call ``info = learner.train(batch, t_env, episode, per_weights)`` and
``info["td_errors_abs"]`` as one priority per sampled episode.  This follows
the PyMARL2 NQLearner that contract comes from:

  * online agent unrolled over t = 0..T (mac.init_hidden -> zeros), Q gathered
    at the taken actions for t < T;
  * target agent unrolled over t = 0..T, double-Q: argmax of the online Q with
    unavailable actions set to -9999999, target Q gathered there;
  * transformer mixers unrolled with recurrent hyper tokens (zeros at t = 0),
    online over t < T with the online agent hidden states, target over t <= T;
  * build_td_lambda_targets(r, term, mask, Qtot_tgt, γ, λ);
  * loss = Σ_b w_b Σ_t ½ td² m / Σ m;  priorities Σ_t |td| m / √Σ_t m;
  * clip_grad_norm_(10) + Adam.
Parity-unpinned beyond the agent/mixer arithmetic: γ, λ, the loss form and the
optimiser are not fixed by any reference file.
"""
import torch

from . import ref_model


def build_td_lambda_targets(rewards, terminated, mask, target_qs, gamma, td_lambda):
    """PyMARL2 utils/rl_utils.py semantics; target_qs [B, T+1], others [B, T]."""
    ret = target_qs.new_zeros(*target_qs.shape)
    ret[:, -1] = target_qs[:, -1] * (1 - torch.sum(terminated, dim=1))
    for t in range(ret.shape[1] - 2, -1, -1):
        ret[:, t] = td_lambda * gamma * ret[:, t + 1] + mask[:, t] * (
            rewards[:, t] + (1 - td_lambda) * gamma * target_qs[:, t + 1] * (1 - terminated[:, t]))
    return ret[:, 0:-1]


def td_forward(p_agent, p_mixer, p_agent_tgt, p_mixer_tgt, batch, cfg, *, gamma=0.99, td_lambda=0.6,
               per_weight=None, detach_mixer_hidden=False, relu=None):
    """Returns (loss, td_errors_abs [B], extras).  relu: an optional
    ref_model.TieAwareRelu used for every FFN ReLU of this call (its recorded ties'
    backward branches can then be chosen before loss.backward)."""
    if relu is not None:
        prev, ref_model._ffn_relu = ref_model._ffn_relu, relu
        try:
            return td_forward(p_agent, p_mixer, p_agent_tgt, p_mixer_tgt, batch, cfg, gamma=gamma,
                              td_lambda=td_lambda, per_weight=per_weight, detach_mixer_hidden=detach_mixer_hidden)
        finally:
            ref_model._ffn_relu = prev
    obs, state = batch["obs"], batch["state"]
    actions, avail = batch["actions"], batch["avail_actions"]
    B, T1, A, _ = obs.shape
    T = T1 - 1
    E = cfg["emb"]
    rewards = batch["reward"][:, :-1, 0]
    terminated = batch["terminated"][:, :-1, 0].float()
    mask = batch["filled"][:, :-1, 0].float()
    mask[:, 1:] = mask[:, 1:] * (1 - terminated[:, :-1])
    h0 = torch.zeros(B, A, E, dtype=obs.dtype)
    mac_out, hs = ref_model.agent_unroll(p_agent, obs, h0, cfg=cfg)
    chosen = torch.gather(mac_out[:, :-1], 3, actions[:, :-1]).squeeze(3)
    with torch.no_grad():
        tgt_out, tgt_hs = ref_model.agent_unroll(p_agent_tgt, obs, h0, cfg=cfg)
        mac_det = mac_out.clone().detach()
        mac_det[avail == 0] = -9999999
        cur_max = mac_det.max(dim=3, keepdim=True)[1]
        target_max_q = torch.gather(tgt_out, 3, cur_max).squeeze(3)
        hw0 = torch.zeros(B, 3, cfg["mixer_emb"], dtype=obs.dtype)
        obs_tok = None if cfg.get("state_entity_mode", True) else obs  # n_transf_mixer.py:60-63
        qtot_tgt, _ = ref_model.mixer_unroll(p_mixer_tgt, target_max_q, tgt_hs, state, hw0, cfg=cfg, obs=obs_tok)
        targets = build_td_lambda_targets(rewards, terminated, mask, qtot_tgt, gamma, td_lambda)
    hid = hs[:, :-1].detach() if detach_mixer_hidden else hs[:, :-1]
    hw0 = torch.zeros(B, 3, cfg["mixer_emb"], dtype=obs.dtype)
    qtot, _ = ref_model.mixer_unroll(p_mixer, chosen, hid, state[:, :-1], hw0, cfg=cfg,
                                     obs=None if obs_tok is None else obs[:, :-1])
    td_error = qtot - targets.detach()
    td_error2 = 0.5 * td_error.pow(2)
    masked = td_error2 * mask
    if per_weight is not None:
        masked = masked.sum(1) * per_weight
    loss = masked.sum() / mask.sum()
    prio = ((td_error.abs() * mask).sum(1) / torch.sqrt(mask.sum(1))).detach()
    return loss, prio, dict(qtot=qtot.detach(), qtot_tgt=qtot_tgt, targets=targets, mac_out=mac_out.detach())


class RefLearner:
    """Minimal stateful CPU learner: params as leaf tensors, Adam, clip 10."""

    def __init__(self, p_agent, p_mixer, cfg, *, lr=1e-3, gamma=0.99, td_lambda=0.6, grad_norm_clip=10.0,
                 target_update_interval=200, detach_mixer_hidden=False):
        self.cfg = cfg
        self.pa = {k: v.clone().requires_grad_(True) for k, v in p_agent.items()}
        self.pm = {k: v.clone().requires_grad_(True) for k, v in p_mixer.items()}
        self.pa_t = {k: v.detach().clone() for k, v in p_agent.items()}
        self.pm_t = {k: v.detach().clone() for k, v in p_mixer.items()}
        self.params = list(self.pa.values()) + list(self.pm.values())
        self.opt = torch.optim.Adam(self.params, lr=lr)
        self.gamma, self.td_lambda, self.clip = gamma, td_lambda, grad_norm_clip
        self.target_update_interval = target_update_interval
        self.detach = detach_mixer_hidden
        self.last_target_update_episode = 0

    def train(self, batch, t_env, episode, per_weight=None):
        loss, prio, ex = td_forward(self.pa, self.pm, self.pa_t, self.pm_t, batch, self.cfg,
                                    gamma=self.gamma, td_lambda=self.td_lambda, per_weight=per_weight,
                                    detach_mixer_hidden=self.detach)
        self.opt.zero_grad()
        loss.backward()
        grad_norm = torch.nn.utils.clip_grad_norm_(self.params, self.clip)
        self.opt.step()
        if (episode - self.last_target_update_episode) / self.target_update_interval >= 1.0:
            self.update_targets()
            self.last_target_update_episode = episode
        return {"loss": loss.item(), "grad_norm": float(grad_norm), "td_errors_abs": prio, **ex}

    def update_targets(self):
        for src, dst in ((self.pa, self.pa_t), (self.pm, self.pm_t)):
            for k in src:
                dst[k].copy_(src[k].detach())
