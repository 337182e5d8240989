"""Algorithmic FLOP / byte counts of the kernels' algorithm (for roofline lines).

Counts the arithmetic the fused kernels are required to do by their algorithm
(token-pruned, folded projections, observation-space agent attention; see
DESIGN.md §3), not what the MFMA tiles pad it to, and excluding the backward's
forward recompute.  A multiply-add is 2 FLOPs; softmax exp/div and LayerNorm
count ~5 FLOPs per element.

SURVEY.md §8(d) also quotes the reference-association-order counts
(1.793 / 2.608 / 7.833 MFLOP per agent-transition at A = 8 / 16 / 64);
``ref_order_flops_per_transition`` reproduces that formula so bench.py can
report both.  bench.py prices its roofline on the §8(d) reference-order count
(``ref_order_kernel_flops``) and reports the executed-algorithm count beside it.
"""


def agent_row_step_flops(E=32, H=3, D=2, F=9, n=8, NA=5, FF=None):
    FF = FF or 4 * E
    HE = H * E
    blk = (2 * HE * E            # u = M x
           + H * 2 * F * E       # w_h = We^T u_h
           + H * 4 * E           # c_h, s_h0
           + H * n * 2 * F       # entity scores
           + H * (n + 1) * 5     # softmax
           + H * n * 2 * F       # ô_h
           + H * (2 * E * F + 4 * E)  # z_h
           + 2 * E * HE          # N z
           + 2 * 2 * FF * E      # FFN
           + 2 * 8 * E)          # residuals + 2 LayerNorms
    return D * blk + 2 * NA * E


def mixer_episode_step_flops(E=32, H=3, D=2, A=8, Fs=8, FF=None):
    FF = FF or 4 * E
    HE = H * E
    Lk, Q = 2 * A + 3, A + 3
    row_blk = (2 * HE * E + H * 2 * Lk * E + H * Lk * 5 + H * 2 * Lk * E + 2 * E * HE + 2 * 2 * FF * E + 2 * 8 * E)
    embed = A * 2 * Fs * E
    head = A * 3 * E + 6 * E
    return D * Q * row_blk + embed + head


def dw_record_flops(E=32, H=3, D=2, FF=None):
    """FLOPs of the tape contraction per record (all D blocks): 2 x |M|+|N|+|W1|+|W2|."""
    FF = FF or 4 * E
    return D * 2 * (2 * H * E * E + 2 * FF * E)


def dw_record_bytes(E=32, H=3, D=2, FF=None, elem=4):
    """Tape bytes per record (all D blocks): written once by the backward, read once
    by the contraction; elem = 4 (fp32 mode) or 2 (bf16 mode)."""
    FF = FF or 4 * E
    return D * elem * (4 * E + 2 * H * E)


def td_update_flops(B, T, A, E=32, H=3, D=2, F=9, Fs=8, NA=5):
    """Per-kernel algorithmic FLOPs of one TD update (fwd online+target, bwd = 2x fwd).

    The backward's share of the M/N/W1/W2 weight-gradient contractions is
    executed by the tape contraction kernels (agent_dw / mixer_dw); the BPTT
    kernels are charged the rest."""
    fa = agent_row_step_flops(E, H, D, F, A, NA)
    fm = mixer_episode_step_flops(E, H, D, A, Fs)
    dw_a = B * T * A * dw_record_flops(E, H, D)
    dw_m = B * T * (A + 3) * dw_record_flops(E, H, D)
    return {
        "agent_fwd": 2 * B * (T + 1) * A * fa,
        "mixer_fwd": (B * T + B * (T + 1)) * fm,
        "mixer_bwd": 2 * B * T * fm - dw_m,
        "mixer_dw": dw_m,
        "agent_bwd": 2 * B * T * A * fa - dw_a,
        "agent_dw": dw_a,
    }


def td_update_bytes(B, T, A, E=32, F=9, Fs=8, NA=5, elem=4):
    """Compulsory HBM bytes per kernel: its inputs read and outputs written once
    (the replay batch's obs / state in fp32, Q / hidden rows, the mixer's per-step
    outputs).  The weight-gradient tape is the implementation's own intermediate,
    not algorithmic traffic: it is reported apart, by ``td_tape_bytes``."""
    obs = B * (T + 1) * A * A * F * 4
    st = B * (T + 1) * A * Fs * 4
    qh = B * (T + 1) * A * (NA + E) * 4
    return {
        "agent_fwd": obs + 2 * qh,
        "mixer_fwd": st + 2 * qh + 2 * B * (T + 1) * ((A + 3) * E + 3 * E + A + 1) * 4,
        "mixer_bwd": st + B * T * ((A + 3) * E + 3 * E + 2 * A + A * E + 2) * 4,
        "agent_bwd": obs + B * T * A * (2 * E + 2) * 4,
    }


def td_tape_bytes(B, T, A, E=32, elem=4):
    """Weight-gradient tape bytes per update (valid records only, in the MFMA operand
    type): written by the BPTT kernel, read back by its contraction (agent_dw /
    mixer_dw).  The mixer's record is always the full one (x, gu, z, gres, gr2, x̂1:
    320 features at E 32 / H 3); the agent's pipelined bf16 kernel writes the lean
    record (gres, gr2, x̂1: 96 of 320) at up to 8 entities."""
    full = dw_record_bytes(E, elem=elem)
    agent_rec = full * 3 * E // (4 * E + 2 * 3 * E) if (elem == 2 and A <= 8) else full
    return {"agent": B * T * A * agent_rec, "mixer": B * T * (A + 3) * full}


def env_step_bytes(A):
    """algorithmic HBM bytes per agent per env step — the agent's
    state (position 16 B, MEC index 4 B, job queue <= ~64 B, ack 4 B) plus its
    observation row written once (9A fp32)."""
    return 16 + 4 + 64 + 4 + 9 * A * 4


def ref_order_network_flops(A, E=32, H=3, D=2, F=9, Fs=8, NA=5, FF=None):
    """(F_agent per sequence-step, F_mixer per episode-step), the
    necessary (token-pruned) forward FLOPs in the reference association order."""
    FF = FF or 4 * E
    HE = H * E
    La, Lm, Lq = A + 1, 2 * A + 3, A + 3
    f_agent = 2 * A * F * E + D * (4 * La * E * HE + 2 * E * HE + 4 * H * La * E + 2 * HE * E + 4 * E * FF) \
        + 2 * E * NA
    f_mixer = 2 * A * Fs * E + D * (4 * Lm * E * HE + 2 * Lq * E * HE + 4 * H * Lq * Lm * E
                                    + 2 * Lq * HE * E + 4 * Lq * E * FF)
    return f_agent, f_mixer


def ref_order_flops_per_transition(A, E=32, H=3, D=2, F=9, Fs=8, NA=5, FF=None):
    """SURVEY.md §8(d) formula: 4*F_agent + 4*F_mixer/A (reference association order)."""
    f_agent, f_mixer = ref_order_network_flops(A, E, H, D, F, Fs, NA, FF)
    return 4 * f_agent + 4 * f_mixer / A


def ref_order_kernel_flops(B, T, A, **kw):
    """SURVEY.md §8(d)'s per-kernel shares of one TD update (the basis of the bench's
    roofline): forward online + target once each, backward = 2x the online forward,
    recompute excluded, the (T+1)/T factor ignored.  The backward share of a network
    is charged to its BPTT kernel (the tape contractions are part of that backward)."""
    f_agent, f_mixer = ref_order_network_flops(A, **kw)
    return {"agent_fwd": 2 * B * T * A * f_agent, "mixer_fwd": 2 * B * T * f_mixer,
            "agent_bwd": 2 * B * T * A * f_agent, "mixer_bwd": 2 * B * T * f_mixer}
