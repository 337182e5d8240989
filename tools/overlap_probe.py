"""Probe: do the agent and mixer recurrences overlap when launched on two streams?

Runs (configs[2], bf16) the agent forward and the mixer forward, then the mixer
BPTT and the agent BPTT, each pair (a) back to back on one stream and (b) on two
streams at once (independent inputs: the pair's data dependence is ignored, only
the co-scheduling is measured).  Prints ms per pair for both.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from t2omca_amd import ops
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args, make_batch
    A, B, T = 8, 1024, 60
    torch.manual_seed(0)
    args = make_args(A)
    lr = TDLearner(TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda(), precision="bf16")
    batch, w = make_batch(B, T, A, seed=1)
    for _ in range(3):
        lr.train(batch, 0, 0, per_weight=w)
    obs, state = batch["obs"], batch["state"]
    act = batch["actions"][..., 0]
    ops.pack_params(lr.sa, lr.params[:lr.na], lr.pack_a)
    ops.pack_params(lr.sm, lr.params[lr.na:], lr.pack_m)
    hmid = torch.empty(B, T + 1, 1, A, 32, device="cuda")
    q_on, h_on, q_tg, h_tg = ops.agent_unroll_fwd(lr.sa, lr.pack_a, obs, pack_tg=lr.pack_at, hmid_on=hmid)
    o_on, o_tg = ops.mixer_unroll_fwd(lr.sm, lr.pack_m, state, h_on, qmode_on=1, q_on=q_on, actions=act,
                                      T_on=T, pack_tg=lr.pack_mt, hid_tg=h_tg, qmode_tg=2, q_tg=q_tg, T_tg=T + 1)
    gy = torch.randn(B, T, device="cuda") * 1e-3
    gq = torch.randn(B, T, A, device="cuda") * 1e-3
    gh = torch.randn(B, T, A, 32, device="cuda") * 1e-3
    tape_m = torch.empty(ops.tape_floats(lr.sm, ops.mixer_tape_tiles(B, T, A, lr.sm)), device="cuda")
    tape_a = torch.empty(ops.tape_floats(lr.sa, ops.agent_tape_tiles(B, T, A)), device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def fwd_a():
        ops.agent_unroll_fwd(lr.sa, lr.pack_a, obs, pack_tg=lr.pack_at, hmid_on=hmid)

    def fwd_m():
        ops.mixer_unroll_fwd(lr.sm, lr.pack_m, state, h_on, qmode_on=1, q_on=q_on, actions=act, T_on=T,
                             pack_tg=lr.pack_mt, hid_tg=h_tg, qmode_tg=2, q_tg=q_tg, T_tg=T + 1)

    def bwd_m():
        ops.mixer_unroll_bwd(lr.sm, lr.pack_m, state, h_on, o_on, gy, tape=tape_m, defer_contract=True)

    def bwd_a():
        ops.agent_unroll_bwd(lr.sa, lr.pack_a, obs, h_on, gchosen=gq, actions=act, gh=gh, hmid=hmid, tape=tape_a)

    def timeit(fn, n=10):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    def pair_serial(f, g):
        return lambda: (f(), g())

    def pair_overlap(f, g):
        def run():
            main = torch.cuda.current_stream()
            s1.wait_stream(main)
            s2.wait_stream(main)
            with torch.cuda.stream(s1):
                f()
            with torch.cuda.stream(s2):
                g()
            main.wait_stream(s1)
            main.wait_stream(s2)
        return run

    for name, f, g in (("fwd agent|mixer", fwd_a, fwd_m), ("bwd mixer|agent", bwd_m, bwd_a)):
        print(f"{name}: alone {timeit(f):.3f} + {timeit(g):.3f} ms; serial pair {timeit(pair_serial(f, g)):.3f} ms; "
              f"two streams {timeit(pair_overlap(f, g)):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
