"""Diagnostic: in-kernel cycle stamps (variant build with -DT2O_PHASE_PROF, loaded
through T2O_LIB).  Runs TD updates and prints median cycles per segment for one
workgroup (WG 7) of the agent BPTT (per phase) and the mixer forward (per step).
s_memtime ticks are shader cycles (MI355X_MICROARCH.md); the stamps themselves
cost a few percent."""
import ctypes
import os
import statistics as st
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from t2omca_amd._lib import lib  # noqa: E402
from t2omca_amd.learner import TDLearner  # noqa: E402
from t2omca_amd.modules import TransformerAgent, TransformerMixer  # noqa: E402
from t2omca_amd.synthetic import make_args, make_batch  # noqa: E402

A, B, T = 8, 1024, 60
torch.manual_seed(0)
margs = make_args(A, device="cuda")
learner = TDLearner(TransformerAgent(None, margs).cuda(), TransformerMixer(margs).cuda(), overlap=False,
                    precision="bf16")
batch, w = make_batch(B, T, A, seed=1, device="cuda")
for _ in range(2):
    learner.train(batch, 0, 0, per_weight=w)
torch.cuda.synchronize()


def read(fn):
    buf = np.zeros(128 * 8 * 4, dtype=np.int64)
    f = getattr(lib(), fn)
    f.argtypes = [ctypes.c_void_p]
    assert f(buf.ctypes.data) == 0
    return buf.reshape(128, 8, 4)


ag = read("t2o_prof_read_agent")[2:2 * T - 2].reshape(T - 2, 2, 8, 4)
print("agent BPTT (two waves per tile), median cycles per phase segment:")
for ph, kind in enumerate(("fwd: inputs | attention | post | barrier", "bwd: inputs | post | attention | barrier")):
    for wv in range(4):
        m = [st.median(ag[:, ph, wv, i]) for i in range(4)]
        print(f"  {kind.split(':')[0]} wave {wv} (block {wv & 1}): " + "  ".join(f"{x:7.0f}" for x in m) +
              f"   [{kind.split(': ')[1]}]")
mx = read("t2o_prof_read_mixer")[1:T - 1]
print("mixer forward (online net), median cycles per step segment: keys | block 0 | block 1 | head+rest")
for wv in range(8):
    m = [st.median(mx[:, wv, i]) for i in range(4)]
    print(f"  wave {wv}: " + "  ".join(f"{x:7.0f}" for x in m) + f"   total {sum(m):7.0f}")
