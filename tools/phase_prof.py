"""Diagnostic: per-phase cycle counts of the pipelined agent BPTT (variant build
with -DT2O_PHASE_PROF, loaded through T2O_LIB).  Runs one TD update and prints
median work / barrier-wait cycles per (phase, role)."""
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
learner = TDLearner(TransformerAgent(None, margs).cuda(), TransformerMixer(margs).cuda(), overlap=False)
batch, w = make_batch(B, T, A, seed=1, device="cuda")
for _ in range(2):
    learner.train(batch, 0, 0, per_weight=w)
torch.cuda.synchronize()
buf = np.zeros(64 * 2 * 4 * 4, dtype=np.int64)
f = lib().t2o_prof_read
f.argtypes = [ctypes.c_void_p]
assert f(buf.ctypes.data) == 0
buf = buf.reshape(64, 2, 4, 4)[1:T]  # skip the first iteration (prologue) and the tail
for ph in range(2):
    for wv in range(4):
        d = wv & 1
        kind = "bwd" if ph == 1 else "fwd"
        m = [st.median(buf[:, ph, wv, i]) for i in range(4)]
        print(f"phase {ph} wave {wv} block {d} {kind}: inputs {m[0]:7.0f}  part1 {m[1]:7.0f}  "
              f"part2 {m[2]:7.0f}  barrier {m[3]:7.0f}  (fwd: attention | post; bwd: post | attention; block-0 waves run one phase late)")
