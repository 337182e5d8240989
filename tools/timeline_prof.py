"""Diagnostic: absolute cycle stamps of one workgroup of the pipelined agent BPTT
(variant build with -DT2O_PHASE_PROF -DT2O_TIMELINE, loaded through T2O_LIB):
per wave and iteration, iteration top / phase-0 start / phase-0 work end /
phase-0 barrier exit / phase-1 work end / phase-1 barrier exit."""
import ctypes
import os
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
buf = np.zeros(128 * 8 * 4, dtype=np.int64)
f = lib().t2o_prof_read_agent
f.argtypes = [ctypes.c_void_p]
assert f(buf.ctypes.data) == 0
buf = buf.reshape(128, 8, 4)
t0 = buf[20, 0, 0]
print("it wave: top  ph0start  ph0end  ph0exit  ph1end  ph1exit   (cycles from it 10 top of wave 0)")
for it in range(10, 14):
    for wv in range(4):
        a, b = buf[2 * it, wv], buf[2 * it + 1, wv]
        print(f"{it} {wv}: " + " ".join(f"{v - t0:8d}" for v in (a[0], a[1], a[2], a[3], b[0], b[1])))
