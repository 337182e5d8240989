"""Per-phase cycle split of the env step kernel, from a timing-probe build of t2o_env.hip
(T2O_LIB=<probe .so> exporting t2o_env_probe_read; not the product library).
Runs configs[4]'s env (8192 envs x 16 AGVs x 2 MEC) for a few steps with random avail actions
and prints mean / p90 cycles per phase over the last step's waves."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

from t2omca_amd import _lib
from t2omca_amd.env import VecEnv

NE, A = int(os.environ.get("NE", 8192)), 16
env = VecEnv(NE, mec_num=2, agv_num=A, episode_limit=150, seed=1)
env.get_env_info()
st, av, obs = env.reset()
g = torch.Generator(device="cuda").manual_seed(0)
for t in range(20):
    u = torch.rand(av.shape, device="cuda", generator=g) * av
    acts = u.argmax(-1)
    env.step(acts)
torch.cuda.synchronize()
nw = (NE + 3) // 4
buf = np.zeros((4096, 16), np.uint64)
_lib.lib().t2o_env_probe_read.restype = ctypes.c_int
rc = _lib.lib().t2o_env_probe_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
assert rc == 0, rc
b = buf[:nw].astype(np.int64)
clk = b[:, 1:12]  # clock64 at probe points 0..10
names = ["state + normaliser loads (wait at the 1st barrier)", "head job + collision counts",
         "per-agent reward + leader sums", "update_users", "terminal sums", "fill L from registers",
         "state/avail/wire + get_obs prologue", "get_obs update loop", "get_obs epilogue + counts", "(unused)"]
d = np.diff(clk, axis=1)
out = {"waves": int(nw),
       "wall_us_100MHz": {"start_spread": float((b[:, 0].max() - b[:, 0].min()) / 100.0),
                          "mean_life": float((b[:, 12] - b[:, 0]).mean() / 100.0),
                          "kernel_span": float((b[:, 12].max() - b[:, 0].min()) / 100.0)},
       "total_cycles_mean": float((clk[:, 10] - clk[:, 0]).mean()),
       "phase_cycles_mean": {}, "phase_cycles_p90": {}}
order = [(0, 1, names[0]), (1, 2, names[1]), (2, 3, names[2]), (3, 4, names[3]), (4, 5, names[4]),
         (5, 6, names[5]), (6, 8, names[6]), (8, 9, names[7]), (9, 10, names[8])]
for i, j, n in order:
    c = clk[:, j] - clk[:, i]
    c = c[(c >= 0) & (c < 1 << 30)]  # waves that took the slow normaliser path skip probe 8
    out["phase_cycles_mean"][n] = float(c.mean())
    out["phase_cycles_p90"][n] = float(np.percentile(c, 90))
print(json.dumps(out, indent=1))
