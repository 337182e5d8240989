"""Writes a timing-probe copy of t2o_env.hip (never the product source): lane 0 of every
wave records clock64() at phase boundaries of the step kernel into a device array read
back by t2o_env_probe_read.  Build: tools/make_env_probe.py <out.hip>, then hipcc."""
import sys

src = open(__file__.replace("tools/make_env_probe.py", "t2omca_amd/csrc/t2o_env.hip")).read()
pts = [
    ("  const Who w = who(a);\n", "after", 0),
    ("  // the head job (load_agent)\n", "before", 1),
    ("  int ack = 0;\n  if (w.agent) {\n    if (act == 0)", "before", 2),
    ("  // update_users (:295-307)", "before", 3),
    ("  if (w.lead) {\n    a.s.draw[w.e] = base + 5 * A;", "before", 4),
    ("  // the worker's get_state / get_avail_actions / get_obs on the new state\n  if (w.agent) {", "before", 5),
    ("  write_state_avail(a, w, L);\n  write_wire(a, w, L);\n  get_obs<true>(a, w, L, pre, false);\n  if (w.lead) a.s.nrm_n", "before", 6),
    ("  get_obs<true>(a, w, L, pre, false);\n  if (w.lead) a.s.nrm_n[w.e] = L.n[w.g];\n}\n\n__global__", "before", 7),
    ("  const double n0 = (double)nref;\n", "before", 8),
    ("  if (w.lead) a.s.nrm_n[w.e] = L.n[w.g];\n}\n\n__global__", "before", 10),
]
for pat, where, k in pts:
    assert src.count(pat) == 1, (k, src.count(pat))
    ins = f"  T2O_PROBE({k});\n"
    src = src.replace(pat, pat + ins if where == "after" else ins + pat)
# end of the fast loop (before norm_fast's closing brace): the line after the i loop
pat = "        }\n      }\n    }\n  }\n}\n\n// This lane's normaliser items"
assert src.count(pat) == 1
src = src.replace(pat, "        }\n      }\n    }\n  }\n  T2O_PROBE(9);\n}\n\n// This lane's normaliser items")
src = src.replace("namespace {\n", """namespace {
__device__ unsigned long long g_probe[4096 * 16];
#define T2O_PROBE(k) do { if ((threadIdx.x & 63) == 0 && a.mode == 2 && blockIdx.x < 4096) { \\
  unsigned long long* P_ = g_probe + (size_t)blockIdx.x * 16; P_[1 + (k)] = clock64(); \\
  if ((k) == 0) P_[0] = wall_clock64(); if ((k) == 10) P_[12] = wall_clock64(); } } while (0)
""", 1)
src = src.replace('extern "C" int t2o_env_run_ex(', '''extern "C" int t2o_env_probe_read(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_probe), bytes, 0, hipMemcpyDeviceToHost);
}

extern "C" int t2o_env_run_ex(''', 1)
open(sys.argv[1], "w").write(src)
