"""Per-kernel summary of rocprofv3 SQ counter passes (counter_collection CSVs).

Usage: python tools/pmc_summary.py <pmc_dir> <out.csv>
Sums each counter over a kernel's dispatches and divides by the dispatch count
(per-launch values), then adds derived ratios: wait / issue-stall / active shares
of SQ_WAVE_CYCLES and MFMA busy / SQ_BUSY_CYCLES.
"""
import csv
import glob
import os
import re
import sys

NAMES = ["agent_fwd_kernel", "mixer_fwd_kernel", "mixer_bwd_kernel", "agent_bwd_kernel", "td_loss_kernel",
         "env_kernel", "reduce_slabs_kernel"]


def short(name):
    m = re.search(r"dw_gemm_kernel(?:<\d+, *\d+, *\d+, *\d+, *|ILi\d+ELi\d+ELi\d+ELi\d+ELi)(\d)", name)
    if m:
        return ("agent_dw", "mixer_dw")[int(m.group(1))]
    if "agent_bwd_pipe_kernel" in name:
        return "agent_bwd"
    if "mixer_bwd_pipe_kernel" in name:
        return "mixer_bwd"
    for n in NAMES:
        if n in name:
            return n.replace("_kernel", "")
    return None


def main():
    d, out = sys.argv[1:3]
    acc = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                if k is None:
                    continue
                c = acc.setdefault(k, {})
                s = c.setdefault(row["Counter_Name"], [0.0, set()])
                s[0] += float(row["Counter_Value"])
                s[1].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    counters = sorted({n for c in acc.values() for n in c})
    rows = []
    for k, c in acc.items():
        r = {"kernel": k}
        for n in counters:
            if n in c:
                r[n] = c[n][0] / max(1, len(c[n][1]))
        wc = r.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in r:
                    r[n + "/WAVE_CYCLES"] = r[n] / wc
        if r.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in r:
            r["MFMA_BUSY/BUSY_CYCLES"] = r["SQ_VALU_MFMA_BUSY_CYCLES"] / r["SQ_BUSY_CYCLES"]
        rows.append(r)
    keys = ["kernel"] + sorted({n for r in rows for n in r if n != "kernel"})
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=keys)
        w.writeheader()
        for r in rows:
            w.writerow({k: (f"{v:.4g}" if isinstance(v, float) else v) for k, v in r.items()})
    for r in rows:
        print(r["kernel"], {k: round(v, 3) for k, v in r.items() if k.endswith("CYCLES") and "/" in k})


if __name__ == "__main__":
    main()
