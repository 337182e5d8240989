"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> [workload-tag]

Corrections (MI355X_MICROARCH.md, HBM section): rocprofv3 reports both counters in KiB;
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so it is doubled.
The two counters are collected in separate passes (they do not fit one TCC pass).
"""
import csv
import glob
import json
import os
import re
import sys

SHORT = {"agent_fwd_kernel": "agent_fwd", "mixer_fwd_kernel": "mixer_fwd", "mixer_bwd_kernel": "mixer_bwd",
         "agent_bwd_kernel": "agent_bwd", "agent_bwd_pipe_kernel": "agent_bwd", "mixer_bwd_pipe_kernel": "mixer_bwd", "td_loss_kernel": "td_loss", "adam_kernel": "adam",
         "env_kernel": "env_step", "reduce_slabs_kernel": "reduce_slabs", "seg_kernel": "pack",
         "select_actions_kernel": "select_actions", "obs_expand_kernel": "obs_expand"}


def _is_bf16(name):
    return "DF16b" in name or "__bf16" in name


def per_kernel(d, counter, want_bf16=None):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                if want_bf16 is not None and _is_bf16(name) != want_bf16:
                    continue  # the other operand type's instance (e.g. an fp32 companion run)
                m = re.search(r"dw_gemm_kernel(?:<\d+, *\d+, *\d+, *\d+, *|ILi\d+ELi\d+ELi\d+ELi\d+ELi)(\d)", name)
                short = ("agent_dw", "mixer_dw")[int(m.group(1))] if m else \
                    next((v for k, v in SHORT.items() if k in name), None)
                if short is None:
                    continue
                vals.setdefault(short, []).append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, out = sys.argv[1:4]
    tag = sys.argv[4] if len(sys.argv) > 4 else ""
    want = True if tag.endswith("_bf16") else False if tag.endswith("_fp32") else None
    fetch, write = per_kernel(fdir, "FETCH_SIZE", want), per_kernel(wdir, "WRITE_SIZE", want)
    res = {"workload": tag, "units": "bytes per launch (FETCH_SIZE x2 x1024, WRITE_SIZE x1024)", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        res["kernels"][k] = {"fetch_bytes": fb, "write_bytes": wb,
                             "hbm_bytes": (fb or 0) + (wb or 0), "launches": [len(f), len(w)]}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
