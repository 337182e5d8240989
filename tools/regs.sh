#!/bin/bash
# Register / scratch use of the kernel instances of one translation unit:
#   tools/regs.sh t2o_agent.hip [name-regex]
cd "$(dirname "$0")/../t2omca_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -c -o /tmp/regs.o "$1" -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
pat = re.compile(sys.argv[1]); name = None; out = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1); continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill): (\d+)", line)
    if m and name and pat.search(name):
        out.setdefault(name, []).append(f"{m.group(1).split()[0]}={m.group(2)}")
for n, v in out.items():
    print(n[:90], " ".join(v))
' "${2:-.}"
