#!/bin/bash
# The debug library for layout / ordering hunts, into t2omca_amd/lib/dbg.so:
# default code, every kernel's dynamic LDS poisoned with NaN at entry
# (T2O_DEBUG_POISON) and every automatic variable pattern-initialised
# (-ftrivial-auto-var-init=pattern: 0xFF.. = NaN for floats).  Run the GPU tests
# against it with T2O_LIB=t2omca_amd/lib/dbg.so T2O_POISON=1 (the latter NaN-fills
# torch.empty* workspaces, tests/conftest.py).
# Round 6 also built the then-switchable forms here (the fp32 flat key mask, the
# full-record pair contraction, odd key-tile pairing); the switches were deleted with
# the verdicts in DESIGN.md §2d, and their builds with them.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/t2omca_amd/csrc
O=${T2O_DBG_OBJ:-/tmp/t2o_dbg_obj}
mkdir -p "$O/dbg"
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-result"
DBG="-DT2O_DEBUG_POISON=1 -ftrivial-auto-var-init=pattern"
NEWEST=$(ls -t "$S"/*.hpp "$R"/include/t2omca.h | head -1)
ALL=$(cd "$S" && ls *.hip)
todo=()
for f in $ALL; do  # (an object newer than its source and every header is kept)
  o="$O/dbg/$f.o"
  if [ -f "$o" ] && [ "$o" -nt "$S/$f" ] && [ "$o" -nt "$NEWEST" ]; then continue; fi
  todo+=("$f")
done
[ ${#todo[@]} -gt 0 ] && printf '%s\n' "${todo[@]}" | xargs -P "${JOBS:-8}" -I{} \
  bash -c "$HIPCC $DBG -c -o '$O/dbg/{}.o' '$S/{}' || { echo 'FAILED {}'; exit 1; }"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/t2omca_amd/lib/dbg.so" "$O"/dbg/*.hip.o
echo "$R/t2omca_amd/lib/dbg.so"
