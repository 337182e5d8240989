#!/bin/bash
# Run ON THE GPU BOX: GPU suite on the working build, then an interleaved A/B
# (overlapped, parity-gated) of the given library builds.
#   tools/r3_h.sh <tag> <lib1.so> <lib2.so> ...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest.log" | head -20; exit 1; }
echo "== ab"
AB_SERIAL= bash tools/ab_box.sh "$TAG/ab" "$@"
