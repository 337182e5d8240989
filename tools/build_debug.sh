#!/bin/bash
# Libraries for the layout-sensitivity hunt, into t2omca_amd/lib/:
#   dbg.so            default code, every kernel's dynamic LDS poisoned with NaN at entry
#                     (T2O_DEBUG_POISON) and every automatic variable pattern-initialised
#                     (-ftrivial-auto-var-init=pattern: 0xFF.. = NaN for floats)
#   {,dbg_}kmf.so     the fp32 flat key mask at both mixer call sites (T2O_KM_FP32_FLAT=3)
#   {,dbg_}pf.so      the full-record tile-pair contraction (T2O_DW_PAIR_FULL=1)
#   {,dbg_}odd.so     odd key-tile counts paired, last comb tile alone (T2O_KF_ODD_PAIR=1)
#   odd2.so / odd3.so the same with the tail in its own accumulator / chained after 16
#                     wait states (T2O_KF_ODD_PAIR=2 / 3)
# A variant recompiles only the translation units its switch reaches and links them
# with the matching (product / debug) objects of the rest.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/t2omca_amd/csrc
O=${T2O_DBG_OBJ:-/tmp/t2o_dbg_obj}
mkdir -p "$O"
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-result"
DBG="-DT2O_DEBUG_POISON=1 -ftrivial-auto-var-init=pattern"
MIX="t2o_mixer.hip t2o_mixer_split.hip"
jobs=()
NEWEST=$(ls -t "$S"/*.hpp "$R"/include/t2omca.h | head -1)
add() {  # add <objdir-tag> <flags> <files...>   (an object newer than its source and every header is kept)
  local tag=$1 fl=$2; shift 2
  mkdir -p "$O/$tag"
  for f in "$@"; do
    local o="$O/$tag/$f.o"
    if [ -f "$o" ] && [ "$o" -nt "$S/$f" ] && [ "$o" -nt "$NEWEST" ]; then continue; fi
    jobs+=("$tag|$fl|$f")
  done
}
ALL=$(cd "$S" && ls *.hip)
add dbg "$DBG" $ALL
add kmf "-DT2O_KM_FP32_FLAT=3" $MIX
add dbg_kmf "$DBG -DT2O_KM_FP32_FLAT=3" $MIX
add odd "-DT2O_KF_ODD_PAIR=1" $MIX
add dbg_odd "$DBG -DT2O_KF_ODD_PAIR=1" $MIX
add odd2 "-DT2O_KF_ODD_PAIR=2" $MIX
add odd3 "-DT2O_KF_ODD_PAIR=3" $MIX
add pf "-DT2O_DW_PAIR_FULL=1" t2o_dwgemm.hip
add dbg_pf "$DBG -DT2O_DW_PAIR_FULL=1" t2o_dwgemm.hip
[ ${#jobs[@]} -gt 0 ] && printf '%s\n' "${jobs[@]}" | xargs -P "${JOBS:-8}" -I{} bash -c '
  IFS="|" read -r tag fl f <<< "{}"
  '"$HIPCC"' $fl -c -o '"$O"'/$tag/$f.o '"$S"'/$f || { echo "FAILED $tag $f"; exit 1; }'
# product objects for the non-debug variants: the in-tree build's
P=$R/t2omca_amd/lib/obj
link() {  # link <name> <base objdir> <variant objdir>
  local objs=()
  for f in $ALL; do
    if [ -f "$O/$3/$f.o" ]; then objs+=("$O/$3/$f.o"); else objs+=("$2/$f.o"); fi
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/t2omca_amd/lib/$1.so" "${objs[@]}"
  echo "$R/t2omca_amd/lib/$1.so"
}
link dbg "$O/dbg" dbg
for v in kmf odd pf; do
  link $v "$P" $v
  link dbg_$v "$O/dbg" dbg_$v
done
for v in odd2 odd3; do link $v "$P" $v; done
