#!/bin/bash
# Library variant that differs in some sources' compile flags, linking the in-tree objects of
# every other source:   tools/build_file_variant.sh <name> <a.hip[,b.hip...]> [flags ...]
set -eu
NAME=$1; SRCS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
for SRC in ${SRCS//,/ }; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-result "$@" -c -o "$T/$SRC.o" \
    "$R/t2omca_amd/csrc/$SRC" &
done
wait
objs=""
for o in "$R"/t2omca_amd/lib/obj/*.o; do [ -f "$T/$(basename "$o")" ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/t2omca_amd/lib/$NAME.so" $objs "$T"/*.o
rm -rf "$T"
echo "$R/t2omca_amd/lib/$NAME.so"
