#!/bin/bash
# Library variant that differs in one source's compile flags, linking the in-tree objects of
# every other source:   tools/build_file_variant.sh <name> <source.hip> [flags ...]
set -eu
NAME=$1; SRC=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-result "$@" -c -o "$T/$SRC.o" "$R/t2omca_amd/csrc/$SRC"
objs=$(ls "$R"/t2omca_amd/lib/obj/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/t2omca_amd/lib/$NAME.so" $objs "$T/$SRC.o"
rm -rf "$T"
echo "$R/t2omca_amd/lib/$NAME.so"
