#!/bin/bash
# Build a library variant that differs only in t2o_env.hip (extra flags), linking the
# in-tree objects of every other source:   tools/build_env_variant.sh <name> [-DFLAG ...]
set -eu
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-result "$@" -c -o "$T/t2o_env.hip.o" "$R/t2omca_amd/csrc/t2o_env.hip"
objs=$(ls "$R"/t2omca_amd/lib/obj/*.o | grep -v t2o_env.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/t2omca_amd/lib/$NAME.so" $objs "$T/t2o_env.hip.o"
rm -rf "$T"
echo "$R/t2omca_amd/lib/$NAME.so"
