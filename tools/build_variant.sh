#!/bin/bash
# Build the working-tree library with extra compiler flags to t2omca_amd/lib/<name>.so
#   tools/build_variant.sh <name> [-DFLAG ...]
set -eu
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
for f in "$R"/t2omca_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-result "$@" -c -o "$T/$(basename "$f").o" "$f" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/t2omca_amd/lib/$NAME.so" "$T"/*.o
rm -rf "$T"
echo "$R/t2omca_amd/lib/$NAME.so"
