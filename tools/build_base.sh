#!/bin/bash
# Build the library of git revision $1 (default HEAD) to t2omca_amd/lib/<name $2, default libt2omca_base>.so
# (A/B baseline).
set -eu
REV=${1:-HEAD}
NAME=${2:-libt2omca_base}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive "$REV" t2omca_amd/csrc include | tar -x -C "$T"
mkdir -p "$T/obj"
for f in "$T"/t2omca_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-result -c -o "$T/obj/$(basename "$f").o" "$f" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/t2omca_amd/lib/$NAME.so" "$T"/obj/*.o
rm -rf "$T"
echo "$R/t2omca_amd/lib/$NAME.so ($REV)"
