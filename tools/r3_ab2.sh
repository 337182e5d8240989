#!/bin/bash
# Run ON THE GPU BOX: interleaved overlapped A/B: runtime-instances build vs
# padded rows everywhere vs padded rows except the pipelined mixer BPTT's pair region.
set -u
AB_SERIAL= bash tools/ab_box.sh r3_ab2 t2omca_amd/lib/libt2omca_rt.so t2omca_amd/lib/libt2omca.so \
  t2omca_amd/lib/libt2omca_ldr32.so
