#!/bin/bash
# Run ON THE GPU BOX: interleaved overlapped A/B: agent BPTT (bf16) with the
# kernel-argument layout vs compile-time offsets.
set -u
AB_SERIAL= bash tools/ab_box.sh r3_ab6 t2omca_amd/lib/libt2omca_agp0.so t2omca_amd/lib/libt2omca.so
