# 32-AGV mixer BPTT regression: current vs no key-tile pairing (parity-gated), 32 and 8 AGVs
set -u
AB_SERIAL= bash tools/ab_box.sh r5_a32b/a32 t2omca_amd/lib/ab_cur.so t2omca_amd/lib/ab_nokp.so -- --agents 32 --batch 1024 --T 60 --steps 4 --warmup 2 || exit 1
AB_SERIAL= bash tools/ab_box.sh r5_a32b/head t2omca_amd/lib/ab_cur.so t2omca_amd/lib/ab_nokp.so || exit 1
