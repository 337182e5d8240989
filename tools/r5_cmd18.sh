# agent tape contraction: 4- vs 8-tile groups (serial: the contraction alone; overlapped: the headline)
set -u
bash tools/ab_box.sh r5_tg8/serial t2omca_amd/lib/ab_tg4.so t2omca_amd/lib/ab_tg8.so || exit 1
AB_SERIAL= bash tools/ab_box.sh r5_tg8/head t2omca_amd/lib/ab_tg4.so t2omca_amd/lib/ab_tg8.so || exit 1
