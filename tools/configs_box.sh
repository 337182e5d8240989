#!/bin/bash
# Run ON THE GPU BOX: the BASELINE configs other than the headline, one MI355X each
#   tools/configs_box.sh <tag>  -> gpurun_out/<tag>/*.json
set -eu
OUT=gpurun_out/$1
mkdir -p "$OUT"
B="timeout -k 10 240 python bench.py --no-cpu-baseline"
$B --agents 16 --batch 32 --T 150 > "$OUT/c1_train.json"
$B --mode forward --agents 16 --batch 128 --T 150 > "$OUT/c2_fwd.json"
$B --agents 16 --batch 1024 --T 150 --steps 5 > "$OUT/a16_train.json"
$B --agents 64 --batch 512 --T 60 --steps 3 --warmup 1 > "$OUT/c4_train.json"
$B --mode rollout --agents 16 --envs 8192 --mecs 2 --T 150 --steps 3 --warmup 1 > "$OUT/c5_rollout.json"
for f in "$OUT"/*.json; do python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],round(d['value']/1e6,2),round(d['ms_per_step'],3))" "$f"; done
