# Run ON THE GPU BOX: the env load-ordering A/B, then the round's final evidence run
bash tools/envord_box.sh || true
bash tools/r4_final.sh r4_final
