# A/B of the key-padding mask form (T2O_KEY_MASK_TILE 1 = default, 0, 2) at 32 AGVs and the headline
AB_SERIAL= bash tools/ab_box.sh r5_km/a32 t2omca_amd/lib/ab_cur.so t2omca_amd/lib/ab_km0.so t2omca_amd/lib/ab_km2.so -- --agents 32 --batch 1024 --T 60 --steps 4 --warmup 2 || exit 1
AB_SERIAL= bash tools/ab_box.sh r5_km/head t2omca_amd/lib/ab_cur.so t2omca_amd/lib/ab_km0.so t2omca_amd/lib/ab_km2.so || exit 1
