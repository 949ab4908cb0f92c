set -e
bash tools/gpu_pmc.sh r04_cfg "k128r32s1500 k1024dense"
bash tools/gpu_pmc.sh r04_mixed k128r32s4096 --mixed
bash tools/gpu_r04m.sh
