set -e
R=$PWD; OUT=$R/gpurun_out/r04t; mkdir -p $OUT
for G in 4096 8192 16384 8192 4096; do
  timeout -k 10 300 python bench.py --G $G --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > $OUT/b_G$G.log 2>&1 || { tail -20 $OUT/b_G$G.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/b_G$G.log') if l.startswith('{')][-1]); print('G=$G', d['value'], d['ms_per_step'], d['warmup_steps_run'], d['kernels_ms'], d['roofline']['frac'])"
done
