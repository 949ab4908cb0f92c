set -e
R=$PWD; OUT=$R/gpurun_out/r04q; mkdir -p $OUT
for C in k32r8s1024 k128r32s1500; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-host-rate > $OUT/b_$C.log 2>&1 || { tail -20 $OUT/b_$C.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/b_$C.log') if l.startswith('{')][-1]); print('$C', d['value'], d['ms_per_step'], d['warmup_steps_run'], d['kernels_ms'])"
done
