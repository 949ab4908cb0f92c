set -e
R=$PWD; OUT=$R/gpurun_out/r04p; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_$i.log 2>&1 || { tail -20 $OUT/driver_$i.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/driver_$i.log') if l.startswith('{')][-1]); print('driver', d['value'], d['ms_per_step'], d['warmup'], d['warmup_steps_run'], d['kernels_fit_in_step'], d['verified'].get('oracle_slice_bit_exact'))"
done
