set -e
# driver-command ramp: bench value at --steps 20 for several warmups, and with the copy probe first
R=$PWD; OUT=$R/gpurun_out/r04m; mkdir -p $OUT
for v in "5 0" "0 0" "10 0" "30 0" "100 0" "5 200" "5 0"; do
  set -- $v
  NTC_BENCH_PROBE_FIRST=$2 timeout -k 10 300 python bench.py --steps 20 --warmup $1 --no-cpu-baseline --no-host-rate > $OUT/b_w$1_p$2.log 2>&1 || { tail -20 $OUT/b_w$1_p$2.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/b_w$1_p$2.log') if l.startswith('{')][-1]); print('W=$1 probe=$2', d['value'], d['ms_per_step'], d.get('ms_per_step_profiled'), d['kernels_ms'])"
done
