set -e
R=$PWD; OUT=$R/gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_random_shapes.py tests/test_gpu_batch.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in base cur; do
  if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/bench_$lib.log 2>&1 || { tail -30 $OUT/bench_$lib.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$lib.log') if l.startswith('{')][-1]); print('$lib', d['value'], d['kernels_ms'])"
done
unset NTC_GF256_LIB
for fold in 0 1; do
  NTC_KSPLIT_FOLD=$fold timeout -k 10 300 python bench.py --config k1024dense --no-cpu-baseline > $OUT/bench5_f$fold.log 2>&1 || { tail -30 $OUT/bench5_f$fold.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench5_f$fold.log') if l.startswith('{')][-1]); print('fold$fold', d['value'], d['ms_per_step'], d['kernels_ms'], d.get('verified'))"
done
