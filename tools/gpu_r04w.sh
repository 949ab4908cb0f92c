set -e
R=$PWD; OUT=$R/gpurun_out/r04w; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_shapes.py tests/test_gpu_large_window.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for C in k128r32s4096 k128r32s1500 k32r8s1024; do
for rep in 1 2; do
for lib in cur planold; do
  if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-host-rate > $OUT/b_${C}_${lib}_$rep.log 2>&1 || { tail -20 $OUT/b_${C}_${lib}_$rep.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/b_${C}_${lib}_$rep.log') if l.startswith('{')][-1]); print('$C $lib', d['value'], d['kernels_ms'])"
done; done; done
