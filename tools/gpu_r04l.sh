set -e
R=$PWD; OUT=$R/gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_shapes.py tests/test_gpu_large_window.py tests/test_gpu_batch.py tests/test_gpu_capi.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in clkb clk6 clkb clk6; do
  echo "$lib $(NTC_GF256_LIB=exp/libntc_gf256_$lib.so timeout -k 10 120 python tools/plan_clock.py k128r32s4096 | cut -c1-330)"
done
echo "clk6 c4 $(NTC_GF256_LIB=exp/libntc_gf256_clk6.so timeout -k 10 120 python tools/plan_clock.py k128r32s1500 8192 | cut -c1-330)"
for lib in base cur base cur; do
  if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/bench_$lib.log 2>&1 || { tail -30 $OUT/bench_$lib.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$lib.log') if l.startswith('{')][-1]); print('$lib', d['value'], d['kernels_ms'])"
done
unset NTC_GF256_LIB
for C in k128r32s1500 k32r8s1024; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-host-rate > $OUT/bench_$C.log 2>&1 || { tail -30 $OUT/bench_$C.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$C.log') if l.startswith('{')][-1]); print('$C', d['value'], d['kernels_ms'])"
done
