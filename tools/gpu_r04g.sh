set -e
R=$PWD; OUT=$R/gpurun_out/r04g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for lib in base cur; do
    if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
    echo "$lib $(timeout -k 10 120 python tools/dense_invert_time.py --iters 20)"
  done
done
unset NTC_GF256_LIB
for lib in dnclk clk5; do
  echo "$lib $(NTC_GF256_LIB=exp/libntc_gf256_$lib.so timeout -k 10 120 python tools/dense_clock.py | cut -c1-400)"
done
for lib in clk3 clk5 clk3 clk5; do
  echo "$lib $(NTC_GF256_LIB=exp/libntc_gf256_$lib.so timeout -k 10 120 python tools/plan_clock.py k128r32s4096 | cut -c1-420)"
done
for lib in base cur; do
  if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/bench_$lib.log 2>&1 || { tail -30 $OUT/bench_$lib.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$lib.log') if l.startswith('{')][-1]); print('$lib', d['value'], d['kernels_ms'])"
done
unset NTC_GF256_LIB
timeout -k 10 300 python bench.py --config k1024dense --no-cpu-baseline > $OUT/bench5.log 2>&1 || { tail -30 $OUT/bench5.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/bench5.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
