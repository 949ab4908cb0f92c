set -e
R=$PWD; OUT=$R/gpurun_out/r04s; mkdir -p $OUT
NTC_GF256_LIB=exp/libntc_gf256_vsel.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "decode or plan" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in clk6 vselclk clk6 vselclk; do
  echo "$lib $(NTC_GF256_LIB=exp/libntc_gf256_$lib.so timeout -k 10 120 python tools/plan_clock.py k128r32s4096 | cut -c1-300)"
done
for lib in cur vsel cur vsel; do
  if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/b_$lib.log 2>&1 || { tail -20 $OUT/b_$lib.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/b_$lib.log') if l.startswith('{')][-1]); print('$lib', d['value'], d['kernels_ms'])"
done
