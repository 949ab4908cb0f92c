set -e
R=$PWD; OUT=$R/gpurun_out/r04r; mkdir -p $OUT
for lib in clk6 capclk; do
  echo "$lib c4 $(NTC_GF256_LIB=exp/libntc_gf256_$lib.so timeout -k 10 120 python tools/plan_clock.py k128r32s1500 8192 | cut -c1-600)"
done
for C in k128r32s1500 k128r32s4096; do
for lib in cur cap; do
  if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-host-rate > $OUT/b_${C}_$lib.log 2>&1 || { tail -20 $OUT/b_${C}_$lib.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/b_${C}_$lib.log') if l.startswith('{')][-1]); print('$C $lib', d['value'], d['kernels_ms'])"
done; done
