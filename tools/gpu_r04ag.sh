set -e
R=$PWD; OUT=$R/gpurun_out/r04ag; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for lib in p3 cur; do
    if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
    echo "$lib $(timeout -k 10 120 python tools/dense_invert_time.py --iters 20)"
  done
done
unset NTC_GF256_LIB
echo "dnclk $(NTC_GF256_LIB=exp/libntc_gf256_dnclk.so timeout -k 10 120 python tools/dense_clock.py | cut -c1-260)"
timeout -k 10 300 python bench.py --config k1024dense --no-host-rate > $OUT/bench_k1024dense.log 2>&1 || { tail -20 $OUT/bench_k1024dense.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/bench_k1024dense.log') if l.startswith('{')][-1]); print('k1024dense', d['value'], d['kernels_ms'])"
