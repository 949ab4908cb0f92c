set -e
R=$PWD; OUT=$R/gpurun_out/r04aj; mkdir -p $OUT
NTC_GF256_LIB=exp/libntc_gf256_xr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for lib in cur xr; do
    if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
    echo "$lib $(timeout -k 10 120 python tools/dense_invert_time.py --iters 20)"
  done
done
echo "xrclk $(NTC_GF256_LIB=exp/libntc_gf256_xrclk.so timeout -k 10 120 python tools/dense_clock.py | cut -c1-260)"
