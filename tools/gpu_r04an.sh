set -e
R=$PWD; OUT=$R/gpurun_out/r04an; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for n in 1024 512 256 128 96; do
  for lib in prev cur; do
    if [ $lib = cur ]; then unset NTC_GF256_LIB; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
    echo "$lib n=$n $(timeout -k 10 120 python tools/dense_invert_time.py --n $n --iters 20)"
  done
done
