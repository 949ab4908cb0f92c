set -e
mkdir -p gpurun_out/r04d
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04d/pytest.log 2>&1 || { tail -30 gpurun_out/r04d/pytest.log; exit 1; }
tail -1 gpurun_out/r04d/pytest.log
for rep in 1 2; do
  for lib in dn0 nolook cur; do
    unset NTC_DENSE_LOOKAHEAD
    if [ $lib = cur ]; then unset NTC_GF256_LIB; elif [ $lib = nolook ]; then unset NTC_GF256_LIB; export NTC_DENSE_LOOKAHEAD=0; else export NTC_GF256_LIB=exp/libntc_gf256_$lib.so; fi
    echo "$lib $(timeout -k 10 120 python tools/dense_invert_time.py --iters 20)"
  done
  unset NTC_DENSE_LOOKAHEAD
done
unset NTC_GF256_LIB
timeout -k 10 300 python bench.py --config k1024dense --no-cpu-baseline > gpurun_out/r04d/bench5.log 2>&1 || { tail -30 gpurun_out/r04d/bench5.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/r04d/bench5.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
