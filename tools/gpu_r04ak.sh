set -e
R=$PWD; OUT=$R/gpurun_out/r04ak; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do echo "cur $(timeout -k 10 120 python tools/dense_invert_time.py --iters 20)"; done
for n in 512 256 96; do echo "cur n=$n $(timeout -k 10 120 python tools/dense_invert_time.py --n $n --iters 20)"; done
echo "dnclk $(NTC_GF256_LIB=exp/libntc_gf256_dnclk.so timeout -k 10 120 python tools/dense_clock.py | cut -c1-260)"
timeout -k 10 300 python bench.py --config k1024dense > $OUT/bench_k1024dense.log 2>&1 || { tail -20 $OUT/bench_k1024dense.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/bench_k1024dense.log') if l.startswith('{')][-1]); print('k1024dense', d['value'], d['kernels_ms'], d['verified'])"
