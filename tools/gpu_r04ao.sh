set -e
R=$PWD; OUT=$R/gpurun_out/r04ao; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --config k1024dense > $OUT/bench_k1024dense.log 2>&1 || { tail -20 $OUT/bench_k1024dense.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/bench_k1024dense.log') if l.startswith('{')][-1]); print('k1024dense', d['value'], d['kernels_ms'])"
