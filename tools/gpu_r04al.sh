set -e
R=$PWD; OUT=$R/gpurun_out/r04al; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -4 $OUT/pytest.log
