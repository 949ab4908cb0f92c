#!/bin/bash
# One GPU session: full GPU test suite, default bench line, rocprofv3 kernel stats of the bench.
# usage: bash tools/gpu_round.sh <tag>
set -e
TAG=${1:-run}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || { tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/$TAG
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 $OLDPWD/bench.py --steps 10 --no-cpu-baseline --no-host-rate > $OUT/prof_bench.log 2>&1) || { tail -20 $OUT/prof_bench.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
