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
# the driver's own command
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver_cmd.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_driver_cmd.log; exit 1; }
tail -1 gpurun_out/$TAG/bench_driver_cmd.log | cut -c1-160
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/$TAG
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 $OLDPWD/bench.py --steps 10 --no-cpu-baseline --no-host-rate > $OUT/prof_bench.log 2>&1) || { tail -20 $OUT/prof_bench.log; exit 1; }
python tools/trace_timed.py $OUT/prof/run_kernel_trace.csv --timed 10 --total 50 --skip-last 10 --bench $OUT/prof_bench.log > $OUT/kernel_trace_timed.json
timeout -k 10 300 python bench.py --per-packet > $OUT/per_packet.log 2>&1 || { tail -20 $OUT/per_packet.log; exit 1; }
tail -1 $OUT/per_packet.log | cut -c1-200
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
