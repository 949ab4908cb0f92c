#!/bin/bash
# rocprofv3 evidence for one bench config: kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes.
# usage: bash tools/gpu_profile.sh <tag> [config]
set -e
TAG=${1:-prof}; CFG=${2:-k128r32s4096}
R=$PWD; OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="$R/bench.py --config $CFG --no-cpu-baseline --no-host-rate"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats -o run -- python3 $B --steps 10 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 $B --steps 2 --warmup 1 > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- python3 $B --steps 2 --warmup 1 > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
find $OUT -name "*.csv" | sed "s|$R/||"
