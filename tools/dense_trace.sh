#!/bin/bash
# rocprofv3 kernel trace of the dense inversion (tools/dense_invert_time.py) under the given
# NTC_DENSE_LOOKAHEAD values.  usage: bash tools/dense_trace.sh <tag> [la ...]
set -e
TAG=${1:-dense_trace}; shift || true; R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
LAS=("$@"); [ ${#LAS[@]} -eq 0 ] && LAS=(1 0)
cd /tmp
for la in "${LAS[@]}"; do
  NTC_DENSE_LOOKAHEAD=$la timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $OUT/la$la -o run -- python3 $R/tools/dense_invert_time.py --iters 10 > $OUT/la$la.log 2>&1 || { tail -20 $OUT/la$la.log; exit 1; }
  python3 $R/tools/dense_trace_summary.py $(find $OUT/la$la -name "*kernel_trace.csv") | tee $OUT/la$la.summary
done
