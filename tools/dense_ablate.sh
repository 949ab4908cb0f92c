#!/bin/bash
# Dense inversion A/B (tools/dense_invert_time.py, n = 1024): the dense parity suite first, then
# panel kinds / NTC_DENSE_ABLATE timing ablations interleaved.  usage: bash tools/dense_ablate.sh <tag> ["kind abl" ...]
set -e
TAG=${1:-dense_abl}; shift || true; OUT=gpurun_out/$TAG; mkdir -p $OUT
VARIANTS=("$@"); [ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=("ra 0" "own 0")
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > $OUT/dense_tests.log 2>&1 || { tail -30 $OUT/dense_tests.log; exit 1; }
echo "dense parity: $(tail -1 $OUT/dense_tests.log)"
for rep in 1 2; do
  for v in "${VARIANTS[@]}"; do set -- $v
    NTC_DENSE_PANEL=$1 NTC_DENSE_ABLATE=$2 timeout -k 10 120 python tools/dense_invert_time.py --iters 30 2>/dev/null | tee -a $OUT/invert_times.jsonl
  done
done
