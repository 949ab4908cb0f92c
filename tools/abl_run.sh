#!/bin/bash
# Timing-only runs of variant libraries / environments (ablation builds fail verification:
# their exit status 3 is expected).  usage: bash tools/abl_run.sh "<lib>|<env>" ... -- [bench args]
OUT=gpurun_out/abl; mkdir -p $OUT
SPECS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do SPECS+=("$1"); shift; done; shift
n=0
for spec in "${SPECS[@]}"; do
  lib=${spec%%|*}; envs=${spec#*|}
  n=$((n+1))
  env NTC_GF256_LIB=$lib $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate "$@" > $OUT/run_$n.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "[$spec] rc=$rc"; tail -5 $OUT/run_$n.log; exit $rc; }
  python -c "import json; d=json.loads([l for l in open('$OUT/run_$n.log') if l.startswith('{')][-1]); print('[$spec] rc=$rc', d['value'], d['ms_per_step'], d['kernels_ms'])"
done
