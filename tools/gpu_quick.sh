#!/bin/bash
# Quick GPU check: selected GPU tests (-k expression), then the default bench line.
# usage: bash tools/gpu_quick.sh <tag> "<pytest -k expr>" [bench args...]
set -e
TAG=${1:-quick}; KEXPR=${2:-}; shift 2 || true
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$KEXPR" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
timeout -k 10 300 python bench.py "$@" > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
