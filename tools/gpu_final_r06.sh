#!/bin/bash
# Round-6 end-of-round evidence at one commit.
#   part A: every GPU test, smoke, the default bench line, the driver's command, the other
#           configs' lines and the per-packet line
#   part B: rocprofv3 kernel trace (+ stats) of the default command, then the PMC passes
#           (tools/gpu_pmc.sh) of the three headline shapes
# usage: bash tools/gpu_final_r06.sh <tag> A|B
set -o pipefail
TAG=$1; PART=$2; R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "[$name] $*"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
         tail -2 $OUT/$name.log | cut -c1-300; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; exit $rc; }; }
if [ "$PART" = A ]; then
  step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench_k128r32s4096 400 python bench.py
  step bench_driver_cmd 400 python bench.py --steps 20 --warmup 5
  step bench_k128r32s4096_mixed 400 python bench.py --mixed
  step bench_k32r8s1024 400 python bench.py --config k32r8s1024
  step bench_k128r32s1500 400 python bench.py --config k128r32s1500
  step bench_k1024dense 400 python bench.py --config k1024dense
  step per_packet 400 python bench.py --per-packet --pp-reps 5
  # more region-MAC work per packet: 4 KiB payloads; a repair every 2 sources
  step per_packet_s4096 400 python bench.py --per-packet --pp-reps 3 --size 4096 --c-items 64
  step per_packet_rate2 400 python bench.py --per-packet --pp-reps 3 --rate 2
  step gfw_bench 300 python tools/bench_gfw.py
else
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-host-rate > $OUT/trace.log 2>&1) || { tail -20 $OUT/trace.log; exit 1; }
  echo "trace done"
  timeout -k 10 1200 bash tools/gpu_pmc.sh $TAG/pmc "k128r32s4096 k32r8s1024 k128r32s1500 k1024dense" || exit 1
fi
echo "PART $PART DONE"
