#!/bin/bash
# Round-5 evidence: default bench line, per-packet line, rocprofv3 kernel trace of the default
# command (stats + the timed launches); usage: bash tools/gpu_evidence_r05.sh <tag>
set -o pipefail
TAG=${1:-ev}; R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 400 python bench.py --per-packet --pp-reps 3 > $OUT/per_packet.log 2>&1 || { tail -20 $OUT/per_packet.log; exit 1; }
python -c "import json; d=json.loads(open('$OUT/per_packet.log').read().strip().splitlines()[-1]); c=d['c_level']; print('pp', d['value'], d['speedup_batched_vs_cpu'], {k: (v['encode_s'], v['decode_s'], v.get('encode_flush_s'), v.get('decode_flush_s')) for k, v in c.items()})"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-host-rate > $OUT/trace.log 2>&1) || { tail -20 $OUT/trace.log; exit 1; }
echo "trace done"
