set -e
R=$PWD; OUT=$R/gpurun_out/r04k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_capi.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python bench.py --per-packet > $OUT/per_packet.log 2>&1 || { tail -30 $OUT/per_packet.log; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$OUT/per_packet.log') if l.startswith('{')][-1])
print(d['value'], d['speedup_batched_vs_cpu'], d['cpu_baseline']['value'])
for k in ('gpu_batched','gpu_immediate','cpu_oracle'): print(k, {x: d['c_level'][k].get(x) for x in ('encode_s','decode_s','packets_per_s','all_runs_s')})
"
