set -e
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_shapes.py tests/test_gpu_large_window.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04c/pytest.log 2>&1 || { tail -30 gpurun_out/r04c/pytest.log; exit 1; }
tail -1 gpurun_out/r04c/pytest.log
for lib in clk0 clk2 clk3 clk0 clk2 clk3; do
  NTC_GF256_LIB=exp/libntc_gf256_$lib.so timeout -k 10 120 python tools/plan_clock.py k128r32s4096 > gpurun_out/r04c/pc3_$lib.json
  echo "$lib $(cat gpurun_out/r04c/pc3_$lib.json)" | cut -c1-330
done
NTC_GF256_LIB=exp/libntc_gf256_clk3.so timeout -k 10 120 python tools/plan_clock.py k128r32s1500 8192 | cut -c1-330
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > gpurun_out/r04c/bench.log 2>&1 || { tail -30 gpurun_out/r04c/bench.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/r04c/bench.log') if l.startswith('{')][-1]); print(d['value'], d['kernels_ms'])"
