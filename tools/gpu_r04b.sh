set -e
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_shapes.py tests/test_gpu_pipeline.py tests/test_gpu_wire.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04b/pytest.log 2>&1 || { tail -30 gpurun_out/r04b/pytest.log; exit 1; }
tail -1 gpurun_out/r04b/pytest.log
bash tools/ab_lib.sh exp/libntc_gf256_base.so
NTC_GF256_LIB=exp/libntc_gf256_clk.so timeout -k 10 120 python tools/plan_clock.py k128r32s4096 > gpurun_out/r04b/plan_clock3.json
cat gpurun_out/r04b/plan_clock3.json
NTC_GF256_LIB=exp/libntc_gf256_clk.so timeout -k 10 120 python tools/plan_clock.py k128r32s1500 8192 > gpurun_out/r04b/plan_clock4.json
cat gpurun_out/r04b/plan_clock4.json
timeout -k 10 300 python bench.py > gpurun_out/r04b/bench.log 2>&1 || { tail -30 gpurun_out/r04b/bench.log; exit 1; }
tail -1 gpurun_out/r04b/bench.log | cut -c1-300
