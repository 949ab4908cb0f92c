#!/bin/bash
# Round-6 GPU steps, one parametrised script (round 5: tools/gpu_r05.sh).
# usage: bash tools/gpu_r06.sh <tag> <step>[,<step>...] [bench args...]
#   steps: tests (pytest -m gpu), dense (test_gpu_dense.py only), mb (tools/mb_issue),
#          bench (default bench line), c2|c4|c5 (per-config lines), smoke, batch (adaptor
#          tests), pp (per-packet line), ppprof / ppsamp (flush / sampling profiles), c4pmc,
#          surface, gatherab / gfwab (A/B against $AB_OTHER), ksplit (config-5 sweep),
#          slice (config 5 with / without pre-sliced sources)
#   round-end evidence: tools/gpu_final_r05.sh
set -o pipefail
TAG=$1; STEPS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$name] $*"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?;
        tail -3 $OUT/$name.log; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; exit $rc; }; }
IFS=, read -ra S <<< "$STEPS"
for s in "${S[@]}"; do
  case $s in
    tests) run pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread ;;
    dense) run dense 300 python -u -m pytest tests/test_gpu_dense.py -x -q -m gpu --timeout 240 --timeout-method thread ;;
    mb) run mb_issue 300 tools/mb_issue ;;
    mbmix) run mb_mix 300 tools/mb_mix ;;
    bench) run bench 300 python bench.py "$@" ;;
    c2) run bench_c2 300 python bench.py --config k32r8s1024 "$@" ;;
    c4) run bench_c4 300 python bench.py --config k128r32s1500 "$@" ;;
    c5) run bench_c5 300 python bench.py --config k1024dense "$@" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    ab) run ab_lib 900 bash tools/ab_lib.sh "$AB_OTHER" "$@" ;;
    abenv) run ab_env 900 bash tools/ab_env.sh "$AB_A" "$AB_B" "$@" ;;
    abl) eval "run abl 900 bash tools/abl_run.sh $ABL -- $*" ;;
    batch) run batch 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_capi.py tests/test_gpu_gather.py -x -q -m gpu --timeout 120 --timeout-method thread ;;
    surface) run surface 600 python -u -m pytest tests/test_gpu_cpp_surface.py -x -q -m gpu --timeout 300 --timeout-method thread ;;
    ppprof) for M in batched async; do   # per-packet C driver with the flush profile (NTC_BATCH_PROFILE)
        NTC_BATCH_PROFILE=1 run pp_prof_$M 120 tests/_build/pp_driver $M 256 128 1024 32 4 10 7; done ;;
    ppsamp) for M in batched async; do for P in enc dec; do  # host sampling profile (exp/prof build)
        NTC_SAMPLER_GATED=1 PP_PROFILE=$P NTC_SAMPLER_OUT=$OUT/samples_${M}_$P.txt run pp_samp_${M}_$P 120 exp/prof/pp_driver_prof $M 256 128 1024 32 4 10 7; done; done ;;
    pp) run per_packet 400 python bench.py --per-packet "$@" ;;
    c4pmc)  # config-4 read traffic by row pitch: FETCH_SIZE and the raw TCC read-request counters
      for ST in ${C4_STRIDES:-1504 1536}; do
        B="$PWD/bench.py --config k128r32s1500 --stride $ST --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
        run c4_line_$ST 300 python bench.py --config k128r32s1500 --stride $ST --no-cpu-baseline --no-host-rate
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OLDPWD/$OUT/c4pmc_$ST/fetch -o run -- python3 $B > $OLDPWD/$OUT/c4pmc_$ST.fetch.log 2>&1) || { echo "fetch pass $ST failed"; exit 1; }
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OLDPWD/$OUT/c4pmc_$ST/write -o run -- python3 $B > $OLDPWD/$OUT/c4pmc_$ST.write.log 2>&1) || { echo "write pass $ST failed"; exit 1; }
        echo "c4pmc $ST done"
      done
      for ST in ${C4_STRIDES:-1504 1536}; do
        B="$PWD/bench.py --config k128r32s1500 --stride $ST --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -f csv -d $OLDPWD/$OUT/c4pmc_$ST/req -o run -- python3 $B > $OLDPWD/$OUT/c4pmc_$ST.req.log 2>&1) || { echo "req pass $ST failed (counter names?)"; tail -3 $OUT/c4pmc_$ST.req.log; break; }
      done ;;
    gatherab)  # adaptor tests on the in-tree libraries, then with libntc_gf256.so = $AB_OTHER (scratch copy)
      T="tests/test_gpu_gather.py tests/test_gpu_batch.py tests/test_gpu_capi.py"
      run gather_cur 300 python -u -m pytest $T -q -m gpu --timeout 120 --timeout-method thread
      cp "$AB_OTHER" netcode_amd/libntc_gf256.so
      run gather_other 300 python -u -m pytest $T -q -m gpu --timeout 120 --timeout-method thread ;;
    gfw)       # GF(2^w) parity (both kernel forms), then both forms timed interleaved
      run gfw_tests 300 python -u -m pytest tests/test_gpu_gfw.py -x -q -m gpu --timeout 120 --timeout-method thread
      run gfw_bench 300 python tools/bench_gfw.py ;;
    gfwab)     # GF(2^w) parity, then tools/bench_gfw.py interleaved against $AB_OTHER
      run gfw_tests 300 python -u -m pytest tests/test_gpu_gfw.py -x -q -m gpu --timeout 120 --timeout-method thread
      for rep in 1 2; do
        run gfw_cur_$rep 120 python tools/bench_gfw.py
        NTC_GF256_LIB=$AB_OTHER run gfw_other_$rep 120 python tools/bench_gfw.py
      done ;;
    ksplit)    # config-5 split-k part counts ($KS, default "3 4 5 6"), two interleaved reps
      for rep in 1 2; do for k in ${KS:-3 4 5 6}; do
        NTC_GF256_KSPLIT=$k run ks${k}_$rep 300 python bench.py --config k1024dense --no-cpu-baseline --no-host-rate
      done; done ;;
    slice)     # config 5 with / without pre-sliced sources (NTC_GF256_SLICE), two interleaved reps,
               # after the tall-encode parity cases and the dense tests
      run slice_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense.py -x -q -m gpu -k "400 or 390 or dense" --timeout 240 --timeout-method thread
      for rep in 1 2; do for v in 0 1; do
        NTC_GF256_SLICE=$v run slice${v}_$rep 300 python bench.py --config k1024dense --no-cpu-baseline --no-host-rate
      done; done ;;
    ptest)     # parity of the tile-pair MAC (NTC_GF256_MAC=paired) on every encode / decode case,
               # for each sources-per-turn / slot-set shape
      for v in "1 4" "1 3" "2 3"; do set -- $v
        NTC_GF256_PAIRJ=$1 NTC_GF256_PAIRSETS=$2 run ptest_$1$2 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "paired" --timeout 240 --timeout-method thread
      done ;;
    pairab)    # bench lines interleaved: solo tiles vs tile pairs ($PAB: "kind J NS lib|-" ...), $REPS reps
      for rep in $(seq ${REPS:-2}); do for v in ${PAB:-"bitslice,1,4,-" "paired,1,3,-" "paired,1,4,-" "paired,2,3,-"}; do
        IFS=, read -r K J NS LIB <<< "$v"; [ "$LIB" = - ] && LIB=
        NTC_GF256_LIB=$LIB NTC_GF256_MAC=$K NTC_GF256_PAIRJ=$J NTC_GF256_PAIRSETS=$NS run pab_$K$J$NS$(basename "${LIB:-x}" .so)_$rep 300 python bench.py --no-cpu-baseline --no-host-rate $BARGS
      done; done
      for f in $OUT/pab_*.log; do python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d['kernels_ms'])"; done ;;
    c4tile)    # config-4 read traffic with one row tile per generation (r = 16) against two (r = 32):
               # if the two tiles refetch sources from HBM, the excess over the rows' bytes vanishes at r = 16
      for R in 16 32; do
        B="$PWD/bench.py --config k128r32s1500 --r $R --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OLDPWD/$OUT/c4tile_$R/fetch -o run -- python3 $B > $OLDPWD/$OUT/c4tile_$R.fetch.log 2>&1) || { echo "fetch pass r=$R failed"; exit 1; }
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OLDPWD/$OUT/c4tile_$R/write -o run -- python3 $B > $OLDPWD/$OUT/c4tile_$R.write.log 2>&1) || { echo "write pass r=$R failed"; exit 1; }
        echo "c4tile r=$R done"
      done ;;
    parity) run parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_shapes.py -x -q -m gpu --timeout 240 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
