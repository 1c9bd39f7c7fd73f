#!/bin/bash
# One GPU session: gpu tests, smoke, bench, rocprof kernel-trace.  Each GPU step has its own
# time limit; a crash/abort/timeout (rc not in {0,1}) stops the script before any further GPU use.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "$OUT/$name.log"
  tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ -n "$STRICT" ]; }; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests smoke bench prof"}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread ;;
    tests_quick) step pytest_gpu_quick 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "kats or random_diff or synthetic_config or role_factor or large_store" ;;
    rehearse) step rehearse_launcher 600 env ACS_BENCH_REHEARSAL=1 python bench.py --gpus 2 --config c2 --steps 5 --warmup 1 --no-cpu-baseline ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py --steps 20 --warmup 3 ;;
    bench2) step bench_c2 600 python bench.py --config c2 --steps 20 --warmup 3 ;;
    nosort) step bench_nosort 600 python bench.py --steps 5 --warmup 1 --no-sort --no-cpu-baseline ;;
    quick) step bench_quick 600 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-pcie ;;
    quick3) step bench_c3_quick 900 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie ;;
    bench3) step bench_c3 900 python bench.py --config c3 --steps 5 --warmup 1 ;;
    prof3) step rocprof_c3 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof3" -o run --output-format csv -- python3 bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --e2e-requests 0 ;;
    quick5) step bench_c5_quick 1200 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie ;;
    ab) # VARIANTS: experiment builds (build.build_variant, compile-time ACS_AB_* flags) vs the product
        for cfg in ${AB_CONFIGS:-c2 c3}; do
          st=20; [ "$cfg" = c3 ] && st=5
          for rep in $(seq 1 ${AB_REPS:-2}); do
            step "ab_${cfg}_product_$rep" 900 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline --no-pcie --e2e-requests 0
            for v in ${VARIANTS:-}; do
              step "ab_${cfg}_${v}_$rep" 900 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline --no-pcie --e2e-requests 0 \
                --lib access-control-srv_amd/lib/variants/$v.so
            done
          done
        done ;;
    abtest) for v in ${VARIANTS:-}; do
          step "pytest_gpu_$v" 600 env ACS_MI355X_LIB=access-control-srv_amd/lib/variants/$v.so \
            python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "kats or random_diff or synthetic_config"
        done ;;
    phase5) step phase_c5 900 python tools/phase_prof.py c5 1000000 ;;
    phase3) step phase_c3 900 python tools/phase_prof.py c3 2000000 ;;
    quick4) step bench_c4_quick 900 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-pcie ;;
    c4) step bench_c4 900 python bench.py --config c4 --steps 10 --warmup 2 ;;
    c5) step bench_c5 1200 python bench.py --config c5 --steps 5 --warmup 1 --cpu-seconds 150 --no-pcie ;;
    c5shard) step bench_c5_rule_shard 1200 python bench.py --config c5 --rule-shard --steps 5 --warmup 1 --no-cpu-baseline ;;
    shard) step bench_rule_shard 600 python bench.py --rule-shard --steps 20 --warmup 3 --no-cpu-baseline ;;
    shard3) step bench_c3_rule_shard 900 python bench.py --config c3 --rule-shard --steps 5 --warmup 1 --no-cpu-baseline ;;
    prof4) step rocprof_c4 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof4" -o run --output-format csv -- python3 bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-pcie ;;
  esac
done
echo "== done"
