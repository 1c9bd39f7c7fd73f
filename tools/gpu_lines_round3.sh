#!/bin/bash
# Round-3 bench lines (each config with its parity / CPU-baseline leg) and the rocprof kernel
# summary of the default command; every step has its own time limit and a failure stops the
# script before any further GPU use.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/lines
mkdir -p $OUT
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "$OUT/$name.log"
  grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*\|"mismatches": [0-9]*\|"oracle_sample": [0-9]*' "$OUT/$name.log" | tr '\n' ' '; echo
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; tail -5 "$OUT/$name.log"; exit $rc; fi
}
for s in ${STEPS:-c2 c4 c5 c3r2 c3adv prof}; do
  case $s in
    c3) step bench_c3 400 python bench.py --steps 20 --warmup 5 ;;
    c2) step bench_c2 300 python bench.py --config c2 --steps 20 --warmup 5 --cpu-seconds 20 ;;
    c4) step bench_c4 600 python bench.py --config c4 --steps 10 --warmup 2 --cpu-seconds 60 ;;
    c5) step bench_c5 900 python bench.py --config c5 --steps 5 --warmup 1 --cpu-seconds 90 --no-pcie --e2e-requests 0 ;;
    c3r2) step bench_c3r2 600 python bench.py --config c3r2 --steps 10 --warmup 2 --cpu-seconds 20 --no-pcie ;;
    c3adv) step bench_c3adv 600 python bench.py --config c3adv --steps 10 --warmup 2 --cpu-seconds 20 --no-pcie ;;
    prof) step rocprof_c3 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --e2e-requests 0 ;;
  esac
done
echo "== lines done"
