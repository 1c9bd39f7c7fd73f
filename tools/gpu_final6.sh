#!/bin/bash
# Round 6 final measurement on the benchmarked tree.  PART=a: full GPU suite, smoke, bench lines for
# c3 / c4 / c3adv under rocprofv3 --kernel-trace --stats.  PART=b: K1 parity tests, bench lines for
# c3adv / c3r1 / c2 / c5 under rocprofv3.  PART=c: PMC passes (tools/pmc.sh) for c3, c4, c3adv, c3r1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_final}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
prof() { local cfg=$1; shift; step 600 bench_$cfg rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o run -- python3 -u bench.py "$@"; }
if [ "${PART:-a}" = a ]; then
  step 900 pytest_gpu python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
  step 300 smoke python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  prof c3 --steps 20 --warmup 5
  prof c4 --config c4 --steps 20 --warmup 5
  prof c3adv --config c3adv --steps 20 --warmup 5
elif [ "$PART" = b ]; then
  step 900 pytest_k1 python3 -u -m pytest tests/test_adverse.py tests/test_gpu.py tests/test_compact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
  prof c3adv --config c3adv --steps 20 --warmup 5
  prof c3r1 --config c3r1 --steps 20 --warmup 5
  prof c2 --config c2 --steps 20 --warmup 5
  prof c5 --config c5 --steps 20 --warmup 5
else
  for cfg in c3 c4 c3adv c3r1; do
    k=is_allowed_kernel; [ $cfg = c4 ] && k=what_is_allowed_kernel
    n=1000000; case $cfg in c3|c3r1) n=10000000;; esac
    PMC_OUT=$O/pmc_$cfg CFG=$cfg KERNEL=$k KEY=$cfg/n$n/w1/requests timeout -k 10 600 bash tools/pmc.sh > $O/pmc_$cfg.log 2>&1 || { echo "STOP pmc $cfg"; exit 1; }
    tail -n 2 $O/pmc_$cfg.log
  done
fi
echo done
