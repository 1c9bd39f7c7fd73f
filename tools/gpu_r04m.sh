#!/bin/bash
# round 4: ACL_NONE (rule-independent verifyACL veto) — GPU parity, then c3adv / c3 / c3r1 K1,
# then c3adv's PMC passes and rocprof trace for this build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_m}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_adverse.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "adverse or kat or random or synthetic or two_role" > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3adv c3 c3r1; do
  timeout -k 10 400 python3 bench.py --config $cfg --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_$cfg.log 2>&1 || exit $?
  echo "$cfg: $(grep -o '"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*' $O/ab_$cfg.log | tr '\n' ' ')"
done
TAG=r04_final CONFIGS="c3adv" bash tools/gpu_pmc_r04.sh || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_final/prof_c3adv -o run --output-format csv -- python3 bench.py --config c3adv --steps 20 --warmup 5 --e2e-requests 0 --no-pcie > gpurun_out/r04_final/bench_c3adv.log 2>&1 || exit $?
grep '^{' gpurun_out/r04_final/bench_c3adv.log | cut -c1-300
echo done
