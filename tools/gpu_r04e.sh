#!/bin/bash
# round 4: the HR owner-test memo — GPU parity subset, then K1 on c3 / c3r1 / c3adv / c5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_e}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py tests/test_adverse.py tests/test_compact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c3r1 c3adv c5; do
  timeout -k 10 400 python3 bench.py --config $cfg --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline $EXTRA > $O/ab_$cfg.log 2>&1 || exit $?
  echo "$cfg: $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*' $O/ab_$cfg.log | tr '\n' ' ')"
done
