#!/bin/bash
# round 4: rule-sharded library handle + whatIsAllowed split (GPU tests), then the current
# numbers on c3, c3r1, c3adv, c2, c4, c5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_i}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_rule_shard_lib.py tests/test_multi_device.py tests/test_adverse.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c3r1 c3adv c2 c4 c5; do
  timeout -k 10 500 python3 bench.py --config $cfg --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_$cfg.log 2>&1 || exit $?
  echo "$cfg: $(grep -o '"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*' $O/ab_$cfg.log | tr '\n' ' ')"
done
echo done
