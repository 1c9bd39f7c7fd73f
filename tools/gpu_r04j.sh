#!/bin/bash
# round 4: XCD-aware tiles A/B (same call): K1 / K2 with and without, c3 c3r1 c2 c4 c5 c3adv
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_j}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kat or random or synthetic" > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c3r1 c2 c4 c5 c3adv; do
  for v in prod noxcd; do
    args=""; [ $v = noxcd ] && args="--lib access-control-srv_amd/lib/variants/noxcd.so"
    timeout -k 10 400 python3 bench.py --config $cfg $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_${cfg}_$v.log 2>&1 || exit $?
    echo "$cfg $v: $(grep -o '"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*' $O/ab_${cfg}_$v.log | tr '\n' ' ')"
  done
done
echo done
