#!/bin/bash
# round 4: non-temporal K2 row stores A/B (same call, alternating), c4 + the c4 GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_k}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "what_is_allowed or overflow" > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in prod nont; do
    args=""; [ $v = nont ] && args="--lib access-control-srv_amd/lib/variants/nont.so"
    timeout -k 10 400 python3 bench.py --config c4 $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_c4_${v}_$rep.log 2>&1 || exit $?
    echo "c4 $v $rep: $(grep -o '"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*' $O/ab_c4_${v}_$rep.log | tr '\n' ' ')"
  done
done
echo done
