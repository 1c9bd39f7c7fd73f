#!/bin/bash
# round 4: c5 updateRule latency (default V8 heap), HR-memo A/B, c3 at 1M requests (batch-size
# effect beside c3adv), JS suites
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_f}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpucodec_js.py tests/test_multi_device.py tests/test_adverse.py -m gpu -x -q -s --timeout 550 --timeout-method thread > $O/pytest_js.log 2>&1
rc=$?; grep -a "c5 update latency\|passed\|failed" $O/pytest_js.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
for spec in "c3_1m|--config c3 --requests 1000000" "c3adv|--config c3adv" "c3_prod|--config c3" "c3_nomemo|--config c3 --lib access-control-srv_amd/lib/variants/nomemo.so"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 400 python3 bench.py $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_$name.log 2>&1 || exit $?
  echo "$name: $(grep -o '"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*' $O/ab_$name.log | tr '\n' ' ')"
done
echo done
