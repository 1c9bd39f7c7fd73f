#!/bin/bash
# round 4: one-class waves read their class's verdicts from LDS also when they hold composed
# lanes (product) vs the L2 form (nouni) — GPU parity first, then same-call alternating A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_q}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py tests/test_adverse.py tests/test_codec.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c4 c3r1 c2 c3adv; do
  for rep in 1 2; do
    for v in prod nouni; do
      args=""; [ $v != prod ] && args="--lib access-control-srv_amd/lib/variants/$v.so"
      timeout -k 10 400 python3 bench.py --config $cfg $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_${cfg}_${v}_$rep.log 2>&1 || exit $?
      echo "$cfg $v $rep: $(grep -o '"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*\|"mismatches": [0-9]*' $O/ab_${cfg}_${v}_$rep.log | tr '\n' ' ')"
    done
  done
done
echo done
