#!/bin/bash
# round 4: K1 prologue share (timing-only build: filter build + line read, no walk)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_l}
mkdir -p $O
for cfg in c3 c3r1 c3adv; do
  for v in prod prologue; do
    args=""; [ $v = prologue ] && args="--lib access-control-srv_amd/lib/variants/prologue.so"
    timeout -k 10 400 python3 bench.py --config $cfg $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline --parity-fraction 0 > $O/ab_${cfg}_$v.log 2>&1 || exit $?
    echo "$cfg $v: $(grep -o '"kernel_ms": [0-9.]*' $O/ab_${cfg}_$v.log)"
  done
done
echo done
