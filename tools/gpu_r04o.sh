#!/bin/bash
# round 4: K1 occupancy A/B on the hinted build (5 waves/SIMD product vs 4 and 6), same call,
# alternating: c3, c3r1, c3adv
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_o}
mkdir -p $O
for cfg in c3 c3r1 c3adv; do
  for rep in 1 2; do
    for v in prod k1w4 k1w6; do
      args=""; [ $v != prod ] && args="--lib access-control-srv_amd/lib/variants/$v.so"
      timeout -k 10 400 python3 bench.py --config $cfg $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_${cfg}_${v}_$rep.log 2>&1 || exit $?
      echo "$cfg $v $rep: $(grep -o '"kernel_ms": [0-9.]*' $O/ab_${cfg}_${v}_$rep.log)"
    done
  done
done
echo done
