#!/bin/bash
# round 4: K1 occupancy A/B on the hinted build (5 waves/SIMD product vs 4 and 6), and the
# codec's wave-aligned class runs forced off / on (ACS_AB_CODEC_PAD), same call, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_o}
mkdir -p $O
for cfg in c3adv c3 c3r1; do
  for rep in 1 2; do
    for v in prod k1w4 k1w6 pad0 pad1; do
      args=""; pad=""
      case $v in k1w*) args="--lib access-control-srv_amd/lib/variants/$v.so" ;; pad*) pad=${v#pad} ;; esac
      ACS_AB_CODEC_PAD=$pad timeout -k 10 400 python3 bench.py --config $cfg $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_${cfg}_${v}_$rep.log 2>&1 || exit $?
      echo "$cfg $v $rep: $(grep -o '"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' $O/ab_${cfg}_${v}_$rep.log | tr '\n' ' ')"
    done
  done
done
echo done
