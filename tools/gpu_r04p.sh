#!/bin/bash
# round 4: wave-aligned class runs (ACS_AB_CODEC_PAD: 1 runs of equal class, 2 runs of equal
# (class, second class)) vs the product rule, and K1 at 4 waves/SIMD for ACL_NONE batches;
# same call, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_p}
mkdir -p $O
for cfg in c3 c3r1 c3adv c2; do
  for rep in 1 2; do
    for v in prod pad1 pad2; do
      ACS_AB_CODEC_PAD=${v#pad} ; [ $v = prod ] && ACS_AB_CODEC_PAD=
      ACS_AB_CODEC_PAD=$ACS_AB_CODEC_PAD timeout -k 10 400 python3 bench.py --config $cfg --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_${cfg}_${v}_$rep.log 2>&1 || exit $?
      echo "$cfg $v $rep: $(grep -o '"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' $O/ab_${cfg}_${v}_$rep.log | tr '\n' ' ')"
    done
  done
done
echo done
