#!/bin/bash
# PMC passes (tools/pmc.sh) for the round-3 build: c3, c2, c5 (K1) and c4 (K2), each config's
# four counter groups in runs of their own; a failing pass stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
set -o pipefail
for spec in "c3|is_allowed_kernel|c3/n10000000/w1/requests" "c2|is_allowed_kernel|c2/n1000000/w1/requests" \
            "c4|what_is_allowed_kernel|c4/n1000000/w1/requests" "c5|is_allowed_kernel|c5/n1000000/w1/requests"; do
  IFS='|' read -r cfg kern key <<< "$spec"
  [ -n "$ONLY" ] && [[ " $ONLY " != *" $cfg "* ]] && continue
  echo "=== $cfg ($(date +%T))"
  PMC_OUT=gpurun_out/pmc_$cfg CFG=$cfg KERNEL=$kern KEY=$key TRAFFIC_SOURCE=profiles/r03_pmc/pmc_$cfg \
    bash tools/pmc.sh || exit $?
  cp gpurun_out/pmc_$cfg/traffic.json gpurun_out/traffic_$cfg.json 2>/dev/null
done
echo "=== pmc round 3 done"
