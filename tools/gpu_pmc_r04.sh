#!/bin/bash
# PMC passes (tools/pmc.sh: one rocprofv3 --pmc run per counter group) for round-4 builds;
# CONFIGS="c3 c3adv ..." picks the configs, TAG the output directory.  A failing pass stops
# the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
set -o pipefail
TAG=${TAG:-r04_pmc}
for cfg in ${CONFIGS:-c3 c3r1 c3adv c2 c5 c4}; do
  case $cfg in
    c3|c3r1) n=10000000 ;;
    *) n=1000000 ;;
  esac
  kern=is_allowed_kernel
  [ $cfg = c4 ] && kern=what_is_allowed_kernel
  echo "=== $cfg ($(date +%T))"
  PMC_OUT=gpurun_out/$TAG/pmc_$cfg CFG=$cfg KERNEL=$kern KEY=$cfg/n$n/w1/requests \
    TRAFFIC_SOURCE=profiles/$TAG/pmc_$cfg bash tools/pmc.sh || exit $?
  cp gpurun_out/$TAG/pmc_$cfg/traffic.json gpurun_out/$TAG/traffic_$cfg.json 2>/dev/null
done
echo "=== pmc done"
