#!/bin/bash
# Round 6: PMC passes for c2 and c5 on the final tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_final_c
for cfg in c2 c5; do
  PMC_OUT=gpurun_out/r06_final_c/pmc_$cfg CFG=$cfg KERNEL=is_allowed_kernel timeout -k 10 600 bash tools/pmc.sh > gpurun_out/r06_final_c/pmc_$cfg.log 2>&1 || { echo "STOP pmc $cfg"; exit 1; }
  tail -n 2 gpurun_out/r06_final_c/pmc_$cfg.log
done
echo done
