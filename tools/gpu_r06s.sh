#!/bin/bash
# Round 6: K2 work bits ORed into the copied row with device atomics (no template re-read) vs the
# rewrite of whole chunks; then PMC passes for c2 and c5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_s}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product k2atomic
step 300 ab_c4_131k python3 -u tools/k1_ab.py c4 131072 product k2atomic
step 400 ab_c4_4m python3 -u tools/k1_ab.py c4 4000000 product k2atomic
mkdir -p gpurun_out/r06_final_c
for cfg in c2 c5; do
  PMC_OUT=gpurun_out/r06_final_c/pmc_$cfg CFG=$cfg KERNEL=is_allowed_kernel timeout -k 10 600 bash tools/pmc.sh > gpurun_out/r06_final_c/pmc_$cfg.log 2>&1 || { echo "STOP pmc $cfg"; exit 1; }
  tail -n 2 gpurun_out/r06_final_c/pmc_$cfg.log
done
echo done
