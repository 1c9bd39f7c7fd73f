#!/bin/bash
# round-4 final, part B: PMC passes (tools/pmc.sh groups) for CONFIGS, then rocprof kernel
# traces of the same configs' bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
TAG=${TAG:-r04_final}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG CONFIGS="${CONFIGS:-c3 c3r1 c3adv}" bash tools/gpu_pmc_r04.sh || exit $?
for cfg in ${CONFIGS:-c3 c3r1 c3adv}; do
  [ $cfg = c3 ] && continue  # part A profiles c3
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 20 --warmup 5 --e2e-requests 0 --no-pcie > $O/bench_$cfg.log 2>&1 || exit $?
  grep '^{' $O/bench_$cfg.log | cut -c1-300
done
echo done
