#!/bin/bash
# round 4: where the two-role c3 K1 time goes — phase profile (c3 with / without second roles)
# and a same-call A/B without target verdicts
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 300 python3 tools/phase_prof.py c3 10000000 0.5 > $O/phase_c3.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/phase_prof.py c3 10000000 0.0 > $O/phase_c3r1.log 2>&1 || exit $?
tail -14 $O/phase_c3.log $O/phase_c3r1.log
for spec in "prod|--config c3" "noverd|--config c3 --lib access-control-srv_amd/lib/variants/noverd.so"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_$name.log 2>&1 || exit $?
  echo "$name: $(grep -o '"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*' $O/ab_$name.log | tr '\n' ' ')"
done
