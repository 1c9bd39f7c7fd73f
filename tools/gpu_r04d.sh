#!/bin/bash
# round 4: c5 bench line (1,000 oracle-checked requests), c3adv with one role association (the
# round-3 shape) beside the default, then PMC passes of c3 and c3adv
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r04_d
mkdir -p $O
timeout -k 10 500 python3 bench.py --config c5 --steps 10 --warmup 3 --e2e-requests 0 --no-pcie > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log | cut -c1-300
timeout -k 10 300 python3 bench.py --config c3adv --second-role 0 --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/bench_c3adv_r1.log 2>&1 || exit $?
grep -o '"kernel_ms": [0-9.]*' $O/bench_c3adv_r1.log
for spec in "prod|" "nohr|--lib access-control-srv_amd/lib/variants/nohr.so" "w4|--lib access-control-srv_amd/lib/variants/w4.so" "w6|--lib access-control-srv_amd/lib/variants/w6.so"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python3 bench.py --config c3 $args --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --no-cpu-baseline > $O/ab_c3_$name.log 2>&1 || exit $?
  echo "c3 $name: $(grep -o '"kernel_ms": [0-9.]*' $O/ab_c3_$name.log)"
done
TAG=r04_d CONFIGS="c3 c3adv" bash tools/gpu_pmc_r04.sh || exit $?
echo done
