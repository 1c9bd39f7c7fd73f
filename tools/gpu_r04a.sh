#!/bin/bash
# round-4 baseline: the round-3 final build on c3 (1 role) and c3r2 (50 % second role), rocprof kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/r04_a
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_a/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --parity-fraction 0.002 > gpurun_out/r04_a/bench_c3.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --config c3r2 --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --parity-fraction 0.002 > gpurun_out/r04_a/bench_c3r2.log 2>&1 || exit $?
echo done
