#!/bin/bash
# round 4: GPU suite on the composed-rows / encoder-order build, then the c3 (1-2 roles) and
# c3r1 bench lines, K1 kernel trace of the c3 line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_b}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --parity-fraction 0.005 > $O/bench_c3.log 2>&1 || exit $?
grep '^{' $O/bench_c3.log | cut -c1-400
timeout -k 10 300 python3 bench.py --config c3r1 --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --parity-fraction 0.002 > $O/bench_c3r1.log 2>&1 || exit $?
grep '^{' $O/bench_c3r1.log | cut -c1-300
timeout -k 10 300 python3 bench.py --config c3adv --steps 20 --warmup 5 --e2e-requests 0 --no-pcie --parity-fraction 0.01 > $O/bench_c3adv.log 2>&1 || exit $?
grep '^{' $O/bench_c3adv.log | cut -c1-300
timeout -k 10 600 python3 tools/node_rate.py 262144 > $O/node_rate.log 2>&1 || exit $?
tail -1 $O/node_rate.log | cut -c1-600
echo done
