#!/bin/bash
# Round 6: obligation-only pass through the work rules of templated requests, reusing K2's templates
# of the same batch; parity; c4 step A/B against the previous build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_x}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 800 pytest_wia python3 -u -m pytest tests/test_wia_template.py tests/test_gpu.py tests/test_multi_device.py tests/test_rule_shard_lib.py tests/test_incremental.py tests/test_compact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
step 400 bench_c4 python3 -u bench.py --config c4 --steps 20 --warmup 5
step 400 bench_c4_prev python3 -u bench.py --config c4 --steps 20 --warmup 5 --lib access-control-srv_amd/lib/variants/prevobl.so
step 400 bench_c4_b python3 -u bench.py --config c4 --steps 20 --warmup 5
step 400 bench_c4_prev_b python3 -u bench.py --config c4 --steps 20 --warmup 5 --lib access-control-srv_amd/lib/variants/prevobl.so
echo done
