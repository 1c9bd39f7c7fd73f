#!/bin/bash
# Round 6: chunked host path + packed obligation logs — GPU parity, then the c3 bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_b}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -3 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 900 pytest_gpu python3 -u -m pytest tests/test_compact_gpu.py tests/test_gpu.py tests/test_wia_template.py tests/test_multi_device.py -m gpu -x -q --timeout 300 --timeout-method thread
step 600 bench_c3 python3 -u bench.py --steps 10 --warmup 3
echo done
