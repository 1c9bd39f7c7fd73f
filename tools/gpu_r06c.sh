#!/bin/bash
# Round 6: fused rule target match A/B, full GPU suite, c3 bench line (chunked PCIe leg).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_c}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log | cut -c1-1200; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c3_10m python3 -u tools/k1_ab.py c3 10000000 product unfused tm2 hr2
step 200 ab_c3r1_1m python3 -u tools/k1_ab.py c3r1 1000000 product unfused
step 300 ab_c5_1m python3 -u tools/k1_ab.py c5 1000000 product unfused
step 300 ab_c3adv_1m python3 -u tools/k1_ab.py c3adv 1000000 product unfused
step 1000 pytest_gpu python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 600 bench_c3 python3 -u bench.py --steps 10 --warmup 3
echo done
