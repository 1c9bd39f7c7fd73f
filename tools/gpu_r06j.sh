#!/bin/bash
# Round 6: K2 cost probes (no copy / no work rules) and multi-row copy; K1 with 32-bit class-row offsets vs HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_j}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-1200; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product k2nocopy k2nowork k2copy2 k2copy4 prev
step 300 ab_c3_10m python3 -u tools/k1_ab.py c3 10000000 product prev
step 300 ab_c3r1_1m python3 -u tools/k1_ab.py c3r1 1000000 product prev
step 300 ab_c3adv_1m python3 -u tools/k1_ab.py c3adv 1000000 product prev
step 700 pytest_gpu python3 -u -m pytest tests/test_gpu.py tests/test_wia_template.py -m gpu -x -q --timeout 300 --timeout-method thread
echo done
