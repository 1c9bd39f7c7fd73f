#!/bin/bash
# Round-6 K1 probes: same-process A/Bs (tools/k1_ab.py) of the product against cost-probe builds,
# then the GPU parity subset, then the clamped scalar-record build last.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_a}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log | cut -c1-900; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c3_10m python3 -u tools/k1_ab.py c3 10000000 product nohr hr2 tm2 w4
step 200 ab_c3r1_1m python3 -u tools/k1_ab.py c3r1 1000000 product hr2 tm2 w4
step 600 pytest_gpu python3 -u -m pytest tests/test_gpu.py tests/test_wia_template.py -x -q --timeout 300 --timeout-method thread
step 300 ab_scal_c3 python3 -u tools/k1_ab.py c3 10000000 product scal
step 300 ab_scal_c5 python3 -u tools/k1_ab.py c5 1000000 product scal
step 300 ab_scal_c4 python3 -u tools/k1_ab.py c4 1000000 product scal
echo done
