#!/bin/bash
# Round 6: K2 copy loops read row j's lane values with readlane instead of ds_bpermute; parity; A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_af}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 700 pytest_wia python3 -u -m pytest tests/test_wia_template.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product k2shfl
step 300 ab_c4_131k python3 -u tools/k1_ab.py c4 131072 product k2shfl
step 400 ab_c4_4m python3 -u tools/k1_ab.py c4 4000000 product k2shfl
echo done
