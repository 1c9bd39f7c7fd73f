#!/bin/bash
# Round 6: K2 template copy A/B + whatIsAllowed parity.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_g}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log | cut -c1-1200; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product rowcopy
step 300 ab_c4_131k python3 -u tools/k1_ab.py c4 131072 product rowcopy
step 600 pytest_wia python3 -u -m pytest tests/test_wia_template.py tests/test_gpu.py tests/test_compact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
echo done
