#!/bin/bash
# Round 6: one 8-B store per obligation log entry; parity; A/B; c4 PMC.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_ac}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 800 pytest_wia python3 -u -m pytest tests/test_wia_template.py tests/test_gpu.py tests/test_multi_device.py tests/test_rule_shard_lib.py -m gpu -x -q --timeout 300 --timeout-method thread
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product obl2st
step 400 ab_c4_4m python3 -u tools/k1_ab.py c4 4000000 product obl2st
step 300 ab_c3_10m python3 -u tools/k1_ab.py c3 10000000 product obl2st
echo done
