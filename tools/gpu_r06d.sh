#!/bin/bash
# Round 6: node-record round-trip probe; multi-device updates; host whatIsAllowed D2H.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_d}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log | cut -c1-1200; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c3_10m python3 -u tools/k1_ab.py c3 10000000 product nodig nr2
step 200 ab_c3r1_1m python3 -u tools/k1_ab.py c3r1 1000000 product nodig nr2
step 300 ab_c3adv_1m python3 -u tools/k1_ab.py c3adv 1000000 product nodig
step 300 ab_c5_1m python3 -u tools/k1_ab.py c5 1000000 product nodig
step 600 pytest_md python3 -u -m pytest tests/test_multi_device.py tests/test_rule_shard_lib.py tests/test_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread
step 300 wia_host python3 -u tools/wia_host_rate.py 1000000
echo done
