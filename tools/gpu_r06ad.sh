#!/bin/bash
# Round 6: K1 decision records as non-temporal 8-B stores (ACS_K1_NT_OUT) A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_ad}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c3_10m python3 -u tools/k1_ab.py c3 10000000 product k1ntout
step 300 ab_c3r1_1m python3 -u tools/k1_ab.py c3r1 1000000 product k1ntout
step 300 ab_c3adv_1m python3 -u tools/k1_ab.py c3adv 1000000 product k1ntout
step 300 ab_c5_1m python3 -u tools/k1_ab.py c5 1000000 product k1ntout
echo done
