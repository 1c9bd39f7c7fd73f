#!/bin/bash
# Round 6: c3adv with and without dropping its mostly-hole class runs (same call), then the PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_r}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c3adv_1m python3 -u tools/k1_ab.py c3adv 1000000 product prevan
step 300 ab_c3adv_1m_b python3 -u tools/k1_ab.py c3adv 1000000 prevan product
TAG=r06_final_c PART=c timeout -k 10 900 bash tools/gpu_final6.sh
