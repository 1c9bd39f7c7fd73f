#!/bin/bash
# Round 6: K2's template copy as one flat run of chunks, unrolled (ACS_K2_FLAT_COPY) vs per row; PMC c2 / c5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_u}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product k2flat
step 300 ab_c4_131k python3 -u tools/k1_ab.py c4 131072 product k2flat
step 400 ab_c4_4m python3 -u tools/k1_ab.py c4 4000000 product k2flat
bash tools/gpu_r06t.sh
