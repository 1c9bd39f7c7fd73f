#!/bin/bash
# Round 6: K1 with the first extension attribute staged in LDS (5 slots; 4 blocks per CU), at 5 and 4 waves/SIMD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_p}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c3_10m python3 -u tools/k1_ab.py c3 10000000 product k1s5 k1s5w4
step 300 ab_c3r1_1m python3 -u tools/k1_ab.py c3r1 1000000 product k1s5 k1s5w4
step 300 ab_c3adv_1m python3 -u tools/k1_ab.py c3adv 1000000 product k1s5 k1s5w4
step 300 ab_c5_1m python3 -u tools/k1_ab.py c5 1000000 product k1s5 k1s5w4
step 300 ab_c2_1m python3 -u tools/k1_ab.py c2 1000000 product k1s5 k1s5w4
step 300 ab_c3_131k python3 -u tools/k1_ab.py c3 131072 product k1s5 k1s5w4
echo done
