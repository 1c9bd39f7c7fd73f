#!/bin/bash
# Round 6: K1 prologue probes on small batches (c3 131,072 / 32,768 / 4,096 requests).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_aa}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 ab_c3_131k python3 -u tools/k1_ab.py c3 131072 product k1nowalk k1norows
step 300 ab_c3_32k python3 -u tools/k1_ab.py c3 32768 product k1nowalk k1norows
step 300 ab_c3_4k python3 -u tools/k1_ab.py c3 4096 product k1nowalk k1norows
echo done
