#!/bin/bash
# Round 6: the encoder's wave-aligned class runs (holes) against the same order without them.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_h}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-1200; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 pad_c3adv_1m python3 -u tools/pad_ab.py c3adv 1000000
step 300 pad_c4_1m python3 -u tools/pad_ab.py c4 1000000
step 300 pad_c3r1_1m python3 -u tools/pad_ab.py c3r1 1000000
step 300 pad_c3_1m python3 -u tools/pad_ab.py c3 1000000
echo done
