#!/bin/bash
# Round 6: the obligation-only pass's range count (16 / 32 / 64) on c4's overflowed logs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_y}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 400 obl_c4_1m python3 -u tools/obl_ab.py 1000000 16 32 64 8
echo done
