#!/bin/bash
# round 4: where c3adv's K1 time comes from (store x ACL x second role, 1M requests via the codec)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-r04_h}
mkdir -p $O
timeout -k 10 700 python3 -u tools/adv_ab.py 1000000 orders > $O/adv_orders.log 2>&1 || exit $?
grep "^{" $O/adv_orders.log
echo done
