#!/bin/bash
# Round 6: K2 with several staged batches of work rules per wave (test_templates_gpu_many_work_rules).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_z}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 600 pytest_wia python3 -u -m pytest tests/test_wia_template.py -m gpu -x -v --timeout 300 --timeout-method thread
echo done
