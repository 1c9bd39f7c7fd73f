#!/bin/bash
# Round 6: sanity on the final rebuilt libraries: smoke, core GPU parity tests, the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_ae}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 300 smoke python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 700 pytest_core python3 -u -m pytest tests/test_gpu.py tests/test_wia_template.py tests/test_compact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
step 600 bench python3 -u bench.py
echo done
