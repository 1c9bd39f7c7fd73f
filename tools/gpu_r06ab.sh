#!/bin/bash
# Round 6: K2 work rules first, then the template into the chunks they did not write (every chunk
# written once); parity; A/B against copy-first; c4 PMC.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_ab}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 800 pytest_wia python3 -u -m pytest tests/test_wia_template.py tests/test_gpu.py tests/test_multi_device.py tests/test_rule_shard_lib.py tests/test_compact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product k2copyfirst
step 300 ab_c4_131k python3 -u tools/k1_ab.py c4 131072 product k2copyfirst
step 400 ab_c4_4m python3 -u tools/k1_ab.py c4 4000000 product k2copyfirst
PMC_OUT=$O/pmc_c4 CFG=c4 KERNEL=what_is_allowed_kernel KEY=c4/n1000000/w1/requests timeout -k 10 600 bash tools/pmc.sh > $O/pmc_c4.log 2>&1 || { echo "STOP pmc"; exit 1; }
tail -n 2 $O/pmc_c4.log
echo done
