#!/bin/bash
# Round 6: K2 store-order fence at workgroup scope (was agent: an L2 writeback per wave); probes; WIA parity; c4 PMC.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_k}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product k2agent k2ps k2nocopy k2nowork k2bare
step 300 ab_c4_131k python3 -u tools/k1_ab.py c4 131072 product k2agent
step 700 pytest_wia python3 -u -m pytest tests/test_wia_template.py tests/test_gpu.py tests/test_compact_gpu.py tests/test_multi_device.py -m gpu -x -q --timeout 300 --timeout-method thread
step 600 bench_c4 python3 -u bench.py --config c4 --steps 10 --warmup 3
PMC_OUT=$O/pmc_c4 CFG=c4 KERNEL=what_is_allowed_kernel timeout -k 10 900 bash tools/pmc.sh > $O/pmc_c4.log 2>&1; echo "pmc rc=$?"; tail -n 3 $O/pmc_c4.log
echo done
