#!/bin/bash
# Round 6: K2 work rules evaluated from rule lines staged in LDS; parity; c4 bench; c3 bench with the cold e2e leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_l}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -n 1 $O/$name.log | cut -c1-1500; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 600 pytest_wia python3 -u -m pytest tests/test_wia_template.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
step 400 ab_c4_1m python3 -u tools/k1_ab.py c4 1000000 product k2nostage k2nowork
step 300 ab_c4_131k python3 -u tools/k1_ab.py c4 131072 product k2nostage
step 400 ab_c4_4m python3 -u tools/k1_ab.py c4 4000000 product k2nostage
step 600 bench_c4 python3 -u bench.py --config c4 --steps 10 --warmup 3
step 600 bench_c3 python3 -u bench.py --steps 10 --warmup 3
echo done
