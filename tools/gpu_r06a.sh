cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06_a; mkdir -p $O
timeout -k 10 300 python3 -u tools/k1_ab.py c3 10000000 product nohr w4 s2w6 > $O/ab_c3_10m.log 2>&1 || exit 1
tail -1 $O/ab_c3_10m.log
timeout -k 10 200 python3 -u tools/k1_ab.py c3r1 1000000 product w4 > $O/ab_c3r1_1m.log 2>&1 || exit 1
tail -1 $O/ab_c3r1_1m.log
timeout -k 10 300 python3 -u tools/k1_ab.py c5 1000000 product w4 > $O/ab_c5_1m.log 2>&1 || exit 1
tail -1 $O/ab_c5_1m.log
timeout -k 10 200 python3 -u tools/k1_ab.py c4 1000000 product > $O/ab_c4_1m.log 2>&1 || exit 1
tail -1 $O/ab_c4_1m.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py tests/test_wia_template.py -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest_gpu.log
