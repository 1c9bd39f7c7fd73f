cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpucodec_js.py tests/test_napi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_b.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_b.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench_c3.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench_c3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench_c4.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench_c4.log; exit $rc
