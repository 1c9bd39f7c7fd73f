cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  timeout -k 10 240 python tools/uniform_debug.py access-control-srv_amd/lib/variants/$v.so >> gpurun_out/uniform_debug.log 2>&1
  rc=$?
  echo "rc=$rc $v" >> gpurun_out/uniform_debug.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
