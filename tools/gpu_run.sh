#!/bin/bash
# One GPU session: each step under its own time limit, stopping at the first failure.
# usage: TAG=<name> tools/gpu_run.sh '<step>' ['<step>' ...]   (outputs under gpurun_out/$TAG)
#   a step is "<seconds> <log name> <command...>", e.g. "600 pytest_gpu python3 -u -m pytest ..."
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${TAG:-run}
mkdir -p $O
for step in "$@"; do
  read -r secs name cmd <<< "$step"
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  tail -4 "$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; exit $rc; fi
done
echo done
