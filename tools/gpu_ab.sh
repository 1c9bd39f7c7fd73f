#!/bin/bash
# Same-call A/B of bench lines: each argument is "name|bench args"; every run has its own
# time limit and a crash / timeout stops the script before any further GPU use.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  echo "== $name ($(date +%T))"
  timeout -k 10 ${AB_LIMIT:-600} python bench.py $args > "$OUT/ab_$name.log" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/ab_$name.log"
  grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.]*\|"step_gpu_ms": [0-9.]*\|"request_classes": [0-9]*' "$OUT/ab_$name.log" | tr '\n' ' '; echo
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; tail -5 "$OUT/ab_$name.log"; exit $rc; fi
done
echo "== done"
