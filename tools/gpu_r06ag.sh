#!/bin/bash
# Round 6: c5 first batch after one updateRule vs a warm batch, from Node (VERDICT #6 measurement).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_ag}; mkdir -p $O
( while sleep 50; do echo "[tick] $(date +%T)" >> $O/progress.log; done ) & TICK=$!
timeout -k 10 1000 python3 -u -m pytest tests/test_gpucodec_js.py -k c5_update_latency -m gpu -x -v -s --timeout 1000 --timeout-method thread > $O/c5_latency.log 2>&1
rc=$?; kill $TICK; grep -E "c5 batch|passed|failed|Error" $O/c5_latency.log | cut -c1-600; exit $rc
