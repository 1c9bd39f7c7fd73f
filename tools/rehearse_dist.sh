#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: 2 ranks over gloo, both on cuda:0 (bench.py
# ACS_BENCH_REHEARSAL=1).  Exercises request sharding and rule sharding end to end.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export ACS_BENCH_REHEARSAL=1
run() {
  local name=$1; shift
  echo "== $name ($(date +%T))"
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 500)) bench.py --gpus 2 "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "rc=$rc"; grep '^{' gpurun_out/$name.log | cut -c1-400 || true
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$name.log; exit $rc; fi
}
run rehearse_requests --requests 200000 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie
run rehearse_rules --rule-shard --requests 200000 --steps 5 --warmup 1 --no-cpu-baseline
run rehearse_rules_c3 --config c3 --rule-shard --requests 200000 --steps 3 --warmup 1 --no-cpu-baseline
