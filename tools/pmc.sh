#!/bin/bash
# PMC counter passes for the K1 eval kernel (one rocprofv3 run per counter group; no tracing
# domains combined with --pmc).  Output: gpurun_out/pmc/<group>/...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
CFG=${CFG:-c2}
EXTRA=${EXTRA:-}
KERNEL=${KERNEL:-is_allowed_kernel}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() {
  local name=$1; shift
  echo "== pmc $name ($(date +%T))"
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$KERNEL" -d $OUT/$name -o pmc \
    --output-format csv -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --e2e-requests 0 $EXTRA \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 2 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "STOP pmc rc=$rc"; exit $rc; fi
}
run g1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES
run g2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR
run g3 FETCH_SIZE
run g4 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
python3 tools/pmc_traffic.py $OUT "${KEY:-$CFG}" $OUT/traffic.json $KERNEL || true
if [ -n "$CALIB" ]; then
  echo "== calib ($(date +%T))"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gather16 -d $OUT/calib -o pmc --output-format csv \
    -- tools/calib_gather > $OUT/calib.log 2>&1
  echo "rc=$?"; tail -n 4 $OUT/calib.log
fi
echo "== pmc done"
