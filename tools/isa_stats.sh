#!/bin/bash
# Register use / occupancy and an instruction-class census of the eval kernels
# (hipcc --save-temps into /tmp/isa).  usage: tools/isa_stats.sh [extra hipcc flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p /tmp/isa
cd /tmp/isa
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I "$ROOT/access-control-srv_amd/csrc" \
  -I "$ROOT/include" --save-temps -Rpass-analysis=kernel-resource-usage "$@" \
  "$ROOT/access-control-srv_amd/csrc/acs_kernels.hip" -o /tmp/isa/t.so 2> remarks.txt
S=acs_kernels-hip-amdgcn-amd-amdhsa-gfx950.s
for k in 17is_allowed_kernel 22what_is_allowed_kernel; do
  echo "== $k"
  grep -A9 "N_1$k" remarks.txt | grep -E "SGPRs:|VGPRs:|Occupancy|Spill" | sed 's/.*remark: [^ ]* *//'
  awk "/^_ZN12_GLOBAL__N_1${k}/,/s_endpgm/" $S > k.s
  printf "lines %s" "$(wc -l < k.s)"
  for p in s_load global_load ds_read v_readlane v_writelane v_readfirstlane s_cbranch; do
    printf " | %s %s" "$p" "$(grep -c "$p" k.s || true)"
  done
  echo
done
