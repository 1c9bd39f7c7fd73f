#!/bin/bash
# Round 6: sharded pipeline + Node drop-in tests, Node rate / latency, K1 at small batch sizes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_f}; mkdir -p $O
step() { local secs=$1 name=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log | cut -c1-1200; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }; }
step 600 pytest_shard_js python3 -u -m pytest tests/test_rule_shard_lib.py tests/test_gpucodec_js.py tests/test_napi.py tests/test_grpc_json.py -m gpu -x -q --timeout 300 --timeout-method thread
step 300 ab_c3adv_1m python3 -u tools/k1_ab.py c3adv 1000000 product nodig
step 400 node_rate python3 -u tools/node_rate.py 262144 16 65536
for n in 4096 32768 65536 131072 1000000; do
  step 200 k1_c3_$n python3 -u tools/k1_ab.py c3 $n product
done
echo done
