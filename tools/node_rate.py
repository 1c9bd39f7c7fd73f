#!/usr/bin/env python3
"""Node-side request rate of the drop-in, on a GPU box: writes a c3 store
(10k rules), N c3 requests (1-2 role associations, "$hrs" forest keys), the forests and the
product's decisions for those requests (acs_is_allowed on the host buffers) into a scratch
dir, then runs tests/js/node_rate.js, which measures requests/s from JS request objects —
gRPC messages through GpuAccessController.isAllowedGrpc (micro-batched), plain objects through
isAllowed (micro-batched) and isAllowedBatch — and checks every decision.  Prints one JSON line.
usage: python3 tools/node_rate.py [N] [threads] [batchMax]"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    batch_max = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    from acs_mi355x import compiler, native, store, synth
    from acs_mi355x.config import SERVICE_URNS, COMBINING_ALGORITHMS
    doc = synth.c3_store()
    m = store.populate(doc)
    cs = compiler.compile_store(m, SERVICE_URNS, COMBINING_ALGORITHMS)
    sb = synth.requests(cs, n, "c3", seed=0xACC1000, second_role=0.5)
    t = native.Tables(compiler.store_blob(cs), 0)
    dec = t.is_allowed(sb.batch)
    t.close()
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        with open(os.path.join(d, "store.json"), "wb") as f:
            f.write(compiler.snapshot_json(m))
        with open(os.path.join(d, "requests.json"), "wb") as f:
            f.write(sb.json_text())
        with open(os.path.join(d, "forests.tsv"), "w") as f:
            for k, v in sb.hrs_forests().items():
                f.write(k + "\t" + json.dumps(v, separators=(",", ":")) + "\n")
        dec["decision"].astype(np.uint8).tofile(os.path.join(d, "expect.bin"))
        with open(os.path.join(d, "meta.json"), "w") as f:
            json.dump({"urns": SERVICE_URNS, "cas": COMBINING_ALGORITHMS, "threads": threads,
                       "batchMax": batch_max}, f)
        r = subprocess.run(["node", "--max-old-space-size=8192", os.path.join(ROOT, "tests", "js", "node_rate.js"), d],
                           capture_output=True, text=True, timeout=900)
        sys.stderr.write(r.stderr[-3000:])
        if r.returncode != 0:
            raise SystemExit(f"node_rate.js failed rc={r.returncode}")
        out = json.loads(r.stdout.strip().splitlines()[-1])
        out["what"] = ("c3 requests (1-2 role associations, HR forests registered per (scope, role)) from JS objects "
                       "in Node through gpuCodec.GpuAccessController; gRPC = context members as protobuf Any with JSON "
                       "values (accessControlService.ts:62-65,103-127); every decision checked against the product's")
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
