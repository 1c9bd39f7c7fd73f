"""The drop-in's gRPC request path (gpuCodec.grpcRequestJson): the JSON text
it splices from the protobuf Any members of a gRPC context equals, parsed, the request the
reference's AccessControlService builds (accessControlService.ts:62-65, 103-127, restated in
tests/js/grpc_json_run.js with the reference's own lodash functions) — including the :106 quirk
(array members become the unmarshalled `resources`) and empty / missing Any values (null)."""
import os
import shutil
import subprocess

import pytest

NODE = shutil.which("node")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON = os.path.join(ROOT, "access-control-srv_amd", "lib", "acs_mi355x.node")
pytestmark = pytest.mark.skipif(NODE is None or not os.path.exists(ADDON), reason="no node / addon")


def test_grpc_request_json_matches_reference_unmarshalling():
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "grpc_json_run.js"), "3000"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert '"checked":3000' in r.stdout


def test_micro_batcher_rejects_unserialisable_calls_alone():
    """a call whose request is not one JSON value (an Any value that only parses spliced
    into the batch — it would inject a request of its own and shift every later caller's record —
    a BigInt, a cycle, undefined) rejects by itself at the call, and nothing is queued."""
    import json
    from acs_mi355x import compiler, store
    from kat_utils import load_fixture
    from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS
    import tempfile
    m = store.populate(load_fixture("roleScopes.yml"))
    with tempfile.NamedTemporaryFile("wb", suffix=".json", delete=False) as f:
        f.write(compiler.snapshot_json(m))
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "microbatch_guard_run.js"), f.name,
                        json.dumps(FULL_URNS), json.dumps(DEFAULT_CAS)], capture_output=True, text=True, timeout=120)
    os.unlink(f.name)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["rejected"] == ["SyntaxError", "SyntaxError", "SyntaxError", "TypeError", "TypeError", "TypeError"], out
    assert out["queued"] == 0
