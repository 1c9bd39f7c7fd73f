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
