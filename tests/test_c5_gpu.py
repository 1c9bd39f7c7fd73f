"""c5 (configs[4]): the full 1M-rule store (1,000 sets x 10 policies x 100 rules) on the GPU.

* a request batch against the whole store: a 1 % C++-oracle sample (1,000 of 100,000; the
  reference's algorithm over the decoded JSON requests) must match every record;
* rule sharding at c5 scale: the store cut into 8 runs of whole policy sets (one per
  rank of the rule-sharded bench), each evaluated on this GPU, the 64-bit keys reduced
  with MAX (what the RCCL all-reduce does across ranks) — bit-identical to the
  unsharded records, which carries "last applicable set wins"
  (accessController.ts:293-295) across shard boundaries.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

from acs_mi355x import compiler, native, shard, store, synth, layout as L  # noqa: E402
from acs_mi355x.device import DeviceBatch, is_allowed_device, decisions_from_tensor  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402
from test_gpu import coracle_check  # noqa: E402

N = 100_000


@pytest.fixture(scope="module")
def c5():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.load()
    doc = synth.c5_store()
    full = store.populate(doc)
    cs = compiler.compile_store(full, FULL_URNS, DEFAULT_CAS)
    assert cs.n_rules == 1_000_000
    sb = synth.requests(cs, N, "c3", seed=0xACC1005)
    t = native.Tables(compiler.store_blob(cs), 0)
    dec = decisions_from_tensor(is_allowed_device(t, DeviceBatch(sb.batch, 0)))
    t.close()
    return doc, full, cs, sb, dec


def test_c5_oracle_sample_gpu(c5):
    doc, full, cs, sb, dec = c5
    codes = np.bincount(dec["decision"], minlength=7)
    assert codes[L.DEC_PERMIT] > 0 and codes[L.DEC_DENY] > 0
    # 1,000 requests (1 % of the batch): the C++ oracle decides ~60 c5 requests/s on 16 threads
    idx = np.random.default_rng(55).choice(N, size=1000, replace=False)
    assert coracle_check(doc, cs, sb, dec, idx, chunk=250) == 1000


def test_c5_rule_shard_8_gpu(c5):
    doc, full, cs, sb, want = c5
    keys = []
    parts = shard.partition(full, 8)
    assert len(parts) == 8
    for a, b in parts:
        c = compiler.compile_store(shard.slice_store(full, a, b), FULL_URNS, DEFAULT_CAS)
        t = native.Tables(compiler.store_blob(c), 0)
        d = is_allowed_device(t, DeviceBatch(synth.requests(c, N, "c3", seed=0xACC1005).batch, 0))
        keys.append(shard.keys_device(t, d, shard.base(full, a)))
        torch.cuda.synchronize()
        t.close()
    red = torch.stack(keys).max(dim=0).values
    got = decisions_from_tensor(shard.decode_device(native.load(), red))
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
