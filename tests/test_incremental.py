"""Incremental recompile: after store mutations through the
controller (updatePolicySet / updatePolicy / updateRule / remove* / Map edits,
accessController.ts:897-937), only the touched policy sets are recompiled
(compiler.IncrementalCompiler) and the image equals a fresh compile of the same Map
field for field, with interned ids compared as the strings they stand for.  Decisions
through the CPU build of the core are identical to a fresh controller's."""
import copy
import random

import numpy as np
import pytest

import host_core
import randgen
from diff_utils import controller_outcome, norm_rq, oracle_from_store, oracle_outcome, gpu_outcome
from oracle.acs_oracle import DEFAULT_CAS, FULL_URNS
from oracle.jsval import JSError, OracleUnsupported
from acs_mi355x import compiler, encoder, results, store as pstore, synth, layout as L
from acs_mi355x.controller import AccessController

ID_FIELDS = ("role", "se", "last_prop_value")
POOL_FIELDS = ("subj_off", "act_off", "res_off", "acl_roles_off")


def canonical(cs):
    """Tables with every interned id replaced by its string and pool offsets by contents."""
    d = cs.dictionary

    def s(i):
        v = d.string(int(i))
        return ("str", v) if isinstance(v, str) else repr(v)

    def node(n):
        rec = {k: int(n[k]) for k in L.NODE_DT.names if k not in ID_FIELDS + POOL_FIELDS + ("pad", "ec")}
        rec.update({k: s(n[k]) for k in ID_FIELDS})
        rec["ec"] = repr(cs.ec_values[int(n["ec"])])
        if n["nflags"] & L.NF_HAS_TARGET:
            rec["subj"] = [(s(p["id"]), s(p["value"])) for p in cs.pairs[n["subj_off"]:n["subj_off"] + n["subj_n"]]]
            rec["act"] = [(s(p["id"]), s(p["value"])) for p in cs.pairs[n["act_off"]:n["act_off"] + n["act_n"]]]
            rec["res"] = [(s(r["value"]), s(r["hash_sfx"]), int(r["kind"]),
                           repr(cs.rx_rows[int(r["row"])]) if r["kind"] & L.K_ENT_LOOSE else None)
                          for r in cs.rres[n["res_off"]:n["res_off"] + n["res_n"]]]
            rec["acl"] = [s(x) for x in cs.u32pool[n["acl_roles_off"]:n["acl_roles_off"] + n["acl_roles_n"]]]
        return rec

    spec = [[None if sp is None else sorted(repr(cs.rx_rows[r]) for r in sp) for sp in sec] for sec in cs.cand_spec]
    return ([node(n) for n in cs.sets], [node(n) for n in cs.pols], [node(n) for n in cs.rules], spec,
            s(cs.id_user))


def _ctl(urns):
    return AccessController({"urns": urns, "combiningAlgorithms": DEFAULT_CAS}, engine=host_core.Tables)


def _mutate(rng, ctl, pool_sets):
    """One random store mutation through the reference's surface; returns its name."""
    keys = list(ctl.policySets)
    op = rng.choice(["updateRule", "removeRule", "updatePolicy", "removePolicy", "updatePolicySet",
                     "removePolicySet", "map_set", "map_pop"])
    if not keys:
        op = "updatePolicySet"
    k = rng.choice(keys) if keys else None
    ps = ctl.policySets.get(k) if keys else None
    pols = list(ps["combinables"]) if ps else []
    donor = copy.deepcopy(rng.choice(pool_sets))
    donor_pols = [p for p in donor["combinables"].values() if isinstance(p, dict)]
    donor_rules = [r for p in donor_pols for r in p["combinables"].values() if isinstance(r, dict)]
    if op == "updateRule" and pols and donor_rules:
        pk = rng.choice(pols)
        if isinstance(ps["combinables"][pk], dict):
            r = copy.deepcopy(rng.choice(donor_rules))
            ctl.updateRule(k, pk, r)
    elif op == "removeRule" and pols:
        pk = rng.choice(pols)
        pol = ps["combinables"][pk]
        if isinstance(pol, dict) and pol["combinables"]:
            ctl.removeRule(k, pk, rng.choice(list(pol["combinables"])))
    elif op == "updatePolicy" and donor_pols:
        ctl.updatePolicy(k, copy.deepcopy(rng.choice(donor_pols)))
    elif op == "removePolicy" and pols:
        ctl.removePolicy(k, rng.choice(pols))
    elif op == "updatePolicySet":
        donor["id"] = f"new{rng.randrange(10**6)}" if rng.random() < 0.5 or not keys else k
        ctl.updatePolicySet(donor)
    elif op == "removePolicySet":
        ctl.removePolicySet(k)
    elif op == "map_set":
        ctl.policySets[k] = donor
    elif op == "map_pop":
        ctl.policySets.pop(k)
    return op


@pytest.mark.parametrize("seed", range(40))
def test_incremental_matches_fresh_compile(seed):
    urns, doc, reqs = randgen.rand_case(seed)
    try:
        base = pstore.populate(doc)
        compiler.compile_store(base, urns, DEFAULT_CAS)
    except Exception:
        pytest.skip("store outside the compiled subset")
    donors = list(pstore.populate(randgen.rand_case(seed + 1000)[1]).values()) or list(base.values())
    rng = random.Random(seed)
    ctl = _ctl(urns)
    ctl.policySets = base
    ctl.isAllowed_batch(reqs[:1])
    for step in range(6):
        op = _mutate(rng, ctl, donors)
        try:
            got = ctl.isAllowed_batch(reqs)
            fresh_cs = compiler.compile_store(ctl.policySets, urns, DEFAULT_CAS)
        except Exception as e:  # a mutation can make the store unsupported: both paths must agree
            with pytest.raises(type(e)):
                compiler.compile_store(ctl.policySets, urns, DEFAULT_CAS)
            return
        assert canonical(ctl._cs) == canonical(fresh_cs), (seed, step, op)
        fresh = _ctl(urns)
        fresh.policySets = pstore.populate({"policy_sets": []}) if not ctl.policySets else dict(ctl.policySets)
        want = fresh.isAllowed_batch(reqs)
        assert [repr(x) for x in got] == [repr(x) for x in want], (seed, step, op)
        o = oracle_from_store(urns, ctl.policySets)  # and the mutated Map through the oracle
        for i, req in enumerate(reqs):
            g = controller_outcome(got[i])
            if g[0] != "HOST":
                try:
                    assert g == oracle_outcome(o, req), (seed, step, op, i)
                except OracleUnsupported:
                    pass


def test_incremental_recompiles_only_touched_sets():
    doc = synth.c3_store()
    ctl = _ctl(FULL_URNS)
    ctl.policySets = pstore.populate(doc)
    sb_cs = compiler.compile_store(ctl.policySets, FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(sb_cs, 2_000, "c3")
    reqs = [sb.decode(i) for i in range(200)]
    ctl.isAllowed_batch(reqs)
    st = ctl._compiler.stats
    assert st["sets_compiled"] == 200 and st["sets_reused"] == 0
    keys = list(ctl.policySets)
    ps = ctl.policySets[keys[7]]
    pk = next(iter(ps["combinables"]))
    rule = copy.deepcopy(next(iter(ps["combinables"][pk]["combinables"].values())))
    rule["effect"] = "DENY" if rule.get("effect") == "PERMIT" else "PERMIT"
    ctl.updateRule(keys[7], pk, rule)
    got = ctl.isAllowed_batch(reqs)
    assert st["sets_compiled"] == 201 and st["sets_reused"] == 199
    ctl.removePolicySet(keys[3])
    ctl.isAllowed_batch(reqs)
    assert st["sets_compiled"] == 201 and st["sets_reused"] == 199 + 199
    assert canonical(ctl._cs) == canonical(compiler.compile_store(ctl.policySets, FULL_URNS, DEFAULT_CAS))
    fresh = _ctl(FULL_URNS)
    fresh.policySets = dict(ctl.policySets)
    assert [repr(x) for x in ctl.isAllowed_batch(reqs)] == [repr(x) for x in fresh.isAllowed_batch(reqs)]
    assert got  # the updated rule was evaluated


def _native_records(blob, reqs):
    """isAllowed records of ``reqs`` against a native-compiled image (its own codec, CPU core)."""
    import ctypes as C
    from acs_mi355x.codec import NativeCodec
    nb = NativeCodec(blob).encode(reqs)
    out = np.zeros(nb.n, L.DECISION_DT)
    assert host_core.lib().acs_host_is_allowed(blob, len(blob), C.byref(nb.struct), out.ctypes.data) == 0
    return out.view(np.uint64)


@pytest.mark.parametrize("seed", range(40))
def test_native_builder_matches_fresh_compile(seed):
    """acs_store_builder (the Node drop-in's incremental compile): its first image is the
    full compiler's byte for byte; after each mutation it recompiles at most the touched set
    and decides every request exactly as a fresh full compile of the mutated Map."""
    urns, doc, reqs = randgen.rand_case(seed)
    try:
        base = pstore.populate(doc)
        first = compiler.native_store_blob(base, urns, DEFAULT_CAS)
    except Exception:
        pytest.skip("store outside the compiled subset")
    b = compiler.NativeStoreBuilder(urns, DEFAULT_CAS)
    assert b.compile(base) == first and b.recompiled == len(base)
    donors = list(pstore.populate(randgen.rand_case(seed + 1000)[1]).values()) or list(base.values())
    rng = random.Random(seed)
    ctl = _ctl(urns)
    ctl.policySets = base
    for step in range(8):
        op = _mutate(rng, ctl, donors)
        try:
            fresh = compiler.native_store_blob(ctl.policySets, urns, DEFAULT_CAS)
        except compiler.Unsupported:
            with pytest.raises(compiler.Unsupported):
                b.compile(ctl.policySets)
            return
        blob = b.compile(ctl.policySets)
        assert b.recompiled <= 1, (seed, step, op)
        assert np.array_equal(_native_records(blob, reqs), _native_records(fresh, reqs)), (seed, step, op)
    b.close()


@pytest.mark.parametrize("seed", range(0, 40, 2))
def test_native_builder_staged_sets(seed):
    """acs_store_builder_stage (the Node drop-in stages one set's text at a time): staging every
    set gives the text compile's image byte for byte; restaging an unchanged set reuses its
    fragment (nothing recompiled); a mutated set staged beside previous-set indices decides like
    a fresh compile; a staging that does not compile leaves the builder as it was."""
    urns, doc, reqs = randgen.rand_case(seed)
    try:
        base = pstore.populate(doc)
        first = compiler.native_store_blob(base, urns, DEFAULT_CAS)
    except Exception:
        pytest.skip("store outside the compiled subset")
    texts = compiler.set_texts(base)
    b = compiler.NativeStoreBuilder(urns, DEFAULT_CAS)
    assert b.compile_items([("staged", b.stage(t)) for t in texts]) == first and b.recompiled == len(texts)
    assert b.compile_items([("staged", b.stage(t)) for t in texts]) == first and b.recompiled == 0
    rng = random.Random(seed)
    donors = list(pstore.populate(randgen.rand_case(seed + 1000)[1]).values()) or list(base.values())
    ctl = _ctl(urns)
    ctl.policySets = base
    for step in range(4):
        _mutate(rng, ctl, donors)
        try:
            fresh = compiler.native_store_blob(ctl.policySets, urns, DEFAULT_CAS)
        except compiler.Unsupported:
            return
        new_texts = compiler.set_texts(ctl.policySets)
        old = {t: k for k, t in enumerate(texts)}
        items = []
        for t in new_texts:  # unchanged texts by index (once each), the rest staged
            j = old.pop(t, None)
            items.append(("prev", j) if j is not None else ("staged", b.stage(t)))
        blob = b.compile_items(items)
        assert np.array_equal(_native_records(blob, reqs), _native_records(fresh, reqs)), (seed, step)
        texts = new_texts
    with pytest.raises(compiler.Unsupported):
        b.stage(b'{"combinables": 7}')
    assert b.compile_items([("prev", k) for k in range(len(texts))]) == blob and b.recompiled == 0
    b.close()


def test_fresh_compile_is_byte_stable():
    """compile_store (one IncrementalCompiler pass) gives the same blob twice."""
    m = pstore.populate(synth.c2_store())
    a = compiler.store_blob(compiler.compile_store(m, FULL_URNS, DEFAULT_CAS))
    b = compiler.store_blob(compiler.compile_store(m, FULL_URNS, DEFAULT_CAS))
    assert a == b
    ic = compiler.IncrementalCompiler(FULL_URNS, DEFAULT_CAS)
    ic.compile(m)
    assert compiler.store_blob(ic.compile(m, dirty=set())) == a  # all fragments reused
    assert np.array_equal(np.frombuffer(a[:64], np.uint32)[2:5], [100, 200, 1000])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_incremental_gpu(seed):
    """The same mutation sequences through the default (GPU) engine: every recompiled image
    decides like a fresh controller's, and whatIsAllowed agrees too."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    urns, doc, reqs = randgen.rand_case(seed)
    try:
        base = pstore.populate(doc)
        compiler.compile_store(base, urns, DEFAULT_CAS)
    except Exception:
        pytest.skip("store outside the compiled subset")
    donors = list(pstore.populate(randgen.rand_case(seed + 1000)[1]).values()) or list(base.values())
    rng = random.Random(seed)
    opts = {"urns": urns, "combiningAlgorithms": DEFAULT_CAS}
    ctl = AccessController(opts)
    ctl.policySets = base
    ctl.isAllowed_batch(reqs[:1])
    compared = 0
    for step in range(5):
        op = _mutate(rng, ctl, donors)
        try:
            got = ctl.isAllowed_batch(reqs)
            got_w = ctl.whatIsAllowed_batch(reqs)
        except Exception as e:  # an unsupported store: a fresh compile refuses it the same way
            with pytest.raises(type(e)):
                compiler.compile_store(ctl.policySets, urns, DEFAULT_CAS)
            return
        fresh = AccessController(opts)
        fresh.policySets = dict(ctl.policySets)
        assert [repr(x) for x in got] == [repr(x) for x in fresh.isAllowed_batch(reqs)], (seed, step, op)
        assert [repr(x) for x in got_w] == [repr(x) for x in fresh.whatIsAllowed_batch(reqs)], (seed, step, op)
        fresh.close()
        # the mutated Map, loaded into the oracle, decides every request the same way
        o = oracle_from_store(urns, ctl.policySets)
        for i, req in enumerate(reqs):
            g = controller_outcome(got[i])
            if g[0] == "HOST":
                continue
            try:
                assert g == oracle_outcome(o, req), (seed, step, op, i)
            except OracleUnsupported:
                continue
            try:
                want = ("OK", norm_rq(o.what_is_allowed(req)))
            except JSError as e:
                want = ("ERR", e.kind)
            except OracleUnsupported:
                continue
            w = got_w[i]
            if isinstance(w, results.HostPathRequired):
                continue
            gw = ("ERR", w.kind) if isinstance(w, results.EvaluationError) else ("OK", norm_rq(w))
            assert gw == want, (seed, step, op, i)
            compared += 1
    ctl.close()
    assert compared > 0 or not reqs


@pytest.mark.gpu
def test_delta_upload_gpu():
    """acs_compile_update (the delta upload): after an updateRule that keeps
    the store's shape, the new handle's image is the previous one with only the changed 64-KB
    blocks uploaded, and it decides exactly like a fresh handle of the new image; a change of
    shape (a rule added) uploads the whole image, with the same guarantee."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x import native, synth
    from oracle.acs_oracle import FULL_URNS
    base = pstore.populate(synth.c3_store())
    ic = compiler.IncrementalCompiler(FULL_URNS, DEFAULT_CAS)
    cs = ic.compile(base)
    t = native.Tables(compiler.store_blob(cs), 0)
    assert t.upload_bytes >= len(compiler.store_blob(cs)) // 2
    sb = synth.requests(cs, 20_000, "c3", seed=3, second_role=0.5)
    texts = sb.json_text()
    import json
    reqs = json.loads(texts)
    key = list(base)[150]
    ps = base[key]
    pkey = list(ps["combinables"])[2]
    rules = ps["combinables"][pkey]["combinables"]
    rkey = list(rules)[4]
    r = dict(rules[rkey])
    r["effect"] = "DENY" if r.get("effect") == "PERMIT" else "PERMIT"
    rules[rkey] = r
    cs2 = ic.compile(base, dirty={key})
    blob2 = compiler.store_blob(cs2)
    t2 = t.updated(blob2)
    assert 0 < t2.upload_bytes <= 1 << 20, t2.upload_bytes
    fresh = native.Tables(blob2, 0)
    b2 = encoder.Encoder(cs2).encode(reqs)
    want = fresh.is_allowed(b2)
    assert np.array_equal(t2.is_allowed(b2).view(np.uint64), want.view(np.uint64))
    assert np.array_equal(t.is_allowed(encoder.Encoder(cs).encode(reqs)).view(np.uint64),
                          native.Tables(compiler.store_blob(cs), 0).is_allowed(
                              encoder.Encoder(cs).encode(reqs)).view(np.uint64))  # the old handle still works
    # a new rule: another shape, a full upload
    nr = dict(r)
    nr["id"] = "added-rule"
    rules["added-rule"] = nr
    cs3 = ic.compile(base, dirty={key})
    blob3 = compiler.store_blob(cs3)
    t3 = t2.updated(blob3)
    assert t3.upload_bytes >= len(blob3) // 2
    b3 = encoder.Encoder(cs3).encode(reqs)
    assert np.array_equal(t3.is_allowed(b3).view(np.uint64), native.Tables(blob3, 0).is_allowed(b3).view(np.uint64))
    for x in (t, t2, t3, fresh):
        x.close()
