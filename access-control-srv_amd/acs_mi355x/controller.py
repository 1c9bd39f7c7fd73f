"""``AccessController`` — the reference's PDP surface over the MI355X evaluator.

Mirrors ``class AccessController`` of src/core/accessController.ts so a caller of
the reference finds the same names, argument meaning and error behaviour:

    constructor(opts)                       accessController.ts:39-77  (urns, combiningAlgorithms)
    policySets (public, mutable Map)        accessController.ts:32; assigned at
                                            accessControlService.ts:50, resourceManager.ts:274,305,...
    clearPolicies()                         accessController.ts:79-81
    isAllowed(request) -> Response          accessController.ts:88-324
    whatIsAllowed(request) -> ReverseQuery  accessController.ts:326-427
    updatePolicySet / removePolicySet /
    updatePolicy / removePolicy /
    updateRule / removeRule                 accessController.ts:897-937

Evaluation goes through the C ABI only (``native.Tables`` on a GPU).  The
policy store is compiled into an immutable table image on first use after a
mutation; ``*_batch`` methods evaluate many requests in one launch (the
micro-batch of SURVEY §8(b)).  Requests the GPU path reports to the host
(subject token I/O, JS ``condition``, non-exact RegExp) go to ``host_evaluator(op, request)`` when one is given, else raise
``HostPathRequired``.  whatIsAllowed requests with more than OBL_MAX maskedProperty
pushes stay on the GPU: an obligation-only pass re-runs them with a longer log
(``Tables.resolve_overflow``).  A request the reference would reject (its promise
throws) raises ``EvaluationError`` with the JS error kind.
"""
from __future__ import annotations

from typing import Callable, Iterable

from . import compiler, encoder, results
from .jsops import MISSING, Unsupported
from .results import EvaluationError, HostPathRequired

_CA_METHODS = ("denyOverrides", "permitOverrides", "firstApplicable")


class InvalidCombiningAlgorithm(Exception):
    """errors.InvalidCombiningAlgorithm of the reference (accessController.ts:57,837)."""


_ALL = object()  # invalidate(): every policy set may have changed


class _Store(dict):
    """The ``policySets`` Map: a dict (insertion order == JS Map order) that tells its
    controller which sets change.  Nested ``combinables`` maps are plain dicts; edits
    made through the controller's update*/remove* methods are tracked per set, direct
    nested edits need ``invalidate(setID)`` (or ``invalidate()`` for all sets)."""

    def __init__(self, owner, *a):
        super().__init__(*a)
        self._owner = owner

    def _touch(self, key=_ALL):
        self._owner.invalidate(key)

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        self._touch(k)

    def __delitem__(self, k):
        super().__delitem__(k)
        self._touch(k)

    def pop(self, *a):
        r = super().pop(*a)
        self._touch(a[0])
        return r

    def clear(self):
        super().clear()
        self._touch()

    def update(self, *a, **kw):
        super().update(*a, **kw)
        self._touch()

    def popitem(self):
        k, v = super().popitem()
        self._touch(k)
        return k, v

    def setdefault(self, k, default=None):
        if k in self:
            return self[k]
        self[k] = default  # __setitem__ tracks it
        return default

    def __ior__(self, other):
        super().__ior__(other)
        self._touch()
        return self

    # JS Map spellings used by callers of the reference
    def set(self, k, v):
        self[k] = v
        return self

    def delete(self, k):
        if k in self:
            del self[k]
            return True
        return False


def _key(v):
    """Map keys are ids as given: None is JS null, jsops.MISSING is undefined (distinct keys)."""
    return v


class AccessController:
    def __init__(self, opts: dict, device: int = 0, engine: Callable | None = None,
                 host_evaluator: Callable | None = None):
        """``opts`` = the service's ``policies.options`` (cfg/config.json:269-308):
        ``{"urns": {...}, "combiningAlgorithms": [{"urn", "method"}, ...]}``.
        ``engine(blob) -> tables`` overrides the default GPU tables (``native.Tables``)."""
        cas = list((opts or {}).get("combiningAlgorithms") or [])
        for ca in cas:  # accessController.ts:51-62
            if ca.get("method") not in _CA_METHODS:
                raise InvalidCombiningAlgorithm(ca.get("urn"))
        self.combiningAlgorithms = cas
        self.urns = dict((opts or {}).get("urns") or {})
        self.device = device
        self.host_evaluator = host_evaluator
        self._engine = engine
        self._compiler = None  # compiler.IncrementalCompiler, created on first compile
        self._dirty, self._all_dirty = set(), True
        self._policy_sets = _Store(self)
        self._cs = None
        self._tables = None
        self._encoder = None
        self.stats = {"compiles": 0, "requests": 0, "host": 0}

    # ------------------------------------------------------------------ store
    @property
    def policySets(self):
        return self._policy_sets

    @policySets.setter
    def policySets(self, m):
        """``accessController.policySets = new Map(...)`` (accessControlService.ts:50)."""
        self._policy_sets = _Store(self, m.items() if hasattr(m, "items") else m)
        self.invalidate()

    def invalidate(self, policySetID=_ALL):
        """Mark the compiled image stale; the next evaluation recompiles the sets marked
        here (``policySetID``), or every set (no argument), and reuses the others'
        compiled fragments (compiler.IncrementalCompiler)."""
        if policySetID is _ALL:
            self._all_dirty = True
        else:
            self._dirty.add(_key(policySetID))
        self._cs = None

    def clearPolicies(self):
        self._policy_sets.clear()

    def updatePolicySet(self, policySet: dict):
        self._policy_sets[_key(policySet.get("id", MISSING))] = policySet

    def removePolicySet(self, policySetID):
        self._policy_sets.pop(_key(policySetID), None)

    def updatePolicy(self, policySetID, policy: dict):
        ps = self._policy_sets.get(_key(policySetID))
        if ps is not None:  # _.isNil guard, accessController.ts:907-909
            ps["combinables"][_key(policy.get("id", MISSING))] = policy
            self.invalidate(policySetID)

    def removePolicy(self, policySetID, policyID):
        ps = self._policy_sets.get(_key(policySetID))
        if ps is not None:
            ps["combinables"].pop(_key(policyID), None)
            self.invalidate(policySetID)

    def updateRule(self, policySetID, policyID, rule: dict):
        ps = self._policy_sets.get(_key(policySetID))
        if ps is not None:
            pol = ps["combinables"].get(_key(policyID))
            if pol is not None:
                pol["combinables"][_key(rule.get("id", MISSING))] = rule
                self.invalidate(policySetID)

    def removeRule(self, policySetID, policyID, ruleID):
        ps = self._policy_sets.get(_key(policySetID))
        if ps is not None:
            pol = ps["combinables"].get(_key(policyID))
            if pol is not None:
                pol["combinables"].pop(_key(ruleID), None)
                self.invalidate(policySetID)

    # ------------------------------------------------------------------ tables
    def _fresh_compiler(self):
        self._compiler = compiler.IncrementalCompiler(self.urns, self.combiningAlgorithms)
        self.stats["compiler_resets"] = self.stats.get("compiler_resets", 0) + 1

    def _ensure(self):
        if self._cs is not None:
            return
        # A fresh compiler (empty dictionary / regex rows) when every set is recompiled anyway
        # (new Map, clearPolicies, invalidate()), or when the append-only tables have grown
        # past twice their live size through updates; never an unbounded dictionary.
        if self._compiler is None or self._all_dirty or self._compiler.stale():
            self._fresh_compiler()
            self._all_dirty = True
        try:
            cs = self._compiler.compile(self._policy_sets, None if self._all_dirty else self._dirty)
        except Unsupported:
            if self._all_dirty:
                raise
            # a capacity cap (65,535 regex rows, 255 evaluation_cacheable values) hit by stale
            # entries: recompile everything from scratch; a live-store overflow raises again
            self._fresh_compiler()
            cs = self._compiler.compile(self._policy_sets, None)
        self._dirty, self._all_dirty = set(), False
        blob = compiler.store_blob(cs)
        prev, self._tables = self._tables, None
        if self._engine is not None:
            if prev is not None:
                prev.close()
            self._tables = self._engine(blob)
        else:
            from . import native
            # the previous image with only its changed blocks uploaded (acs_compile_update); if
            # that fails (a device allocation, an image the update refuses), a full upload; the
            # previous handle is closed only once a new one exists, and kept if neither succeeds
            new = None
            try:
                if prev is not None:
                    try:
                        new = prev.updated(blob)
                    except Exception:
                        new = None
                if new is None:
                    new = native.Tables(blob, self.device)
            except Exception:
                self._tables = prev  # the old image still serves the old store until a retry
                raise
            self._tables = new
            if prev is not None:
                prev.close()
            self.stats["upload_bytes"] = self._tables.upload_bytes
        self._cs = cs
        self._encoder = encoder.Encoder(cs)
        self.stats["compiles"] += 1

    def close(self):
        if self._tables is not None:
            self._tables.close()
            self._tables = None
        self._cs = None

    # ------------------------------------------------------------------ decisions
    def _host(self, op, request, err: HostPathRequired):
        self.stats["host"] += 1
        if self.host_evaluator is None:
            raise err
        return self.host_evaluator(op, request)

    def isAllowed_batch(self, requests: Iterable[dict]) -> list:
        """One launch for many requests.  Each entry is a Response dict, or the
        exception the reference would reject that request's promise with."""
        requests = list(requests)
        self._ensure()
        b = self._encoder.encode(requests)
        dec = self._tables.is_allowed(b)
        self.stats["requests"] += len(requests)
        out = []
        for i, req in enumerate(requests):
            try:
                out.append(results.decision_record(self._cs, dec[i], b.host_reasons.get(i)))
            except HostPathRequired as e:
                try:
                    out.append(self._host("isAllowed", req, e))
                except Exception as x:  # noqa: BLE001 — delivered per request
                    out.append(x)
            except EvaluationError as e:
                out.append(e)
        return out

    def whatIsAllowed_batch(self, requests: Iterable[dict]) -> list:
        requests = list(requests)
        self._ensure()
        b = self._encoder.encode(requests)
        bits, obl, obl_n, dec = self._tables.what_is_allowed(b)
        long_logs = self._tables.resolve_overflow(b, dec)  # > OBL_MAX pushes: obligation-only GPU pass
        self.stats["requests"] += len(requests)
        out = []
        for i, req in enumerate(requests):
            try:
                log = long_logs[i] if i in long_logs else obl[i][:obl_n[i]]
                out.append(results.reverse_query(self._cs, b.overlay, bits[i], log, dec[i],
                                                 b.host_reasons.get(i)))
            except HostPathRequired as e:
                try:
                    out.append(self._host("whatIsAllowed", req, e))
                except Exception as x:  # noqa: BLE001
                    out.append(x)
            except EvaluationError as e:
                out.append(e)
        return out

    def isAllowed(self, request: dict) -> dict:
        r = self.isAllowed_batch([request])[0]
        if isinstance(r, Exception):
            raise r
        return r

    def whatIsAllowed(self, request: dict) -> dict:
        r = self.whatIsAllowed_batch([request])[0]
        if isinstance(r, Exception):
            raise r
        return r


__all__ = ["AccessController", "InvalidCombiningAlgorithm", "HostPathRequired", "EvaluationError", "Unsupported"]
