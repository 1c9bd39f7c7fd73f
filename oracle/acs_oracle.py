"""CPU oracle for the access-control decision path — TEST INFRASTRUCTURE ONLY.

A scalar, un-interned restatement of the reference PDP of
restorecommerce/access-control-srv (TypeScript), evaluated over JSON-shaped
Python values with explicit JS semantics (``oracle/jsval.py``).  It is the
checker for the MI355X evaluator: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  The product package
(``access-control-srv_amd/acs_mi355x``) never does.

Restated reference functions (paths relative to the reference repo root):

    AccessController.isAllowed            src/core/accessController.ts:88-324
    AccessController.whatIsAllowed        src/core/accessController.ts:326-427
    checkMultipleEntitiesMatch            src/core/accessController.ts:429-463
    resourceAttributesMatch               src/core/accessController.ts:465-654
    targetMatches                         src/core/accessController.ts:661-672
    attributesMatch                       src/core/accessController.ts:681-699
    checkSubjectMatches                   src/core/accessController.ts:793-823
    decide / denyOverrides /
      permitOverrides / firstApplicable   src/core/accessController.ts:832-893
    store mutators                        src/core/accessController.ts:79-81,897-937
    checkHierarchicalScope                src/core/hierarchicalScope.ts:10-259
    verifyACLList                         src/core/verifyACL.ts:11-251
    formatTarget / conditionMatches       src/core/utils.ts:35-56
    populate (store loader used by tests) test/utils.ts:345-383

Parity pinning: every isAllowed / whatIsAllowed assertion of the reference's
own test suite (test/core.spec.ts, test/properties.spec.ts, test/acl.spec.ts,
test/microservice.spec.ts) is committed as golden vectors under
``tests/golden/`` and checked against this oracle by ``tests/test_oracle_kats.py``.

Documented limits (raise ``OracleUnsupported``): subject ``token`` (needs the
identity service + Redis/Kafka I/O of accessController.ts:110-123,735-783),
``context_query`` with a resource adapter (GraphQL I/O), JS regex patterns
outside the subset of ``jsval.js_regex_search``.  Rule ``condition`` strings
are evaluated with Node (``node`` on PATH) exactly as utils.ts:47-56 does.
"""
from __future__ import annotations

import json
import os
import subprocess

try:  # package-relative when imported as oracle.acs_oracle, flat otherwise
    from .jsval import (UNDEF, JSError, JSTypeError, InvalidCombiningAlgorithm,
                        OracleUnsupported, get, prop, iterate, or_empty, length_gt0,
                        truthy, strict_eq, loose_eq, nullish, js_includes,
                        lodash_is_empty, lodash_find_matches_property, opt_method,
                        js_regex_search)
except ImportError:  # pragma: no cover
    from jsval import (UNDEF, JSError, JSTypeError, InvalidCombiningAlgorithm,  # type: ignore
                       OracleUnsupported, get, prop, iterate, or_empty, length_gt0,
                       truthy, strict_eq, loose_eq, nullish, js_includes,
                       lodash_is_empty, lodash_find_matches_property, opt_method,
                       js_regex_search)

PERMIT = "PERMIT"
DENY = "DENY"
INDETERMINATE = "INDETERMINATE"
# rc-grpc-clients string enum Response_Decision (keys == values), incl. ts-proto's UNRECOGNIZED
RESPONSE_DECISION = {"PERMIT", "DENY", "NOT_APPLICABLE", "INDETERMINATE", "UNRECOGNIZED"}

# cfg/config.json:272-307 (policies.options) — the service's URN + CA configuration
FULL_URNS = {
    "roleScopingEntity": "urn:restorecommerce:acs:names:roleScopingEntity",
    "roleScopingInstance": "urn:restorecommerce:acs:names:roleScopingInstance",
    "hierarchicalRoleScoping": "urn:restorecommerce:acs:names:hierarchicalRoleScoping",
    "ownerEntity": "urn:restorecommerce:acs:names:ownerIndicatoryEntity",
    "ownerInstance": "urn:restorecommerce:acs:names:ownerInstance",
    "resourceID": "urn:oasis:names:tc:xacml:1.0:resource:resource-id",
    "entity": "urn:restorecommerce:acs:names:model:entity",
    "role": "urn:restorecommerce:acs:names:role",
    "operation": "urn:restorecommerce:acs:names:operation",
    "aclIndicatoryEntity": "urn:restorecommerce:acs:names:aclIndicatoryEntity",
    "aclInstance": "urn:restorecommerce:acs:names:aclInstance",
    "actionID": "urn:oasis:names:tc:xacml:1.0:action:action-id",
    "create": "urn:restorecommerce:acs:names:action:create",
    "modify": "urn:restorecommerce:acs:names:action:modify",
    "read": "urn:restorecommerce:acs:names:action:read",
    "delete": "urn:restorecommerce:acs:names:action:delete",
    "user": "urn:restorecommerce:acs:model:user.User",
    "skipACL": "urn:restorecommerce:acs:names:skipACL",
    "property": "urn:restorecommerce:acs:names:model:property",
    "maskedProperty": "urn:restorecommerce:acs:names:obligation:maskedProperty",
}
# test/core.spec.ts:26-36 — the reduced URN set of the PDP-level tests
CORE_SPEC_URNS = {k: FULL_URNS[k] for k in (
    "roleScopingEntity", "roleScopingInstance", "hierarchicalRoleScoping", "ownerEntity",
    "ownerInstance", "resourceID", "entity", "role", "operation")}
CA_DENY = "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:deny-overrides"
CA_PERMIT = "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:permit-overrides"
CA_FIRST = "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:first-applicable"
DEFAULT_CAS = [
    {"urn": CA_DENY, "method": "denyOverrides"},
    {"urn": CA_PERMIT, "method": "permitOverrides"},
    {"urn": CA_FIRST, "method": "firstApplicable"},
]


class _Key:
    """JS Map key with SameValueZero identity (strings/undefined in practice)."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __hash__(self):
        return hash(("u",)) if self.v is UNDEF else hash((type(self.v).__name__, self.v))

    def __eq__(self, o):
        return isinstance(o, _Key) and strict_eq(self.v, o.v)


def format_target(t):
    """utils.ts:35-45"""
    if not truthy(t):
        return None
    return {
        "subjects": t["subjects"] if truthy(get(t, "subjects")) else [],
        "resources": t["resources"] if truthy(get(t, "resources")) else [],
        "actions": t["actions"] if truthy(get(t, "actions")) else [],
    }


def _from_partial(obj, keys):
    """ts-proto ``X.fromPartial``: optional fields absent -> undefined (dropped here)."""
    return {k: obj[k] for k in keys if k in obj}


_RULE_KEYS = ("id", "name", "description", "target", "effect", "condition",
              "context_query", "evaluation_cacheable")
_POLICY_KEYS = ("id", "name", "description", "target", "effect", "combining_algorithm",
                "evaluation_cacheable")


def populate_store(doc):
    """test/utils.ts:345-383: YAML doc -> ordered store with JS-Map semantics.

    Returns an insertion-ordered dict ``_Key(id) -> policySet`` whose
    ``combinables`` are ordered dicts of policies / rules.  Re-setting an
    existing key keeps its original position (Map.prototype.set).
    """
    store = {}
    for ps in doc["policy_sets"]:
        policies = {}
        for py in iterate(ps["policies"]):
            if isinstance(py, dict) and py.get("$null"):  # a null Map entry under this id (fixture form)
                policies[_Key(py.get("id", UNDEF))] = None
                continue
            rules = {}
            for ry in (py.get("rules") or []):
                rule = _from_partial(ry, _RULE_KEYS)
                rule["target"] = format_target(ry.get("target", UNDEF))
                rules[_Key(rule.get("id", UNDEF))] = rule
            pol = _from_partial(py, _POLICY_KEYS)
            pol["combinables"] = rules
            pol["target"] = format_target(py.get("target", UNDEF))
            policies[_Key(pol.get("id", UNDEF))] = pol
        pset = {"combinables": policies, "target": format_target(ps.get("target", UNDEF)),
                "policies": []}
        for k in ("id", "name", "description", "combining_algorithm"):
            if k in ps:
                pset[k] = ps[k]
        store[_Key(pset.get("id", UNDEF))] = pset
    return store


class NodeConditionEvaluator:
    """utils.ts:47-56 ``conditionMatches`` evaluated by Node's JS engine.

    ``target``, ``context`` and ``request`` are in scope as in the reference's ``eval``;
    a function-valued result is called with (request, target, context).  The condition
    text comes from test fixtures, so it runs in a fresh ``vm`` context holding only those
    three values — no ``require``, ``process`` or module scope — under a 1 s time limit.
    """

    _SCRIPT = r"""
const vm = require('vm');
const rl = require('readline').createInterface({input: process.stdin});
rl.on('line', (line) => {
  const msg = JSON.parse(line);
  const request = msg.request;
  let out;
  try {
    const r = ((condition, request) => {
      const { target, context } = request;
      condition = condition.replace(/\\n/g, '\n');
      const sandbox = vm.createContext({target, context, request});
      const evalResult = vm.runInContext(condition, sandbox, {timeout: 1000});
      if (typeof evalResult === 'function') { return evalResult(request, target, context); }
      return evalResult;
    })(msg.condition, request);
    out = {ok: true, truthy: !!r};
  } catch (err) {
    out = {ok: false, code: (err && Number.isInteger(err.code)) ? err.code : 500,
           message: (err && err.message !== undefined && err.message !== null) ? err.message : 'Unknown Error!'};
  }
  process.stdout.write(JSON.stringify(out) + '\n');
});
"""

    def __init__(self):
        self._p = None

    def _proc(self):
        if self._p is None:
            self._p = subprocess.Popen(["node", "-e", self._SCRIPT], stdin=subprocess.PIPE,
                                       stdout=subprocess.PIPE, text=True, bufsize=1)
        return self._p

    def __call__(self, condition, request):
        p = self._proc()
        p.stdin.write(json.dumps({"condition": condition, "request": _to_json(request)}) + "\n")
        p.stdin.flush()
        return json.loads(p.stdout.readline())

    def close(self):
        if self._p is not None:
            self._p.stdin.close()
            self._p.wait(timeout=10)
            self._p = None


def _to_json(v):
    if v is UNDEF:
        return None
    if isinstance(v, dict):
        return {k: _to_json(x) for k, x in v.items() if x is not UNDEF}
    if isinstance(v, list):
        return [_to_json(x) for x in v]
    return v


class Oracle:
    """Scalar restatement of ``AccessController`` (accessController.ts:31-966)."""

    def __init__(self, urns=None, combining_algorithms=None, condition_eval=None):
        # accessController.ts:46-67
        self.urns = dict(FULL_URNS if urns is None else urns)
        cas = DEFAULT_CAS if combining_algorithms is None else combining_algorithms
        self.cas = {}
        for ca in cas:
            if ca["method"] not in ("denyOverrides", "permitOverrides", "firstApplicable"):
                raise InvalidCombiningAlgorithm(ca["urn"])
            self.cas[_Key(ca.get("urn", UNDEF))] = ca["method"]
        self.policy_sets = {}
        self.condition_eval = condition_eval
        self.resource_adapter = None

    def U(self, name):
        return self.urns.get(name, UNDEF)

    # ------------------------------------------------------------ store mutators
    def load(self, doc):
        for k, ps in populate_store(doc).items():
            self.policy_sets[k] = ps

    def clear_policies(self):
        self.policy_sets.clear()

    def update_policy_set(self, ps):
        self.policy_sets[_Key(ps.get("id", UNDEF))] = ps

    def remove_policy_set(self, ps_id):
        self.policy_sets.pop(_Key(ps_id), None)

    def update_policy(self, ps_id, policy):
        ps = self.policy_sets.get(_Key(ps_id))
        if ps is not None:
            ps["combinables"][_Key(policy.get("id", UNDEF))] = policy

    def remove_policy(self, ps_id, pol_id):
        ps = self.policy_sets.get(_Key(ps_id))
        if ps is not None:
            ps["combinables"].pop(_Key(pol_id), None)

    def update_rule(self, ps_id, pol_id, rule):
        ps = self.policy_sets.get(_Key(ps_id))
        if ps is not None:
            pol = ps["combinables"].get(_Key(pol_id))
            if pol is not None:
                pol["combinables"][_Key(rule.get("id", UNDEF))] = rule

    def remove_rule(self, ps_id, pol_id, rule_id):
        ps = self.policy_sets.get(_Key(ps_id))
        if ps is not None:
            pol = ps["combinables"].get(_Key(pol_id))
            if pol is not None:
                pol["combinables"].pop(_Key(rule_id), None)

    # ------------------------------------------------------------ combining
    def _decide(self, ca, effects):
        """accessController.ts:832-893"""
        method = self.cas.get(_Key(ca))
        if method is None:
            raise InvalidCombiningAlgorithm(ca)
        if method == "firstApplicable":
            return effects[0]
        want = DENY if method == "denyOverrides" else PERMIT
        chosen = {"effect": UNDEF, "evaluation_cacheable": UNDEF}
        for e in effects:
            chosen = {"effect": e["effect"], "evaluation_cacheable": e["evaluation_cacheable"]}
            if strict_eq(e["effect"], want):
                break
        return chosen

    def _ca_policy_effect(self, policy, policy_effect):
        """accessController.ts:138-148: the CA branch compares a function with a
        string and can never fire; only a truthy policy.effect updates it."""
        eff = prop(policy, "effect")
        if truthy(eff):
            return eff
        return policy_effect

    # ------------------------------------------------------------ matchers
    def _attributes_match(self, rule_attrs, req_attrs):
        """accessController.ts:681-699 (loose ==)"""
        for a in or_empty(rule_attrs):
            aid, av = get(a, "id"), get(a, "value")
            found = False
            if not nullish(req_attrs):
                for ra in iterate(req_attrs):
                    if loose_eq(get(ra, "id"), aid) and loose_eq(get(ra, "value"), av):
                        found = True
                        break
            if not found:
                return False
        return True

    def _subject_matches(self, rule_subs, req_subs, request):
        """accessController.ts:793-823"""
        ctx = get(request, "context")
        role_urn = self.U("role")
        if nullish(rule_subs) or len(rule_subs) == 0:
            return True
        rule_role = UNDEF
        for s in rule_subs:
            if strict_eq(get(s, "id"), role_urn):
                rule_role = get(s, "value")
        if not truthy(rule_role):
            return self._attributes_match(rule_subs, req_subs)
        ras = get(get(ctx, "subject"), "role_associations")
        if not truthy(ras):
            return False
        return any(strict_eq(get(r, "role"), rule_role) for r in iterate(ras))

    def _regex_entity(self, rule_value, req_value):
        """Shared namespace/regex entity test (accessController.ts:528-566,
        hierarchicalScope.ts:64-101).  Returns (reset, hit); raises JSTypeError on
        a nullish value (``nsEntityArray[0]`` of undefined) and JSSyntaxError on a
        malformed pattern."""
        pattern = opt_method(rule_value, "substring", opt_method(rule_value, "lastIndexOf", ":") + 1) \
            if not nullish(rule_value) else UNDEF
        ns_arr = opt_method(pattern, "split", ".")
        ns_or_entity = prop(ns_arr, 0)
        entity_rx = prop(ns_arr, len(ns_arr) - 1)
        rule_ns = UNDEF
        if ns_or_entity.upper() != entity_rx.upper():
            rule_ns = ns_or_entity.upper()
        req_ns_prefix = UNDEF if nullish(req_value) else opt_method(
            req_value, "substring", 0, opt_method(req_value, "lastIndexOf", ":"))
        rule_ns_prefix = UNDEF if nullish(rule_value) else opt_method(
            rule_value, "substring", 0, opt_method(rule_value, "lastIndexOf", ":"))
        reset = not loose_eq(req_ns_prefix, rule_ns_prefix)
        req_pattern = UNDEF if nullish(req_value) else opt_method(
            req_value, "substring", opt_method(req_value, "lastIndexOf", ":") + 1)
        req_arr = opt_method(req_pattern, "split", ".")
        req_ns_or_entity = prop(req_arr, 0)
        req_entity = prop(req_arr, len(req_arr) - 1)
        req_ns = UNDEF
        if req_ns_or_entity.upper() != req_entity.upper():
            req_ns = req_ns_or_entity.upper()
        hit = False
        if (truthy(req_ns) and truthy(rule_ns) and strict_eq(req_ns, rule_ns)) or \
                (not truthy(req_ns) and not truthy(rule_ns)):
            hit = js_regex_search(entity_rx, req_entity)
        return reset, hit

    def _resource_attrs_match(self, rule_attrs, req_attrs, operation, masks, effect, regex):
        """accessController.ts:465-654"""
        ent, prop_urn = self.U("entity"), self.U("property")
        masked_urn, op_urn = self.U("maskedProperty"), self.U("operation")
        entity_match = property_match = rule_props = req_props = operation_match = False
        req_entity_urn = ""
        skip_deny = True
        rule_prop_value = ""
        if lodash_is_empty(rule_attrs):
            return True
        req_list = or_empty(req_attrs)
        for ra in req_list:
            if strict_eq(prop(ra, "id"), prop_urn):
                req_props = True
        for qa in req_list:
            property_match = False
            for r in or_empty(rule_attrs):
                rid, rval = get(r, "id"), get(r, "value")
                qid, qval = get(qa, "id"), get(qa, "value")
                if strict_eq(prop(r, "id"), prop_urn):
                    rule_props = True
                    rule_prop_value = prop(r, "value")
                if not regex:
                    if strict_eq(qid, ent) and strict_eq(rid, ent) and strict_eq(qval, rval):
                        entity_match = True
                        req_entity_urn = prop(qa, "value")
                    elif strict_eq(qid, op_urn) and strict_eq(rid, op_urn) and strict_eq(qval, rval):
                        operation_match = True
                    elif entity_match and strict_eq(qid, prop_urn) and strict_eq(rid, prop_urn):
                        if nullish(req_entity_urn):
                            entity_name = UNDEF
                        else:
                            entity_name = opt_method(req_entity_urn, "substring",
                                                     opt_method(req_entity_urn, "lastIndexOf", ":") + 1)
                        idx = opt_method(qval, "indexOf", entity_name)
                        if idx is not UNDEF and idx > -1:
                            if strict_eq(rval, qval):
                                property_match = True
                        elif strict_eq(effect, PERMIT):
                            property_match = True
                else:
                    if strict_eq(qid, ent) and strict_eq(rid, ent):
                        reset, hit = self._regex_entity(rval, qval)
                        req_entity_urn = qval
                        if reset:
                            entity_match = False
                        if hit:
                            entity_match = True
                    elif entity_match and strict_eq(qid, prop_urn) and strict_eq(rid, prop_urn):
                        rps = UNDEF if nullish(rval) else opt_method(rval, "substring",
                                                                      opt_method(rval, "lastIndexOf", "#") + 1)
                        qps = UNDEF if nullish(qval) else opt_method(qval, "substring",
                                                                      opt_method(qval, "lastIndexOf", "#") + 1)
                        if strict_eq(rps, qps):
                            property_match = True
            qid = get(qa, "id")
            scope = strict_eq(qid, prop_urn) or not req_props
            if operation == "isAllowed" and strict_eq(effect, DENY) and scope and entity_match \
                    and rule_props and property_match:
                skip_deny = False
            if operation == "isAllowed" and strict_eq(effect, PERMIT) and scope and entity_match \
                    and rule_props and not property_match:
                return False
            if operation == "whatIsAllowed" and strict_eq(effect, PERMIT) and scope and entity_match \
                    and rule_props and not property_match:
                if not req_props:
                    return False
                if self._push_mask(masks, qa, req_props, req_entity_urn, rule_prop_value):
                    continue
            if operation == "whatIsAllowed" and strict_eq(effect, DENY) and scope and entity_match \
                    and rule_props and (property_match or not req_props):
                if self._push_mask(masks, qa, req_props, req_entity_urn, rule_prop_value):
                    continue
        if skip_deny and rule_props and req_props and strict_eq(effect, DENY) \
                and operation == "isAllowed" and not property_match:
            return False
        if not entity_match and not operation_match:
            return False
        return True

    def _push_mask(self, masks, qa, req_props, req_entity_urn, rule_prop_value):
        """maskedProperty obligation append (accessController.ts:597-614, 622-639).
        Returns True where the reference ``continue``s."""
        existing = UNDEF
        for m in masks:
            if strict_eq(get(m, "value"), req_entity_urn):
                existing = m
                break
        mask_prop = UNDEF
        qval = get(qa, "value")
        if req_props and truthy(qval):
            mask_prop = qval
        elif not req_props:
            mask_prop = rule_prop_value
        idx = opt_method(mask_prop, "indexOf", "#")
        if idx is not UNDEF and idx <= -1:
            return True
        entry = {"id": self.U("maskedProperty"), "value": mask_prop, "attributes": []}
        if existing is UNDEF:
            masks.append({"id": self.U("entity"), "value": req_entity_urn, "attributes": [entry]})
        else:
            existing["attributes"].append(entry)
        return False

    def _target_matches(self, target, request, operation, masks, effect=UNDEF, regex=False):
        """accessController.ts:661-672 (``effect`` defaults to PERMIT when undefined)."""
        if effect is UNDEF:
            effect = PERMIT
        req_target = prop(request, "target")
        if not self._subject_matches(prop(target, "subjects"), prop(req_target, "subjects"), request):
            return False
        if not self._attributes_match(prop(target, "actions"), prop(req_target, "actions")):
            return False
        return self._resource_attrs_match(prop(target, "resources"), prop(req_target, "resources"),
                                          operation, masks, effect, regex)

    def _multiple_entities_match(self, pset, request, masks):
        """accessController.ts:429-463"""
        exact = True
        ent = self.U("entity")
        for qa in or_empty(get(get(request, "target"), "resources")):
            if strict_eq(prop(qa, "id"), ent):
                multi = False
                for pol in pset["combinables"].values():
                    pe = UNDEF
                    if truthy(prop(pol, "effect")):
                        pe = pol["effect"]
                    if length_gt0(get(get(pol, "target"), "resources")):
                        if self._resource_attrs_match(pol["target"]["resources"], [qa], "isAllowed",
                                                      masks, pe, False):
                            multi = True
                if not multi:
                    exact = False
                    break
        return exact

    # ------------------------------------------------------------ HR scope
    def _flat_hr(self, scopes, rule_role):
        """hierarchicalScope.ts:207-220: unique truthy ids of the HR subtrees whose
        top-level role === ruleRole (descendants unfiltered).  Only membership is
        used by the caller, so it is returned as a set (memoised per request)."""
        if nullish(scopes):
            raise JSTypeError("undefined is not iterable")  # getAllChildNodes(undefined)
        key = (id(scopes), rule_role if rule_role is UNDEF or isinstance(rule_role, str) else repr(rule_role))
        memo = getattr(self, "_flat_memo", None)
        if memo is not None and key in memo:
            return memo[key]
        roots = [h for h in iterate(scopes) if strict_eq(get(h, "role"), rule_role)]
        out = set()
        stack = list(reversed(roots))
        while stack:
            h = stack.pop()
            hid = get(h, "id")
            if truthy(hid):
                if isinstance(hid, (dict, list)):
                    raise OracleUnsupported("object-valued HR id")
                out.add(hid)
            if length_gt0(get(h, "children")):
                stack.extend(reversed(iterate(h["children"])))
        if memo is not None:
            memo[key] = out
        return out

    def _check_hierarchical_scope(self, target, request):
        """hierarchicalScope.ts:10-259"""
        owners_map = {}  # _Key(resourceId) -> owners, insertion ordered (Map)
        subs = get(target, "subjects")
        if not nullish(subs) and strict_eq(get(subs, "length"), 0):
            return True
        hr_check = "true"
        rule_role = UNDEF
        scoping_entity = UNDEF
        role_urn = self.U("role")
        for s in or_empty(subs) if not nullish(subs) else []:
            sid = get(s, "id")
            if strict_eq(sid, role_urn):
                rule_role = get(s, "value")
            elif strict_eq(sid, self.U("hierarchicalRoleScoping")):
                hr_check = prop(s, "value")
            elif strict_eq(sid, self.U("roleScopingEntity")):
                scoping_entity = prop(s, "value")
        if not truthy(scoping_entity):
            return True
        ctx = get(request, "context")
        if lodash_is_empty(ctx):
            return False
        ctx_resources = or_empty(get(ctx, "resources"))
        req_target = get(request, "target")
        eoo = UNDEF
        for attr in or_empty(prop(target, "resources")):
            if loose_eq(get(attr, "id"), self.U("entity")):
                eoo = get(attr, "value")
                entities_match = False
                for qa in or_empty(prop(req_target, "resources")):
                    if loose_eq(get(qa, "id"), get(attr, "id")) and loose_eq(get(qa, "value"), eoo):
                        entities_match = True
                    elif loose_eq(get(qa, "id"), get(attr, "id")):
                        reset, hit = self._regex_entity(eoo, get(qa, "value"))
                        if reset:
                            entities_match = False
                        if hit:
                            entities_match = True
                    elif loose_eq(get(qa, "id"), self.U("resourceID")) and entities_match:
                        inst_id = get(qa, "value")
                        res = lodash_find_matches_property(ctx_resources, "instance.id", inst_id)
                        if truthy(res):
                            res = get(res, "instance")
                        else:
                            res = lodash_find_matches_property(ctx_resources, "id", inst_id)
                        if truthy(res):
                            meta = get(res, "meta")
                            if lodash_is_empty(meta) or lodash_is_empty(get(meta, "owners")):
                                return False
                            owners_map[_Key(inst_id)] = meta["owners"]
                        else:
                            return False
            elif strict_eq(get(attr, "id"), self.U("operation")):
                eoo = get(attr, "value")
                for qa in or_empty(prop(req_target, "resources")):
                    if strict_eq(get(qa, "id"), get(attr, "id")) and strict_eq(get(qa, "value"), get(attr, "value")):
                        res = lodash_find_matches_property(ctx_resources, "id", eoo)
                        if truthy(res):
                            meta = get(res, "meta")
                            if lodash_is_empty(meta) or lodash_is_empty(get(meta, "owners")):
                                return False
                            owners_map[_Key(eoo)] = meta["owners"]
                        else:
                            return False
        ras = get(get(ctx, "subject"), "role_associations")
        if lodash_is_empty(ras):
            return False
        reduced = [r for r in iterate(ras) if strict_eq(prop(r, "role"), rule_role)]
        rse, oe, rsi = self.U("roleScopingEntity"), self.U("ownerEntity"), self.U("roleScopingInstance")

        def direct(owner):
            for ra in reduced:
                for rae in or_empty(get(ra, "attributes")) if not nullish(get(ra, "attributes")) else []:
                    if strict_eq(get(rae, "id"), rse) and strict_eq(get(owner, "id"), oe) \
                            and strict_eq(prop(owner, "value"), scoping_entity) \
                            and strict_eq(prop(owner, "value"), get(rae, "value")):
                        insts = get(rae, "attributes")
                        if nullish(insts):
                            continue
                        for inst in iterate(insts):
                            if strict_eq(get(inst, "id"), rsi):
                                oattrs = get(owner, "attributes")
                                if nullish(oattrs):
                                    continue
                                for oa in iterate(oattrs):
                                    if strict_eq(get(oa, "value"), get(inst, "value")):
                                        if truthy(oa):
                                            return True
                                        break
        # Map iteration + deferred delete (hierarchicalScope.ts:164-191)
        remaining = [k for k, owners in owners_map.items()
                     if not any(direct(o) for o in iterate(owners))]
        if not remaining:
            return True
        if strict_eq(hr_check, "true"):
            if truthy(get(get(ctx, "subject"), "token")) and lodash_is_empty(get(ctx["subject"], "hierarchical_scopes")):
                raise OracleUnsupported("createHRScope I/O (token)")
            flat = self._flat_hr(get(get(ctx, "subject"), "hierarchical_scopes"), rule_role)

            def owner_ok(owner):
                for ra in reduced:
                    for rae in or_empty(get(ra, "attributes")) if not nullish(get(ra, "attributes")) else []:
                        if strict_eq(get(rae, "id"), rse) and strict_eq(get(owner, "id"), oe) \
                                and strict_eq(get(owner, "value"), scoping_entity) \
                                and strict_eq(get(owner, "value"), get(rae, "value")):
                            return True
                return False
            still = []
            for k in remaining:
                insts = []
                for owner in iterate(owners_map[k]):
                    if owner_ok(owner):
                        oattrs = get(owner, "attributes")
                        if nullish(oattrs):
                            insts.append(UNDEF)
                        else:
                            insts.extend(get(a, "value") for a in iterate(oattrs)
                                         if strict_eq(get(a, "id"), self.U("ownerInstance")))
                if not any(isinstance(x, str) and x in flat for x in insts):
                    still.append(k)
            remaining = still
        return not remaining

    # ------------------------------------------------------------ ACL
    def _verify_acl(self, target, request):
        """verifyACL.ts:11-251"""
        scoped_roles = []
        for a in or_empty(prop(target, "subjects")):
            if strict_eq(prop(a, "id"), self.U("role")):
                scoped_roles.append(a["value"] if "value" in a else UNDEF)
            elif strict_eq(prop(a, "id"), self.U("skipACL")):
                return True
        ctx = get(request, "context")
        if lodash_is_empty(ctx):
            ctx = {}
        ctx_resources = or_empty(prop(ctx, "resources"))
        req_target = get(request, "target")
        tmap = {}  # _Key(scopingEntity) -> [instances]
        for qa in or_empty(prop(req_target, "resources")):
            if loose_eq(prop(qa, "id"), self.U("resourceID")) or strict_eq(prop(qa, "id"), self.U("operation")):
                inst_id = prop(qa, "value")
                res = lodash_find_matches_property(ctx_resources, "instance.id", inst_id)
                acl_list = UNDEF
                if truthy(res):
                    res = prop(res, "instance")
                else:
                    res = lodash_find_matches_property(ctx_resources, "id", inst_id)
                if truthy(res):
                    meta = prop(res, "meta")
                    if length_gt0(get(meta, "acls")):
                        acl_list = meta["acls"]
                if lodash_is_empty(acl_list):
                    return True
                for acl in iterate(acl_list):
                    if strict_eq(get(acl, "id"), self.U("aclIndicatoryEntity")):
                        se = prop(acl, "value")
                        if _Key(se) not in tmap:
                            tmap[_Key(se)] = []
                        attrs = prop(acl, "attributes")
                        if not truthy(attrs) or strict_eq(get(attrs, "length"), 0):
                            return False
                        for at in iterate(attrs):
                            if strict_eq(prop(at, "id"), self.U("aclInstance")):
                                tmap[_Key(se)].append(prop(at, "value"))
                            else:
                                return False
                    else:
                        return False
        subj = prop(ctx, "subject")
        if truthy(get(subj, "token")) and lodash_is_empty(get(subj, "hierarchical_scopes")):
            raise OracleUnsupported("createHRScope I/O (token)")
        ras = prop(subj, "role_associations")
        if lodash_is_empty(ras):
            return False
        smap = {}
        t_entities = [k.v for k in tmap]
        for ra in iterate(ras):
            role = get(ra, "role")
            attrs = or_empty(get(ra, "attributes"))
            if js_includes(scoped_roles, role):
                for rattr in iterate(attrs):
                    if strict_eq(get(rattr, "id"), self.U("roleScopingEntity")) \
                            and js_includes(t_entities, get(rattr, "value")):
                        rse_v = get(rattr, "value")
                        if not truthy(smap.get(_Key(rse_v))):
                            smap[_Key(rse_v)] = []
                        if length_gt0(get(rattr, "attributes")):
                            for ri in iterate(rattr["attributes"]):
                                if strict_eq(get(ri, "id"), self.U("roleScopingInstance")):
                                    smap[_Key(rse_v)].append(get(ri, "value"))
        actions = get(req_target, "actions")
        role_orgs = {}  # _Key(role) -> [org ids]

        def walk(nodes, role):
            for h in iterate(nodes):
                hr = prop(h, "role")
                key = role if nullish(hr) else hr
                if truthy(get(h, "id")):
                    role_orgs.setdefault(_Key(key), []).append(h["id"])
                if length_gt0(get(h, "children")):
                    walk(h["children"], key)
        walk(get(subj, "hierarchical_scopes"), UNDEF)
        a0 = get(actions, 0) if truthy(actions) else UNDEF
        is_action = truthy(actions) and truthy(a0) and strict_eq(prop(a0, "id"), self.U("actionID"))
        if is_action and strict_eq(prop(a0, "value"), self.U("create")):
            valid = False
            if len(t_entities) == 0:
                return True
            for se in t_entities:
                if strict_eq(se, self.U("user")):
                    valid = True
                    continue
                t_inst = tmap[_Key(se)]
                if _Key(se) not in smap:  # smap.get(se) undefined -> `!subjectInstances`
                    return False
                validated = []
                for rk, orgs in role_orgs.items():
                    if js_includes(scoped_roles, rk.v):
                        for ti in t_inst:
                            if js_includes(orgs, ti):
                                valid = True
                                validated.append(ti)
                                continue
                            elif not js_includes(validated, ti):
                                valid = False
                                break
                if not valid:
                    return False
            if valid:
                return True
        if is_action and (strict_eq(prop(a0, "value"), self.U("read")) or strict_eq(prop(a0, "value"), self.U("modify"))
                          or strict_eq(prop(a0, "value"), self.U("delete"))):
            valid_sub = False
            if len(t_entities) == 0:
                return True
            for se in t_entities:
                t_inst = tmap[_Key(se)]
                s_inst = smap.get(_Key(se), UNDEF)
                if strict_eq(se, self.U("user")):
                    if js_includes(t_inst, get(subj, "id")):
                        valid_sub = True
                        break
                if length_gt0(s_inst):
                    for si in s_inst:
                        if js_includes(t_inst, si):
                            valid_sub = True
                            break
            return valid_sub
        return False

    # ------------------------------------------------------------ condition
    def _condition(self, rule, request):
        """accessController.ts:227-270 (+ utils.ts:47-56).  Returns (matches, early_response)."""
        ad = self.resource_adapter
        cq = get(rule, "context_query")
        if ad is not None and (length_gt0(get(cq, "filters")) or length_gt0(get(cq, "query"))):
            raise OracleUnsupported("context_query via resource adapter (GraphQL I/O)")
        if self.condition_eval is None:
            raise OracleUnsupported("rule condition without a JS evaluator")
        res = self.condition_eval(rule["condition"], request)
        if res["ok"]:
            return res["truthy"], None
        return False, {"code": res["code"], "message": res["message"]}

    # ------------------------------------------------------------ isAllowed
    def is_allowed(self, request):
        """accessController.ts:88-324.  Returns the Response dict, raises JSError
        where the reference's promise rejects."""
        if not truthy(get(request, "target")):
            return {"decision": DENY, "evaluation_cacheable": False, "obligations": [],
                    "operation_status": {"code": 400,
                                         "message": "Access request had no target. Skipping request"}}
        effect = UNDEF
        obligations = []
        self._flat_memo = {}
        ctx = get(request, "context")
        if truthy(get(get(ctx, "subject"), "token")):
            raise OracleUnsupported("subject token (identity-srv / Redis I/O)")
        for pset in list(self.policy_sets.values()):
            policy_effects = []
            pe = UNDEF
            st = get(pset, "target")
            if truthy(st) and not self._target_matches(st, request, "isAllowed", obligations):
                continue
            exact = False
            for pol in pset["combinables"].values():
                pe = self._ca_policy_effect(pol, pe)
                if truthy(get(pol, "target")) and self._target_matches(pol["target"], request, "isAllowed",
                                                                        obligations, pe):
                    exact = True
                    break
            ent = self.U("entity")
            if exact:
                n_ent = sum(1 for a in or_empty(get(get(request, "target"), "resources"))
                            if strict_eq(get(a, "id"), ent))
                if n_ent > 1:
                    exact = self._multiple_entities_match(pset, request, obligations)
            for pol in pset["combinables"].values():
                if not truthy(pol):
                    continue
                rule_effects = []
                ptarget = get(pol, "target")
                gate = (not truthy(ptarget)) or \
                    (exact and self._target_matches(ptarget, request, "isAllowed", obligations, pe)) or \
                    ((not exact) and self._target_matches(ptarget, request, "isAllowed", obligations, pe, True))
                if not gate:
                    continue
                if length_gt0(get(ptarget, "subjects")):
                    psm = self._check_hierarchical_scope(ptarget, request)
                else:
                    psm = True
                rules = pol["combinables"]
                if len(rules) == 0 and truthy(get(pol, "effect")):
                    policy_effects.append({"effect": pol["effect"],
                                           "evaluation_cacheable": get(pol, "evaluation_cacheable")})
                    continue
                ec_rule = True
                for rule in rules.values():
                    if not truthy(rule):
                        continue
                    ec = get(rule, "evaluation_cacheable")
                    if not truthy(ec):
                        ec_rule = False
                    rt = get(rule, "target")
                    m = (not truthy(rt)) or self._target_matches(rt, request, "isAllowed", obligations,
                                                                 get(rule, "effect"))
                    if not m:
                        m = self._target_matches(rt, request, "isAllowed", obligations, get(rule, "effect"), True)
                    if not m:
                        continue
                    if truthy(rt):
                        m = self._check_hierarchical_scope(rt, request)
                    if m and length_gt0(get(rule, "condition")):
                        m, early = self._condition(rule, request)
                        if early is not None:
                            return {"decision": DENY, "obligations": obligations, "evaluation_cacheable": ec,
                                    "operation_status": early}
                    if m and truthy(rt):
                        m = self._verify_acl(rt, request)
                    if m and psm:
                        if not ec_rule:
                            ec = False
                        rule_effects.append({"effect": get(rule, "effect"), "evaluation_cacheable": ec})
                if rule_effects:
                    policy_effects.append(self._decide(get(pol, "combining_algorithm"), rule_effects))
            if policy_effects:
                effect = self._decide(get(pset, "combining_algorithm"), policy_effects)
        if effect is UNDEF:
            return {"decision": INDETERMINATE, "obligations": obligations, "evaluation_cacheable": UNDEF,
                    "operation_status": {"code": 200, "message": "success"}}
        e = effect["effect"]
        decision = e if isinstance(e, str) and e in RESPONSE_DECISION else INDETERMINATE
        return {"decision": decision, "obligations": obligations,
                "evaluation_cacheable": effect["evaluation_cacheable"],
                "operation_status": {"code": 200, "message": "success"}}

    # ------------------------------------------------------------ whatIsAllowed
    def what_is_allowed(self, request):
        """accessController.ts:326-427.  Returns {policy_sets, obligations,
        operation_status} with policy/rule objects reduced to the picked fields."""
        ctx = get(request, "context")
        if truthy(get(get(ctx, "subject"), "token")):
            raise OracleUnsupported("subject token (identity-srv / Redis I/O)")
        out_sets = []
        obligations = []
        for pset in list(self.policy_sets.values()):
            st = get(pset, "target")
            if not (lodash_is_empty(st) or self._target_matches(st, request, "whatIsAllowed", obligations)):
                continue
            ps_rq = {"combining_algorithm": get(pset, "combining_algorithm")}
            for k in ("id", "target", "effect"):
                if k in pset:
                    ps_rq[k] = pset[k]
            ps_rq["policies"] = []
            exact = False
            pe = UNDEF
            for pol in pset["combinables"].values():
                pe = self._ca_policy_effect(pol, pe)
                if truthy(get(pol, "target")) and self._target_matches(pol["target"], request, "whatIsAllowed",
                                                                        obligations, pe):
                    exact = True
                    break
            ent = self.U("entity")
            if exact:
                n_ent = sum(1 for a in or_empty(get(get(request, "target"), "resources"))
                            if strict_eq(get(a, "id"), ent))
                if n_ent > 1:
                    exact = self._multiple_entities_match(pset, request, obligations)
            for pol in pset["combinables"].values():
                if not truthy(pol):
                    continue
                pt = get(pol, "target")
                gate = lodash_is_empty(pt) or \
                    (exact and self._target_matches(pt, request, "whatIsAllowed", obligations, pe)) or \
                    ((not exact) and self._target_matches(pt, request, "whatIsAllowed", obligations, pe, True))
                if not gate:
                    continue
                p_rq = {"combining_algorithm": get(pol, "combining_algorithm")}
                for k in ("id", "target", "effect", "evaluation_cacheable"):
                    if k in pol:
                        p_rq[k] = pol[k]
                p_rq["rules"] = []
                p_rq["has_rules"] = truthy(get(pol, "combinables")) and len(pol["combinables"]) > 0
                for rule in pol["combinables"].values():
                    if not truthy(rule):
                        continue
                    rt = get(rule, "target")
                    m = lodash_is_empty(rt) or self._target_matches(rt, request, "whatIsAllowed", obligations,
                                                                    get(rule, "effect"))
                    if not m:
                        m = self._target_matches(rt, request, "whatIsAllowed", obligations, get(rule, "effect"),
                                                 True)
                    if lodash_is_empty(rt) or m:
                        r_rq = {"context_query": get(rule, "context_query")}
                        for k in ("id", "target", "effect", "condition", "evaluation_cacheable"):
                            if k in rule:
                                r_rq[k] = rule[k]
                        p_rq["rules"].append(r_rq)
                if truthy(get(p_rq, "effect")) or (not truthy(get(p_rq, "effect")) and p_rq["rules"]):
                    ps_rq["policies"].append(p_rq)
            if ps_rq["policies"]:
                out_sets.append(ps_rq)
        return {"policy_sets": out_sets, "obligations": obligations,
                "operation_status": {"code": 200, "message": "success"}}


def run_is_allowed(oracle, request):
    """Normalised outcome for parity checks: ('OK', response) or ('ERR', kind)."""
    try:
        return "OK", oracle.is_allowed(request)
    except JSError as e:
        return "ERR", e.kind


def run_what_is_allowed(oracle, request):
    try:
        return "OK", oracle.what_is_allowed(request)
    except JSError as e:
        return "ERR", e.kind
