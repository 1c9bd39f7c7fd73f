"""Restatement of the reference test helper ``buildRequest`` (test/utils.ts:24-280).

Produces the request in its post-``unmarshallContext`` JSON shape (undefined
keys dropped, as ``marshallRequest`` -> gRPC -> ``JSON.parse`` does).  The
acs-client ``urns`` constants it reads (``urns.role`` …) are the
``authorization.urns`` block of cfg/config.json:224-253, the same strings the
helper itself spells out literally in its multi-entity branch.
"""
from __future__ import annotations

URN_ROLE = "urn:restorecommerce:acs:names:role"
URN_SUBJECT_ID = "urn:oasis:names:tc:xacml:1.0:subject:subject-id"
URN_EXECUTE = "urn:restorecommerce:acs:names:action:execute"
URN_OPERATION = "urn:restorecommerce:acs:names:operation"
URN_ENTITY = "urn:restorecommerce:acs:names:model:entity"
URN_RESOURCE_ID = "urn:oasis:names:tc:xacml:1.0:resource:resource-id"
URN_PROPERTY = "urn:restorecommerce:acs:names:model:property"
URN_ACTION_ID = "urn:oasis:names:tc:xacml:1.0:action:action-id"
URN_ACL_IE = "urn:restorecommerce:acs:names:aclIndicatoryEntity"
URN_ACL_INST = "urn:restorecommerce:acs:names:aclInstance"
URN_OWNER_IE = "urn:restorecommerce:acs:names:ownerIndicatoryEntity"
URN_OWNER_INST = "urn:restorecommerce:acs:names:ownerInstance"
URN_RSE = "urn:restorecommerce:acs:names:roleScopingEntity"
URN_RSI = "urn:restorecommerce:acs:names:roleScopingInstance"


def _attr(i, v):
    a = {"id": i, "attributes": []}
    if v is not None:
        a["value"] = v
    return a


def _drop_none(d):
    return {k: v for k, v in d.items() if v is not None}


def build_request(o: dict) -> dict:
    rtype = o.get("resourceType")
    resources, actions = [], []
    subjects = [_attr(URN_ROLE, o.get("subjectRole") or "SimpleUser"),
                _attr(URN_SUBJECT_ID, o.get("subjectID"))]
    rid = o.get("resourceID")
    rprop = o.get("resourceProperty")
    if o.get("actionType") == URN_EXECUTE:
        for name in ([rtype] if isinstance(rtype, str) else rtype):
            resources.append(_attr(URN_OPERATION, name))
    elif isinstance(rtype, str):
        resources += [_attr(URN_ENTITY, rtype), _attr(URN_RESOURCE_ID, rid)]
        if rprop and isinstance(rprop, str):
            resources.append(_attr(URN_PROPERTY, rprop))
        elif rprop and isinstance(rprop, list):
            for p in rprop:
                resources.append(_attr(URN_PROPERTY, p))
    else:
        for i, t in enumerate(rtype):
            r_i = rid[i] if (rid and i < len(rid) and rid[i]) else None
            resources += [_attr(URN_ENTITY, t), _attr(URN_RESOURCE_ID, r_i)]
            if rprop and isinstance(rprop, str):
                resources.append(_attr(URN_PROPERTY, rprop))
            elif rprop and isinstance(rprop, list):
                for p in rprop:
                    if isinstance(p, str):
                        resources.append(_attr(URN_PROPERTY, p))
                    elif isinstance(p, list):
                        ename = t[t.rfind(":") + 1:]
                        for q in p:
                            if ename in q:
                                resources.append(_attr(URN_PROPERTY, q))
    actions.append(_attr(URN_ACTION_ID, o.get("actionType")))

    acls = []
    if o.get("aclIndicatoryEntity") and o.get("aclInstances"):
        acls = [{"id": URN_ACL_IE, "value": o["aclIndicatoryEntity"],
                 "attributes": [{"id": URN_ACL_INST, "value": x} for x in o["aclInstances"]]}]
    elif o.get("multipleAclIndicatoryEntity") and o.get("orgInstances") and o.get("subjectInstances"):
        acls = [{"id": URN_ACL_IE, "value": o["multipleAclIndicatoryEntity"][0],
                 "attributes": [{"id": URN_ACL_INST, "value": x} for x in o["orgInstances"]]},
                {"id": URN_ACL_IE, "value": o["multipleAclIndicatoryEntity"][1],
                 "attributes": [{"id": URN_ACL_INST, "value": x} for x in o["subjectInstances"]]}]

    stamp = "2024-01-01T00:00:00.000Z"
    oie, oinst = o.get("ownerIndicatoryEntity"), o.get("ownerInstance")
    ctx_res = []
    if isinstance(rtype, str):
        owners = []
        if oie and not isinstance(oinst, list):
            owners = [{"id": URN_OWNER_IE, "value": oie,
                       "attributes": [_drop_none({"id": URN_OWNER_INST, "value": oinst})]}]
        ctx_res = [_drop_none({"id": rid, "meta": {"created": stamp, "modified": stamp,
                                                    "acls": acls, "owners": owners}})]
    else:
        for i in range(len(rtype)):
            r_i = rid[i] if (rid and i < len(rid) and rid[i]) else None
            owners = []
            if oie and oinst:
                owners = [{"id": URN_OWNER_IE, "value": oie,
                           "attributes": [_drop_none({"id": URN_OWNER_INST,
                                                      "value": oinst[i] if i < len(oinst) else None})]}]
            ctx_res.append(_drop_none({"id": r_i, "meta": {"created": stamp, "modified": stamp,
                                                           "acls": acls, "owners": owners}}))
    role = o.get("subjectRole")
    rse, rsi = o.get("roleScopingEntity"), o.get("roleScopingInstance")
    ras = []
    if role and rse and rsi:
        ras = [{"role": role, "attributes": [{"id": URN_RSE, "value": rse,
                                              "attributes": [{"id": URN_RSI, "value": rsi}]}]}]
    hrs = []
    if rsi and rse:
        hrs = [_drop_none({"id": "SuperOrg1", "role": role, "children": [
            {"id": "Org1", "children": [{"id": "Org2", "children": [{"id": "Org3"}]}]}]})]
    subject = _drop_none({"id": o.get("subjectID"), "role_associations": ras, "hierarchical_scopes": hrs})
    return {"target": {"subjects": subjects, "resources": resources, "actions": actions},
            "context": {"resources": ctx_res, "subject": subject}}
