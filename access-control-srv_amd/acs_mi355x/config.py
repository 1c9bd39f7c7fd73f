"""The service's evaluator configuration: `policies.options` of the reference's
cfg/config.json:269-308 — the URN names every matcher compares against and the
combining-algorithm URN -> method table (AccessController's constructor reads both,
src/core/accessController.ts:51-67).

These are product inputs: the table compiler (compiler.compile_store / acs_store_compile)
and the request codec intern against them.  The oracle (oracle/acs_oracle.py) keeps its own
restatement of the same JSON as test infrastructure; tests/test_config.py checks the two agree.
"""

# cfg/config.json:272-293, policies.options.urns
SERVICE_URNS = {
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

# test/core.spec.ts:26-36: the reduced URN set the reference's PDP-level tests construct
# AccessController with (no property / maskedProperty / ACL / skipACL / action URNs, which
# changes matcher behaviour); the golden vectors of core.spec.ts are decided under it.
CORE_SPEC_URNS = {k: SERVICE_URNS[k] for k in (
    "roleScopingEntity", "roleScopingInstance", "hierarchicalRoleScoping", "ownerEntity",
    "ownerInstance", "resourceID", "entity", "role", "operation")}

CA_DENY_OVERRIDES = "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:deny-overrides"
CA_PERMIT_OVERRIDES = "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:permit-overrides"
CA_FIRST_APPLICABLE = "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:first-applicable"

# cfg/config.json:294-307, policies.options.combiningAlgorithms
COMBINING_ALGORITHMS = [
    {"urn": CA_DENY_OVERRIDES, "method": "denyOverrides"},
    {"urn": CA_PERMIT_OVERRIDES, "method": "permitOverrides"},
    {"urn": CA_FIRST_APPLICABLE, "method": "firstApplicable"},
]
