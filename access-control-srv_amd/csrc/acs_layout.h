// acs_layout.h — packed, HBM-resident layout of the compiled policy store and of
// request batches for the MI355X access-control evaluator.
//
// Mirrors access-control-srv_amd/acs_mi355x/layout.py field for field (the host
// compiler/encoder writes these bytes).  Every string the reference compares
// (attribute ids/values, roles, scoping entities, owner/ACL instances, HR ids)
// is interned to a u32 id: equal ids <=> JS strict equality (===).  Two ids are
// reserved so that undefined and null stay distinct (loose == treats them equal).
#pragma once
#include <stdint.h>

#ifndef __HIPCC__  // plain C++ (g++) translation units: the host codec, compiler, validator
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace acs {

// ---------------------------------------------------------------- interned ids
constexpr uint32_t ID_UNDEF = 0;  // JS undefined (absent key)
constexpr uint32_t ID_NULL = 1;   // JS null
constexpr uint32_t ID_EMPTY = 2;  // the empty string '' (falsy); ids > ID_EMPTY are non-empty strings
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr uint8_t NONE8 = 0xFF;

// ---------------------------------------------------------------- effect codes
// Effect strings of rules/policies (rc-grpc-clients string enum + free strings).
enum EffectCode : uint8_t {
  EFF_UNDEF = 0, EFF_NULL = 1, EFF_PERMIT = 2, EFF_DENY = 3, EFF_NOT_APPLICABLE = 4,
  EFF_INDETERMINATE = 5, EFF_UNRECOGNIZED = 6,
  EFF_OTHER_TRUTHY = 7,  // any other non-empty string -> decision INDETERMINATE
  EFF_OTHER_FALSY = 8,   // '' / false / 0              -> decision INDETERMINATE
};
// Response_Decision codes written to the output (same numbering as effects).
enum DecisionCode : uint8_t {
  DEC_PERMIT = 2, DEC_DENY = 3, DEC_NOT_APPLICABLE = 4, DEC_INDETERMINATE = 5, DEC_UNRECOGNIZED = 6,
};
// evaluation_cacheable raw value codes; >= EC_OTHER0 index a host-side table.
enum EcCode : uint8_t { EC_UNDEF = 0, EC_NULL = 1, EC_FALSE = 2, EC_TRUE = 3, EC_OTHER0 = 4 };

// combining algorithm per policy / set, resolved against the URN->method config
enum CaCode : uint8_t { CA_INVALID = 0, CA_DENY_OVERRIDES = 1, CA_PERMIT_OVERRIDES = 2, CA_FIRST_APPLICABLE = 3 };

// ---------------------------------------------------------------- error kinds
enum ErrKind : uint8_t {
  ERR_NONE = 0,
  ERR_TYPE = 1,          // JS TypeError (e.g. nsEntityArray[0] of undefined, null policy)
  ERR_INVALID_CA = 2,    // errors.InvalidCombiningAlgorithm from decide()
  ERR_REGEX_SYNTAX = 3,  // new RegExp() SyntaxError
  ERR_REGEX_HOST = 4,    // pattern outside the precomputed subset -> host
};

// ---------------------------------------------------------------- attribute kinds
// Kind bits of a resource attribute id, precomputed against the URN config.
enum AttrKind : uint8_t {
  K_ENT = 1u << 0,       // id === urns.entity
  K_ENT_LOOSE = 1u << 1, // id ==  urns.entity
  K_OP = 1u << 2,        // id === urns.operation
  K_PROP = 1u << 3,      // id === urns.property
  K_RID_LOOSE = 1u << 4, // id ==  urns.resourceID
  K_OI = 1u << 5,        // (owner attr) id === urns.ownerInstance
  K_HAS_HASH = 1u << 6,  // value is a string containing '#'
};

// ---------------------------------------------------------------- tables (policy store)
enum TargetFlags : uint32_t {
  TF_SUBJ_EMPTY = 1u << 0,   // subjects.length === 0 -> checkSubjectMatches true
  TF_SUBJ_ROLE = 1u << 1,    // a truthy rule role: role-association membership
  TF_RES_EMPTY = 1u << 2,    // _.isEmpty(resources) -> resourceAttributesMatch true
  TF_RULE_PROPS = 1u << 3,   // some resources attr id === urns.property
  TF_HR_TRIVIAL = 1u << 4,   // checkHierarchicalScope returns true before reading context
  TF_HR_CHECK = 1u << 5,     // hierarchicalRoleScoping === 'true'
  TF_ACL_SKIP = 1u << 6,     // skipACL subject attribute present
  TF_HAS_SUBJECTS = 1u << 7, // subjects.length > 0 (policySubjectMatch gate)
  TF_LASTPROP_STR = 1u << 8, // last property value is a string
  TF_LASTPROP_HASH = 1u << 9,// ... containing '#'
  TF_RES_ENT_ONLY = 1u << 10,// non-empty resources without property / operation attrs:
                             // resourceAttributesMatch reduces to its entity test
};

// One set / policy / rule with its target inline (64 B: a single scalar load per node).
enum NodeFlags : uint8_t {
  NF_NULL = 1u << 0,           // null Map entry (policy: TypeError in loop 2a; rule: skipped)
  NF_HAS_TARGET = 1u << 1,     // !!node.target
  NF_EFFECT_TRUTHY = 1u << 2,  // !!node.effect
  NF_HAS_CONDITION = 1u << 3,  // rule.condition?.length
  NF_EC_TRUTHY = 1u << 4,      // !!rule.evaluation_cacheable
  NF_COND_FREE = 1u << 5,      // policy: no rule carries a condition; set: none of its policies'
                               // rules does and no policy has an invalid combining algorithm
                               // (absent: K1 never cuts the node's loop short)
  NF_CLEAN_BELOW = 1u << 6,    // set: every set before it is "clean" — NF_COND_FREE, a valid
                               // combining algorithm, no null policy — so nothing there can
                               // throw or reach a condition for a safe request (K1 walks the
                               // sets last to first and stops at the deciding one)
  NF_CLEAN = 1u << 7,          // set: itself clean (K1 skips it below the deciding set)
};

struct NodeRec {
  uint32_t tflags;           // TargetFlags of the inline target (0 without target)
  uint32_t role;             // last subjects value with id === urns.role (raw, may be UNDEF)
  uint32_t se;               // last roleScopingEntity value
  uint32_t subj_off;         // ATTRS mode: (id,value) pairs in the pair pool
  uint32_t act_off;          // (id,value) pairs in the pair pool
  uint32_t res_off;          // RuleResAttr pool
  uint32_t acl_roles_off;    // scopedRoles (role values in subject order) in the u32 pool
  uint32_t last_prop_value;  // value of the last property attr (whatIsAllowed mask source)
  uint16_t subj_n, act_n, res_n, acl_roles_n;
  uint32_t child_begin, child_end;  // set: its policies; policy: its rules
  uint32_t map_size;         // policy: combinables.size (null entries included)
  uint32_t fe;               // policy: first non-null rule with falsy evaluation_cacheable (else child_end)
  uint8_t effect, ec, ca, nflags;
  uint8_t pe_at;             // policy: loop-2a policyEffect after visiting this policy
  uint8_t pad[3];
};

struct Pair {                // (id, value) of a subject / action attribute, interned
  uint32_t id, value;
};

struct RuleResAttr {         // 16 B
  uint32_t value;
  uint32_t hash_sfx;         // id of value.substring(lastIndexOf('#')+1)  (K_PROP)
  uint16_t row;              // regex-matrix row of value                  (K_ENT_LOOSE)
  uint8_t kind;
  uint8_t pad;
  uint32_t pad2;
};

// ---------------------------------------------------------------- request batch
constexpr int QMAX = 16;     // resource attributes per request
constexpr int SMAX = 8;      // subject attributes
constexpr int AMAX = 4;      // action attributes
constexpr int RMAX = 8;      // role associations

enum ReqFlags : uint32_t {
  RQ_NO_TARGET = 1u << 0,    // !request.target
  RQ_HOST = 1u << 1,         // needs the host path (subject token I/O, unsupported shape)
  RQ_CTX_EMPTY = 1u << 2,    // _.isEmpty(request.context)
  RQ_RA_TRUTHY = 1u << 3,    // context.subject.role_associations truthy
  RQ_RA_EMPTY = 1u << 4,     // _.isEmpty(role_associations)
  RQ_SUBJ_MISSING = 1u << 5, // verifyACL: context.subject nullish -> TypeError
  RQ_HRS_ITERABLE = 1u << 6, // hierarchical_scopes is an array
  RQ_ANY_PROP = 1u << 7,     // some resource attr id === urns.property
  RQ_MULTI_ENT = 1u << 8,    // >1 resource attrs with id === urns.entity
  RQ_ACT_CREATE = 1u << 9,   // actions[0] is {actionID, create}
  RQ_ACT_RMD = 1u << 10,     // actions[0] is {actionID, read|modify|delete}
  RQ_ACL_SHIFT = 11,         // 2 bits: verifyACL request-loop outcome
  RQ_ENT_SHIFT = 13,         // 3 bits: 0 no entity attr, 1+j the only one at slot j (j < 6), 7 other
  RQ_PCOL_SHIFT = 16,        // 16 bits: candidate column of the request's entity attrs
};
constexpr uint32_t PCOL_ALL = 0xFFFF;  // several distinct entity columns / unfiltered request
// ACL_NONE: the loop continues (the resource has ACLs) but verifyACL is false for every rule —
// rule-independently (verifyACL.ts:89-251: no owner / grant instance matches an ACL instance, a
// `create` with an ACL entity no role association scopes, another action, no role associations)
// and without an error, so the kernel need not evaluate rules whose push it would veto.
enum AclState : uint32_t { ACL_CONTINUE = 0, ACL_RET_TRUE = 1, ACL_RET_FALSE = 2, ACL_NONE = 3 };
constexpr uint32_t HINT_ACL_NONE = 1u;  // acs_req_batch.hints: some request is ACL_NONE

struct ReqHdr {              // 16 B
  uint32_t flags;
  uint8_t nres, nsubj, nact, nroles;
  uint32_t arena_off;        // u32-word offset of this request's context arena
  uint32_t subject_id;       // context.subject.id
};

struct ReqRes {              // 16 B
  uint32_t value;
  uint32_t hash_sfx;         // K_PROP: id of the '#'-suffix
  uint16_t col;              // K_ENT_LOOSE: regex-matrix column of value
  uint16_t contains;         // K_PROP: bit i <=> value.indexOf(entityName(res[i].value)) > -1
  uint8_t kind;
  uint8_t slot_a;            // ctx resource via instance.id then id (NONE8: not found)
  uint8_t slot_b;            // ctx resource via id only (operation lookup)
  uint8_t pad;               // RES_RX_SAFE: no regex cell of this value's column throws or needs the host
};
constexpr uint32_t RES_RX_SAFE = 1;  // ReqRes.pad bit (absent: the request may throw in a RegExp test)

// One request's first rows packed into one 128-B line (acs_req_batch.lines): K1 reads it with
// one gather instead of one per SoA row (header, 4 attributes, 2 subjects, action, 2 roles,
// arena counts: ~8 lines per request).  res[j] / s* / a0 / r* are zero past the request's
// counts, ar0 / ar1 the arena's two count words (0 for RQ_HOST / RQ_NO_TARGET requests).
// The rows that do not fit (attributes 4.., subjects 2.., actions 1.., roles 2..) live in the
// request's extension record in acs_req_batch.ext (ReqLine.ext = 1 + its offset in 16-B
// units; 0 = none):
//   ReqRes res[LINE_RES..nres) | Pair subj[2..nsubj) | Pair act[1..nact) | u32 roles[2..nroles)
// padded to a multiple of 4 words.  A batch is either SoA rows (+ optional lines, equal to
// them) or compact: lines + ext only (hdr / res / subj / act / roles NULL), the form the
// native codec emits and the host-buffer entry points upload.  Built by both encoders
// (encoder.pack_lines, acs_codec.cpp) and checked by the host entry points.
constexpr int LINE_RES = 4, LINE_SUBJ = 2, LINE_ACT = 1, LINE_ROLES = 2;
struct ReqLine {             // 128 B
  ReqHdr h;
  ReqRes res[LINE_RES];
  Pair s0, s1, a0;
  uint32_t r0, r1;
  uint32_t ar0, ar1;
  uint32_t ext;              // 1 + 16-B unit offset of the extension record (0: none)
  uint32_t cls2;             // composed class rows: 1 + the request's second class (0: none), see below
};
// Composed class rows (candidates.py "composed" level): a request whose role associations name
// two roles some target requires carries the classes of (entity, action, role a) and (entity,
// action, role b); its filter is the OR of the two rows and its target verdicts are the OR of
// their known-true sections and the AND of their known-false sections.  Both rows are built with
// the role-relaxed useful sections that make the OR exact-or-wider (candidates.py).

// Extension record geometry (u32 words) of a request with the given counts.
struct ExtGeom {
  uint32_t res, subj, act, roles, words;  // word offsets of each part, total padded size
};
__host__ __device__ inline ExtGeom ext_geom(uint32_t nres, uint32_t nsubj, uint32_t nact, uint32_t nroles) {
  ExtGeom g;
  g.res = 0;
  g.subj = 4u * (nres > (uint32_t)LINE_RES ? nres - LINE_RES : 0u);
  g.act = g.subj + 2u * (nsubj > (uint32_t)LINE_SUBJ ? nsubj - LINE_SUBJ : 0u);
  g.roles = g.act + 2u * (nact > (uint32_t)LINE_ACT ? nact - LINE_ACT : 0u);
  const uint32_t end = g.roles + (nroles > (uint32_t)LINE_ROLES ? nroles - LINE_ROLES : 0u);
  g.words = (end + 3u) & ~3u;
  return g;
}

// Context arena (u32 words), per request:
//   [0] n_grants | n_rolese<<8 | n_slots<<16 | n_roots<<24
//   [1] n_tse | n_hrkeys<<8
//   grants  : n_grants x (role, se, inst)        roleScopingEntity/Instance triples
//   rolese  : n_rolese x (role, se)              role has a roleScopingEntity attr == se
//   roots   : n_roots  x raw root role           hierarchical_scopes[i].role
//   hrkeys  : n_hrkeys x effective role          verifyACL roleWithOrgScopesMap key order
//   slotoff : n_slots  x word offset (rel. to arena start) of the slot record
//   tse     : n_tse    x (se, n_inst, inst_rel_off) -> n_inst x (inst, eligible_key_mask)
// slot record: [owners_empty, n_owners, owner...]; owner: [is_oe | n_attrs<<8, value,
//   n_attrs x (value, kind(K_OI), root_mask)]
constexpr int MAX_ROOTS = 32, MAX_HRKEYS = 32, MAX_SLOTS = 254;

// ---------------------------------------------------------------- output
enum OutFlags : uint8_t {
  OF_ERR = 1u << 0,          // the reference rejects (aux = ErrKind)
  OF_HOST_COND = 1u << 1,    // a reached rule carries a JS condition (aux = rule index)
  OF_HOST_REQ = 1u << 2,     // request flagged RQ_HOST by the encoder
  OF_NO_TARGET = 1u << 3,    // status 400 response
  OF_HAS_EFFECT = 1u << 4,   // some policy set produced an effect
  OF_OBL_OVERFLOW = 1u << 5, // whatIsAllowed obligation log overflowed
};

struct Decision {            // 8 B
  uint8_t decision;          // DecisionCode
  uint8_t ec;                // EcCode of evaluation_cacheable
  uint8_t flags;             // OutFlags
  uint8_t err;               // ErrKind
  uint32_t aux;              // last applicable set index (+1; 0 = none) or rule index
};

constexpr int OBL_MAX = 128;  // whatIsAllowed maskedProperty push log entries per request (c4: 3 % of requests push > 64, far fewer > 128)

}  // namespace acs
