#!/usr/bin/env node
// gen_regex_cells.js — V8 ground truth for the entity namespace / RegExp test.
//
// TEST INFRASTRUCTURE.  Writes tests/golden/regex_cells.json: for every (rule entity value,
// request entity value) pair of the vocabulary below, the outcome of one step of the
// reference's RegExp-mode entity test, evaluated by this Node's own RegExp engine:
//
//   src/core/accessController.ts:528-566   (resourceAttributesMatch, regexMatch branch)
//   src/core/hierarchicalScope.ts:64-101   (checkHierarchicalScope, same test, `==` forms)
//
// Bits (csrc/acs_eval.h RxBits): 1 HIT (entityMatch set), 2 RESET (namespace prefix differs:
// entityMatch cleared first), 4 THROW_TYPE (nsEntityArray[0] of undefined), 8 THROW_SYNTAX
// (new RegExp throws).  The step below is this file's own restatement of those lines; it
// reads no reference file.  Usage:  node tests/golden/gen_regex_cells.js > tests/golden/regex_cells.json
'use strict';

const RX_HIT = 1, RX_RESET = 2, RX_THROW_TYPE = 4, RX_THROW_SYNTAX = 8;

function cell(ruleValue, reqValue) {
  let bits = 0;
  try {
    const pattern = ruleValue == null ? undefined : ruleValue.substring(ruleValue.lastIndexOf(':') + 1);
    const nsEntityArray = pattern == null ? undefined : pattern.split('.');
    const nsOrEntity = nsEntityArray[0];  // TypeError when the rule value is nullish
    const entityRegexValue = nsEntityArray[nsEntityArray.length - 1];
    let reqNS, ruleNS;
    if ((nsOrEntity == null ? undefined : nsOrEntity.toUpperCase()) !=
        (entityRegexValue == null ? undefined : entityRegexValue.toUpperCase())) {
      ruleNS = nsOrEntity.toUpperCase();
    }
    const reqValue2 = reqValue;
    const reqAttributeNS = reqValue2 == null ? undefined : reqValue2.substring(0, reqValue2.lastIndexOf(':'));
    const ruleAttributeNS = ruleValue == null ? undefined : ruleValue.substring(0, ruleValue.lastIndexOf(':'));
    if (reqAttributeNS != ruleAttributeNS) bits |= RX_RESET;
    const reqPattern = reqValue2 == null ? undefined : reqValue2.substring(reqValue2.lastIndexOf(':') + 1);
    const reqNSEntityArray = reqPattern == null ? undefined : reqPattern.split('.');
    const reqNSOrEntity = reqNSEntityArray[0];  // TypeError when the request value is nullish
    const requestEntityValue = reqNSEntityArray[reqNSEntityArray.length - 1];
    if ((reqNSOrEntity == null ? undefined : reqNSOrEntity.toUpperCase()) !=
        (requestEntityValue == null ? undefined : requestEntityValue.toUpperCase())) {
      reqNS = reqNSOrEntity.toUpperCase();
    }
    if ((reqNS && ruleNS && (reqNS === ruleNS)) || (!reqNS && !ruleNS)) {
      const reExp = new RegExp(entityRegexValue);
      if (requestEntityValue.match(reExp)) bits |= RX_HIT;
    }
  } catch (e) {
    if (e instanceof SyntaxError) return RX_THROW_SYNTAX;
    if (e instanceof TypeError) return RX_THROW_TYPE;
    throw e;
  }
  return bits;
}

// ---------------------------------------------------------------- vocabulary
// Rule entity patterns (the last dot segment after the last ':') — literals with shared
// prefixes (Ent1 in Ent12), anchors (V8's `$` is end of input only; a trailing '\n' in the
// subject must NOT match), alternation, groups, classes, quantifiers (greedy / lazy),
// malformed patterns (SyntaxError) and patterns outside any restated subset (escapes,
// braces, '/', non-ASCII) that the evaluator sends to the host.
const patterns = [
  'Ent1', 'Ent12', 'Ent', 'ent1', 'nt1', '1', '', 'Ent1 ', 'Ent 1', "Ent'1", 'Ent-1', 'Ent_1', 'Ent#1', 'Ent@1',
  'Ent1$', '^Ent1', '^Ent1$', '$', '^', '^$', 'Ent1$|Ent2', '^Ent(1|2)$', 'Ent(1|2)', '(Ent)?1$', 'Ent1|',
  '|', '()', '(Ent1)', 'Ent[0-9]', 'Ent[0-9]+$', 'Ent[12]$', 'Ent[^1]', '[A-Z]nt1', '[a-z]nt1', '[A-z]nt',
  '[-1]', '[1-]', 'E*nt1', 'En+t1', 'Ent1?$', 'Ent1+', 'Ent1*?$', 'Ent1+?', 'Ent1??', 'Ent1*', '^E.*',
  'Ent1**', 'Ent1*+', '*Ent', '+', '?', 'Ent(', 'Ent)', 'Ent[', 'Ent]', '(Ent', '[]', '[^]', 'a[]b', '^*',
  '$*', '(^)*Ent1', '(?:Ent1)', '(?=E)Ent1', 'Ent\\d', 'Ent\\n', 'Ent{1}', 'Ent1{', 'Ent1}', 'Ent/1',
  'Ént1', 'Ent1\n', '\nEnt1', 'Ent1$\n', 'Ent12$', 'Ent1(2)?$', '^Ent1[0-9]*$', 'Ent[[]', 'Ent1|^Ent2$',
  'nt1$', 'ENT1', 'Ent1 ', 'Ent1\t',
];
// Namespace / prefix variants of the rule value around each pattern.
const rulePrefixes = ['urn:x:model:ent.', 'urn:x:model:', 'urn:y:model:ent.', 'urn:x:model:ns.ent.'];
const requestValues = [
  'urn:x:model:ent.Ent1', 'urn:x:model:ent.Ent12', 'urn:x:model:ent.Ent2', 'urn:x:model:ent.Ent1\n',
  'urn:x:model:ent.Ent1\nfoo', 'urn:x:model:ent.\nEnt1', 'urn:x:model:ent.ent1', 'urn:x:model:ent.ENT1',
  'urn:x:model:ent.XEnt1', 'urn:x:model:ent.Ent', 'urn:x:model:ent.', 'urn:x:model:Ent1', 'urn:x:model:Ent12',
  'urn:x:model:Ent1\n', 'urn:x:model:ns.ent.Ent1', 'urn:y:model:ent.Ent1', 'urn:x:model:ENT.Ent1',
  'urn:x:model:other.Ent1', 'Ent1', 'ent.Ent1', 'urn:x:model:ent.Ent 1', 'urn:x:model:ent.Ent1 ',
  'urn:x:model:ent.Ent-1', 'urn:x:model:ent.E', 'urn:x:model:ent.Ént1', 'urn:x:model:ent.Ent1 ',
  'urn:x:model:ent.Ent1\t', 'urn:x:model:ent.Ent#1', 'urn:x:model:ent.1', 'urn:x:model:ent.Ent[1',
];

const pairs = [];
for (const p of patterns) {
  for (const pre of rulePrefixes) {
    const rv = pre + p;
    for (const q of requestValues) pairs.push([rv, q, cell(rv, q)]);
  }
}
// Seeded random patterns over the metacharacter subset the evaluator computes itself
// (letters, digits, '-', '_', '|', '(', ')', '[', ']', '^', '$', '*', '+', '?'): V8 decides
// both which of them are SyntaxErrors and what they match.
let seed = 0xACC5;
const rnd = (k) => { seed = (seed * 1103515245 + 12345) & 0x7fffffff; return seed % k; };
const alphabet = ['E', 'n', 't', '1', '2', '-', '_', '|', '(', ')', '[', ']', '^', '$', '*', '+', '?'];
const fuzzSubjects = ['urn:x:model:ent.Ent1', 'urn:x:model:ent.Ent12', 'urn:x:model:ent.Ent1\n', 'urn:x:model:ent.nt',
                      'urn:x:model:ent.E-1', 'urn:x:model:ent.', 'urn:x:model:ent.t2t'];
const seen = new Set();
while (seen.size < 1500) {
  let p = '';
  const len = 1 + rnd(7);
  for (let k = 0; k < len; ++k) p += alphabet[rnd(alphabet.length)];
  if (seen.has(p)) continue;
  seen.add(p);
  const rv = 'urn:x:model:ent.' + p;
  for (const q of fuzzSubjects) pairs.push([rv, q, cell(rv, q)]);
}
// nullish operands (JSON null): the TypeError cells
for (const q of ['urn:x:model:ent.Ent1', null]) pairs.push([null, q, cell(null, q)]);
pairs.push(['urn:x:model:ent.Ent1', null, cell('urn:x:model:ent.Ent1', null)]);

process.stdout.write(JSON.stringify({
  generator: 'tests/golden/gen_regex_cells.js',
  node: process.version,
  v8: process.versions.v8,
  bits: {HIT: RX_HIT, RESET: RX_RESET, THROW_TYPE: RX_THROW_TYPE, THROW_SYNTAX: RX_THROW_SYNTAX},
  pairs,
}) + '\n');
