#!/usr/bin/env python3
"""Generate tests/golden/kats.json from the reference's own test suite.

Runs ONLY in the build container (it reads /root/reference, which the GPU box
does not have).  It extracts, for every ``it(...)`` block of

    test/core.spec.ts, test/properties.spec.ts, test/acl.spec.ts,
    test/microservice.spec.ts

that calls isAllowed / whatIsAllowed: the policy fixture in force, the
``buildRequest`` options (a plain JS object literal, read by the restricted
literal parser below — objects, arrays, strings, numbers, true / false / null /
undefined and comments, nothing else; no reference text is ever executed), the
request post-edits the test
makes, and the asserted outcome (decision / status, or the whatIsAllowed
structure assertions as path checks).  Each vector records its spec file:line.
The fixture YAMLs the vectors refer to are converted to JSON next to it.

Usage:  python tests/golden/extract_kats.py [/root/reference]
"""
from __future__ import annotations

import json
import os
import re
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from build_request import build_request  # noqa: E402

SPECS = ["core.spec.ts", "properties.spec.ts", "acl.spec.ts", "microservice.spec.ts"]


class LiteralError(ValueError):
    pass


_UNDEF = object()


def js_literal_to_json(text: str):
    """Value of a JS object / array / scalar literal, as JSON.stringify would give it
    (``undefined`` object members dropped, ``undefined`` array items -> null).  A restricted
    recursive-descent parser: anything but objects, arrays, quoted strings, numbers,
    true / false / null / undefined, trailing commas and comments raises LiteralError —
    the text comes from the reference's spec files and is never evaluated."""
    i, n = 0, len(text)

    def ws():
        nonlocal i
        while i < n:
            if text[i].isspace():
                i += 1
            elif text.startswith("//", i):
                j = text.find("\n", i)
                i = n if j < 0 else j + 1
            elif text.startswith("/*", i):
                j = text.find("*/", i + 2)
                if j < 0:
                    raise LiteralError("unterminated comment")
                i = j + 2
            else:
                return

    def string():
        nonlocal i
        q = text[i]
        i += 1
        out = []
        while i < n and text[i] != q:
            c = text[i]
            if c == "\\":
                i += 1
                if i >= n:
                    raise LiteralError("bad escape")
                e = text[i]
                simple = {"n": "\n", "t": "\t", "r": "\r", "b": "\b", "f": "\f", "v": "\v", "0": "\0"}
                if e in simple:
                    out.append(simple[e])
                elif e == "u":
                    out.append(chr(int(text[i + 1:i + 5], 16)))
                    i += 4
                elif e == "\n":
                    pass  # line continuation
                else:
                    out.append(e)
                i += 1
            else:
                out.append(c)
                i += 1
        if i >= n:
            raise LiteralError("unterminated string")
        i += 1
        return "".join(out)

    def ident():
        nonlocal i
        m = re.match(r"[A-Za-z_$][\w$]*", text[i:])
        if not m:
            raise LiteralError(f"unexpected {text[i:i + 20]!r}")
        i += m.end()
        return m.group(0)

    def value():
        nonlocal i
        ws()
        if i >= n:
            raise LiteralError("unexpected end")
        c = text[i]
        if c == "{":
            i += 1
            obj = {}
            while True:
                ws()
                if text[i] == "}":
                    i += 1
                    return obj
                key = string() if text[i] in "'\"" else ident()
                ws()
                if text[i] != ":":
                    raise LiteralError(f"expected ':' after {key!r}")
                i += 1
                v = value()
                if v is not _UNDEF:
                    obj[key] = v
                else:
                    obj.pop(key, None)
                ws()
                if text[i] == ",":
                    i += 1
                elif text[i] != "}":
                    raise LiteralError("expected ',' or '}'")
        if c == "[":
            i += 1
            arr = []
            while True:
                ws()
                if text[i] == "]":
                    i += 1
                    return arr
                v = value()
                arr.append(None if v is _UNDEF else v)
                ws()
                if text[i] == ",":
                    i += 1
                elif text[i] != "]":
                    raise LiteralError("expected ',' or ']'")
        if c in "'\"":
            return string()
        m = re.match(r"-?(\d+\.?\d*(e[+-]?\d+)?|\.\d+)", text[i:], re.I)
        if m:
            i += m.end()
            x = float(m.group(0))
            return int(x) if x.is_integer() else x
        word = ident()
        consts = {"true": True, "false": False, "null": None, "undefined": _UNDEF}
        if word not in consts:
            raise LiteralError(f"identifier {word!r} is not a literal")
        return consts[word]

    v = value()
    ws()
    if i != n:
        raise LiteralError(f"trailing text {text[i:i + 20]!r}")
    return None if v is _UNDEF else v


def matching_paren(src: str, i: int) -> int:
    """index of the ')' matching the '(' at src[i], skipping strings/comments."""
    depth = 0
    j = i
    n = len(src)
    while j < n:
        c = src[j]
        if c in "'\"`":
            q = c
            j += 1
            while j < n and src[j] != q:
                if src[j] == "\\":
                    j += 1
                j += 1
        elif src.startswith("//", j):
            j = src.index("\n", j)
        elif c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
            if depth == 0:
                return j
        j += 1
    raise ValueError("unbalanced")


PATH_TOKEN = re.compile(r"([A-Za-z_][A-Za-z_0-9]*)|\[(\d+)\]")


def parse_path(expr: str, aliases: dict):
    expr = expr.replace("!", "").replace("?", "")
    toks = []
    for m in PATH_TOKEN.finditer(expr):
        toks.append(m.group(1) if m.group(1) is not None else int(m.group(2)))
    if not toks:
        return None
    head = toks[0]
    if head in aliases:
        return aliases[head] + toks[1:]
    if head in ("result", "response"):
        return toks[1:]
    return None


ASSERT_LEN = re.compile(r"^\s*(.+?)\.should\.(?:be|have)\.length\((\d+)\)")
ASSERT_EQ = re.compile(r"^\s*(.+?)\.should\.equal\((.+)\);")
ASSERT_EXIST = re.compile(r"^\s*should\.exist\((.+)\);")
ASSERT_NOT_EXIST = re.compile(r"^\s*should\.not\.exist\((.+)\);")
ALIAS = re.compile(r"^\s*const (\w+) = (result[^;]+);")


def value_of(tok: str):
    tok = tok.strip()
    m = re.match(r"Response_Decision\.(\w+)", tok)
    if m:
        return m.group(1)
    return js_literal_to_json(tok)


def path_assertions(lines, aliases):
    out = []
    for ln in lines:
        m = ALIAS.match(ln)
        if m:
            aliases[m.group(1)] = parse_path(m.group(2), aliases)
            continue
        m = ASSERT_NOT_EXIST.match(ln)
        if m:
            p = parse_path(m.group(1), aliases)
            if p is not None:
                out.append([p, "not_exists", None])
            continue
        m = ASSERT_EXIST.match(ln)
        if m:
            p = parse_path(m.group(1), aliases)
            if p is not None:
                out.append([p, "exists", None])
            continue
        m = ASSERT_LEN.match(ln)
        if m:
            p = parse_path(m.group(1), aliases)
            if p is not None:
                out.append([p, "len", int(m.group(2))])
            continue
        m = ASSERT_EQ.match(ln)
        if m:
            p = parse_path(m.group(1), aliases)
            if p is not None and "operation_status" not in p[:1]:
                out.append([p, "eq", value_of(m.group(2))])
    return out


def helper_assertions(src: str, name: str, without_props: bool):
    """Inline a ``const name = (result, withoutProps?) => {...}`` validation helper."""
    i = src.index(f"const {name} = ")
    body_start = src.index("{", src.index("=>", i))
    body_end = matching_paren(src, body_start)
    body = src[body_start + 1:body_end]
    # keep the branch selected by withoutProps
    m = re.search(r"if \(withoutProps\) \{(.*?)\} else \{(.*?)\n  \}", body, re.S)
    if m:
        body = body[:m.start()] + (m.group(1) if without_props else m.group(2)) + body[m.end():]
    return path_assertions(body.splitlines(), {})


def extract(ref_root: str):
    vectors = []
    fixtures = set()
    for spec in SPECS:
        path = os.path.join(ref_root, "test", spec)
        src = open(path).read()
        for m in re.finditer(r"\n(\s*)it\((['\"])(.*?)\2,", src):
            start = m.start() + 1
            open_paren = src.index("(", start)
            end = matching_paren(src, open_paren)
            block = src[start:end]
            lineno = src.count("\n", 0, start) + 1
            if "isAllowed(" not in block and "whatIsAllowed(" not in block and "requestAndValidate(" not in block:
                continue
            # fixture in force: last prepare()/create() before this block
            fx = None
            for fm in re.finditer(r"(?:prepare|create)\('\./test/fixtures/([\w\-.]+)'\)", src[:start]):
                fx = fm.group(1)
            bi = block.find("buildRequest(")
            if bi < 0:
                continue
            bo = block.index("(", bi)
            be = matching_paren(block, bo)
            opts = js_literal_to_json(block[bo + 1:be])
            req = build_request(opts)
            edits = []
            hm = re.search(r"hierarchical_scopes = (\[.*?\]);", block)
            if hm:
                req["context"]["subject"]["hierarchical_scopes"] = js_literal_to_json(hm.group(1))
                edits.append("hierarchical_scopes")
            if re.search(r"(request|accessRequest)\.context = undefined;", block):
                grpc = "accessControlService" in block
                # gRPC path: AccessControlService.isAllowed maps an absent context to {} (accessControlService.ts:65)
                if grpc:
                    req["context"] = {}
                else:
                    del req["context"]
                edits.append("context_undefined")
            op = "whatIsAllowed" if "whatIsAllowed(" in block else "isAllowed"
            vec = {"name": m.group(3), "spec": f"test/{spec}:{lineno}", "fixture": fx,
                   "urns": "core" if spec == "core.spec.ts" else "full", "op": op,
                   "opts": opts, "edits": edits, "request": req}
            if op == "isAllowed":
                dm = re.findall(r"Response_Decision\.(\w+)", block)
                vec["expect"] = {"decision": dm[-1]}
                if "requestAndValidate(" in block:
                    if "requestAndValidate(ac, request, Response_Decision." in block and ", true)" not in block:
                        vec["expect"]["status"] = 200
                elif "operation_status!.code!.should.equal(200)" in block:
                    vec["expect"]["status"] = 200
            else:
                lines = block.splitlines()
                asserts = []
                hm2 = re.search(r"(validate\w+)\(result(?:, (true|false))?\)", block)
                if hm2:
                    asserts += helper_assertions(src, hm2.group(1), hm2.group(2) == "true")
                asserts += path_assertions(lines, {})
                vec["expect"] = {"asserts": asserts}
            vectors.append(vec)
            fixtures.add(fx)
    return vectors, sorted(f for f in fixtures if f)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    vectors, fixtures = extract(ref)
    fdir = os.path.join(HERE, "fixtures")
    os.makedirs(fdir, exist_ok=True)
    for fx in fixtures + ["policy_sets_with_targets.yml"]:
        doc = yaml.safe_load(open(os.path.join(ref, "test", "fixtures", fx)))
        with open(os.path.join(fdir, fx.replace(".yml", ".json")), "w") as f:
            json.dump(doc, f, indent=1)
    # seed data (data/seed_data/*.yaml): flat DB-shaped documents, stitched per resourceManager.load
    seed = {n: yaml.safe_load(open(os.path.join(ref, "data", "seed_data", n + ".yaml")))
            for n in ("policy_sets", "policies", "rules")}
    with open(os.path.join(fdir, "seed_data.json"), "w") as f:
        json.dump(seed, f, indent=1)
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump({"source": "restorecommerce/access-control-srv test suite", "vectors": vectors}, f, indent=1)
    n_ia = sum(v["op"] == "isAllowed" for v in vectors)
    print(f"{len(vectors)} vectors ({n_ia} isAllowed, {len(vectors) - n_ia} whatIsAllowed), fixtures: {fixtures}")


if __name__ == "__main__":
    main()
