#!/usr/bin/env python3
"""Extract Alink's parameter *API surface* (names, aliases, types, defaults, descriptions) and the
param interfaces each operator/stage implements, into a Python data table.

This is metadata extraction for API compatibility (PyAlink users call ``setK(3)`` etc.); no
reference logic is carried over.  Output: ``alink_amd/params/_spec.py``.

Usage: python tools/gen_param_spec.py /root/reference
"""
import os
import pprint
import re
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
JAVA = os.path.join(ROOT, "core/src/main/java")
OUT = os.path.join(os.path.dirname(__file__), "..", "alink_amd", "params", "_spec.py")


def strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    s = re.sub(r"//[^\n]*", "", s)
    return s


def java_files():
    for d, _, fs in os.walk(JAVA):
        for f in fs:
            if f.endswith(".java"):
                yield os.path.join(d, f)


PARAM_RE = re.compile(
    r"ParamInfo\s*<\s*(?P<jtype>[^=]+?)\s*>\s*(?P<const>\w+)\s*=\s*ParamInfoFactory\s*"
    r"\.\s*createParamInfo\s*\(\s*\"(?P<name>[^\"]+)\"\s*,\s*(?P<cls>[\w\.\[\]]+)\.class\s*\)"
    r"(?P<chain>.*?)\.\s*build\s*\(\s*\)\s*;", re.S)

ENUM_RE = re.compile(r"\benum\s+(\w+)\s*(?:implements[^{]*)?\{(.*?)(?:;|\})", re.S)


def parse_string_concat(expr):
    parts = re.findall(r'"((?:[^"\\]|\\.)*)"', expr)
    return "".join(bytes(p, "utf-8").decode("unicode_escape") if "\\" in p else p for p in parts)


def find_call_arg(chain, meth):
    i = chain.find("." + meth)
    if i < 0:
        i = chain.find(meth + "(")
        if i < 0:
            return None
    j = chain.find("(", i)
    depth = 0
    k = j
    in_str = False
    while k < len(chain):
        c = chain[k]
        if in_str:
            if c == "\\":
                k += 2
                continue
            if c == '"':
                in_str = False
        else:
            if c == "'":
                k = chain.index("'", k + 2 if chain[k + 1] == "\\" else k + 1) + 1
                continue
            if c == '"':
                in_str = True
            elif c == "(":
                depth += 1
            elif c == ")":
                depth -= 1
                if depth == 0:
                    return chain[j + 1:k].strip()
        k += 1
    return None


def parse_default(expr, jcls):
    e = expr.strip()
    if e == "null":
        return None
    if e in ("true", "Boolean.TRUE"):
        return True
    if e in ("false", "Boolean.FALSE"):
        return False
    if e == "Integer.MAX_VALUE":
        return 2147483647
    if e == "Integer.MIN_VALUE":
        return -2147483648
    if e == "Double.MAX_VALUE":
        return 1.7976931348623157e308
    if e == "Long.MAX_VALUE":
        return 9223372036854775807
    if e == "1 << 18":
        return 1 << 18
    if e == "MLEnvironmentFactory.DEFAULT_ML_ENVIRONMENT_ID":
        return 0
    if e.startswith('"'):
        return parse_string_concat(e)
    if e.startswith("'"):
        return e[1:-1].encode().decode("unicode_escape")
    if e.startswith("new String[0]"):
        return []
    m = re.match(r"new\s+(\w+)\s*\[\s*\]\s*\{(.*)\}", e, re.S)
    if m:
        items = [x.strip() for x in m.group(2).split(",") if x.strip()]
        return [parse_default(x, m.group(1)) for x in items]
    m = re.match(r"^-?\d+L$", e)
    if m:
        return int(e[:-1])
    try:
        if re.match(r"^-?\d+$", e):
            return float(e) if jcls in ("Double", "double", "Float") else int(e)
        return float(e.rstrip("dDfF"))
    except ValueError:
        pass
    # enum constant  X.Y or A.X.Y
    if re.match(r"^[\w\.]+$", e):
        return {"__enum__": e.split(".")[-1]}
    return {"__expr__": e}


def main():
    interfaces = {}
    enums = {}           # qualified "Iface.Enum" and simple "Enum" -> members
    ops = {}
    for path in java_files():
        src = strip_comments(open(path, encoding="utf-8", errors="replace").read())
        fname = os.path.basename(path)[:-5]
        # enums
        for m in ENUM_RE.finditer(src):
            body = m.group(2)
            members = []
            for tok in re.split(r",(?![^()]*\))", body):
                tok = tok.strip()
                mm = re.match(r"^([A-Za-z_]\w*)", tok)
                if mm and tok and not tok.startswith(("private", "public", "final")):
                    members.append(mm.group(1))
            if members:
                # the simple name belongs to a top-level enum (its own file) over a nested one of the same name
                # (nlp FeatureType vs FeatureMeta.FeatureType)
                if fname == m.group(1):
                    enums[m.group(1)] = members
                else:
                    enums.setdefault(m.group(1), members)
                enums[fname + "." + m.group(1)] = members
        # interfaces
        im = re.search(r"public\s+interface\s+(\w+)\s*(?:<[^{]*?>)?\s*(?:extends\s+([^{]*))?\{", src)
        has_pi = "ParamInfoFactory" in src
        if (im and ("/params/" in path or has_pi)) or (has_pi and not im):
            if not im:
                im = re.search(r"(?:class|interface)\s+(\w+)\s*(?:<[^{]*?>)?()", src)
            extends = []
            if im.group(2):
                ext = re.sub(r"<[^<>]*(<[^<>]*>[^<>]*)*>", "", im.group(2))
                extends = [x.strip().split(".")[-1] for x in ext.split(",") if x.strip()]
                extends = [x for x in extends if x not in ("WithParams", "Serializable")]
            params = []
            for pm in PARAM_RE.finditer(src):
                chain = pm.group("chain")
                desc = find_call_arg(chain, "setDescription")
                alias = find_call_arg(chain, "setAlias")
                dflt = find_call_arg(chain, "setHasDefaultValue")
                jcls = pm.group("cls").split(".")[-1]
                entry = {
                    "const": pm.group("const"), "name": pm.group("name"), "jtype": jcls,
                    "desc": parse_string_concat(desc) if desc else "",
                    "alias": re.findall(r'"([^"]*)"', alias) if alias else [],
                    "required": ".setRequired()" in re.sub(r"\s", "", chain),
                    "has_default": dflt is not None,
                    "default": parse_default(dflt, jcls) if dflt is not None else None,
                }
                if entry["has_default"]:
                    entry["required"] = False
                params.append(entry)
            interfaces[im.group(1)] = {"extends": extends, "params": params, "file": fname}
        # operator / stage classes
        cm = re.search(r"public\s+(?:final\s+)?(?:abstract\s+)?class\s+(\w+)\s*(?:<[^{]*?>)?\s*"
                       r"(?:extends\s+([\w\.]+)\s*(?:<[^{]*?>)?)?\s*(?:implements\s+([^{]*))?\{", src)
        if cm and ("/operator/" in path or "/pipeline/" in path):
            impl = []
            if cm.group(3):
                s = re.sub(r"<[^<>]*(<[^<>]*>[^<>]*)*>", "", cm.group(3))
                impl = [x.strip().split(".")[-1] for x in s.split(",") if x.strip()]
            ops[cm.group(1)] = {"extends": (cm.group(2) or "").split(".")[-1], "implements": impl,
                                "path": os.path.relpath(path, ROOT)}
    with open(OUT, "w") as f:
        f.write('"""GENERATED by tools/gen_param_spec.py from the reference API surface (names, aliases,\n'
                'defaults, descriptions of every param interface; operator -> param interfaces).\n'
                'Do not edit by hand."""\n\n')
        f.write("INTERFACES = ")
        f.write(pprint.pformat(interfaces, width=110, sort_dicts=True))
        f.write("\n\nENUMS = ")
        f.write(pprint.pformat(enums, width=110, sort_dicts=True))
        f.write("\n\nOPS = ")
        f.write(pprint.pformat(ops, width=110, sort_dicts=True))
        f.write("\n")
    print(f"interfaces={len(interfaces)} params={sum(len(v['params']) for v in interfaces.values())} "
          f"enums={len(enums)} ops={len(ops)}")


if __name__ == "__main__":
    main()
