#!/usr/bin/env python3
"""Type-eraser: the reference merge-tree TypeScript -> Node-12 CommonJS
(TEST INFRASTRUCTURE, SURVEY.md §8(c) "optional true oracle").

There is no TypeScript compiler in this image and Node 12 rejects `?.` / `??`
(SURVEY.md §0 fact 3), so this script does the mechanical part of `tsc
--target es2017 --module commonjs` for the subset of TypeScript the
packages/dds/merge-tree sources use: it removes type annotations, interfaces,
type aliases, generics, casts, non-null assertions, access modifiers and
overload signatures, turns enums into objects, parameter properties into
constructor assignments, ES imports / exports into CommonJS, and downlevels
`?.`, `??` and `??=`.

Output goes to oracle/_ref/ts/ (git-ignored and gpurun-ignored: the reference
never enters the repository's history and never travels to the GPU box).  Only
its *outputs* (golden vectors under tests/golden/) are committed.  The
modules outside merge-tree whose values the sources use are erased from the
reference too, into oracle/_ref/ts/node_modules/@fluidframework/<package>/
(EXTERNAL below): common-utils assert / Trace / unreachableCase,
protocol-definitions MessageType, container-definitions AttachState.
oracle/ref_stubs.js supplies only what cannot be erased here:
the telemetry loggers, the error classes of telemetry-utils / container-utils
(whose module needs the third-party `uuid`, absent offline; they are raised
only on failure paths) and runtime-utils' SummaryTreeBuilder (needs
protocol-base) and common-utils' bufferToString (bufferNode.ts declares an
ambient Buffer class this eraser does not handle); neither is on a path the
oracle runs (summary emit / load).  Packages imported for types only
become empty modules.

Usage: python3 oracle/ts_erase.py [--src DIR] [--out DIR]
"""
import argparse
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_SRC = "/root/reference/packages/dds/merge-tree/src"
DEFAULT_OUT = os.path.join(HERE, "_ref", "ts")
REF_ROOT = "/root/reference"

# package -> (module name, reference source file) erased into
# node_modules/@fluidframework/<package>/<module>.js, plus the package's
# index.js re-exporting them (the reference package's own index re-exports the
# same names).  trace.ts imports { performance } from "./indexNode", which the
# reference wires to performanceNode.ts.
EXTERNAL = {
    "common-utils": [("assert", "common/lib/common-utils/src/assert.ts"),
                     ("trace", "common/lib/common-utils/src/trace.ts"),
                     ("typedEventEmitter", "common/lib/common-utils/src/typedEventEmitter.ts"),
                     ("unreachable", "common/lib/common-utils/src/unreachable.ts"),
                     ("performanceNode", "common/lib/common-utils/src/performanceNode.ts")],
    "protocol-definitions": [("protocol", "common/lib/protocol-definitions/src/protocol.ts")],
    "container-definitions": [("runtime", "packages/common/container-definitions/src/runtime.ts")],
}
INDEX_ALIASES = {"common-utils": {"indexNode": "performanceNode"}}
STUBBED = ("telemetry-utils", "container-utils", "runtime-utils")  # oracle/ref_stubs.js
STUB_EXTRA = ("common-utils",)  # + bufferToString from oracle/ref_stubs.js
# the sequence package's interval collection over the erased merge-tree
# (oracle/ref_interval_farm.js): erased into <out>/sequence/, with
# @fluidframework/merge-tree resolving to the erased merge-tree itself.  Its
# only third-party import, uuid, makes the ids of intervals added without one;
# the farm always passes ids, and node_modules/uuid throws if it is ever called.
SEQUENCE_SRC = "packages/dds/sequence/src"
SEQUENCE_FILES = ("intervalCollection.ts", "intervalTree.ts")
TYPE_ONLY = ("core-interfaces", "shared-object-base", "datastore-definitions", "runtime-definitions",
             "common-definitions", "driver-definitions")

PUNCTS = sorted("""
>>>= ... === !== **= <<= >>= >>> ??= ?. ?? => == != <= >= && || ++ -- += -= *= /= %= &= |= ^= << >> ** &&= ||=
{ } ( ) [ ] ; , < > + - * / % & | ^ ! ~ ? : = . @ #
""".split(), key=len, reverse=True)

KEYWORDS_BEFORE_PAREN = {"if", "for", "while", "switch", "catch", "with", "return", "typeof", "await", "yield",
                         "delete", "void", "in", "of", "new", "case", "throw", "else", "do", "instanceof"}
MODIFIERS = {"public", "private", "protected", "readonly", "abstract", "override", "declare"}
EXPR_END = {"id", "num", "str", "tmpl", "regex"}


class Tok:
    __slots__ = ("kind", "text", "ws", "drop", "pre", "post")

    def __init__(self, kind, text, ws):
        self.kind, self.text, self.ws = kind, text, ws
        self.drop = False
        self.pre = ""   # text inserted before the token
        self.post = ""  # text inserted after the token

    def __repr__(self):
        return f"{self.kind}:{self.text!r}"


# ---------------------------------------------------------------------------
# tokenizer
# ---------------------------------------------------------------------------
def tokenize(src):
    toks, i, n, ws = [], 0, len(src), ""
    while i < n:
        c = src[i]
        if c in " \t\r\n":
            j = i
            while j < n and src[j] in " \t\r\n":
                j += 1
            ws += src[i:j]
            i = j
            continue
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            ws += src[i:j]
            i = j
            continue
        if src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            ws += src[i:j]
            i = j
            continue
        if c.isalpha() or c in "_$":
            j = i + 1
            while j < n and (src[j].isalnum() or src[j] in "_$"):
                j += 1
            toks.append(Tok("id", src[i:j], ws))
            ws, i = "", j
            continue
        if c.isdigit() or (c == "." and i + 1 < n and src[i + 1].isdigit()):
            m = re.compile(r"0[xXbBoO][0-9a-fA-F_]+n?|(\d[\d_]*\.?[\d_]*|\.\d[\d_]*)([eE][+-]?\d+)?n?").match(src, i)
            toks.append(Tok("num", m.group(0), ws))
            ws, i = "", m.end()
            continue
        if c in "'\"":
            j = i + 1
            while src[j] != c:
                j += 2 if src[j] == "\\" else 1
            toks.append(Tok("str", src[i:j + 1], ws))
            ws, i = "", j + 1
            continue
        if c == "`":
            j, depth = i + 1, 0
            while True:
                if src[j] == "\\":
                    j += 2
                    continue
                if depth == 0 and src[j] == "`":
                    break
                if src.startswith("${", j):
                    depth += 1
                    j += 2
                    continue
                if depth and src[j] == "{":
                    depth += 1
                elif depth and src[j] == "}":
                    depth -= 1
                j += 1
            toks.append(Tok("tmpl", src[i:j + 1], ws))
            ws, i = "", j + 1
            continue
        if c == "/" and _regex_allowed(toks):
            j, cls = i + 1, False
            while True:
                if src[j] == "\\":
                    j += 2
                    continue
                if src[j] == "[":
                    cls = True
                elif src[j] == "]":
                    cls = False
                elif src[j] == "/" and not cls:
                    break
                j += 1
            j += 1
            while j < n and src[j].isalpha():
                j += 1
            toks.append(Tok("regex", src[i:j], ws))
            ws, i = "", j
            continue
        for p in PUNCTS:
            if src.startswith(p, i):
                if p == "?." and i + 2 < n and src[i + 2].isdigit():
                    continue
                toks.append(Tok("p", p, ws))
                ws, i = "", i + len(p)
                break
        else:
            raise SyntaxError(f"unexpected {c!r} at {i}")
    toks.append(Tok("eof", "", ws))
    return toks


def _regex_allowed(toks):
    if not toks:
        return True
    t = toks[-1]
    if t.kind in ("num", "str", "tmpl", "regex"):
        return False
    if t.kind == "id":
        return t.text in ("return", "typeof", "case", "do", "else", "in", "of", "new", "delete", "void", "throw")
    return t.text not in (")", "]", "}")


# ---------------------------------------------------------------------------
# helpers over the token list
# ---------------------------------------------------------------------------
class Src:
    def __init__(self, toks):
        self.t = toks
        self.match = {}
        stack = []
        for i, tk in enumerate(toks):
            if tk.kind != "p":
                continue
            if tk.text in "([{":
                stack.append(i)
            elif tk.text in ")]}":
                j = stack.pop()
                self.match[i] = j
                self.match[j] = i

    def nxt(self, i):
        """index of the next non-dropped token after i"""
        i += 1
        while self.t[i].drop and self.t[i].kind != "eof":
            i += 1
        return i

    def prv(self, i):
        i -= 1
        while i >= 0 and self.t[i].drop:
            i -= 1
        return i

    def is_p(self, i, *texts):
        return 0 <= i < len(self.t) and self.t[i].kind == "p" and self.t[i].text in texts

    def is_id(self, i, *texts):
        return 0 <= i < len(self.t) and self.t[i].kind == "id" and (not texts or self.t[i].text in texts)

    def drop(self, a, b):
        """drop tokens [a, b)"""
        for k in range(a, b):
            self.t[k].drop = True

    # -- types -----------------------------------------------------------------
    def skip_type(self, i, stop_arrow=False, brace_ends=False):
        """i = first token of a type; returns the index just past it.
        stop_arrow: a top-level `=>` ends the type (arrow return types).
        brace_ends: a `{` after a complete type ends it (function bodies)."""
        t = self.t
        depth = 0
        start = i
        prev_complete = False
        while True:
            tk = t[i]
            if tk.kind == "eof":
                return i
            x = tk.text if tk.kind == "p" else None
            if depth == 0:
                if x in (",", ")", "]", "}", ";", "=", "?.", "??", "&&", "||") and not (x == "=" and False):
                    return i
                if x == "=>" and (stop_arrow or not (i > start and t[i - 1].text == ")")):
                    if stop_arrow:
                        return i
                if x == "{" and brace_ends and prev_complete:
                    return i
                if x == ">" or x == ">>" or x == ">>>" or x == ">=":
                    return i
                if tk.kind == "id" and tk.text in ("implements",) and i > start:
                    return i
                if x == ":" or (x == "?" and prev_complete and not _cond_type(t, i)):
                    return i
            if x in ("(", "[", "{"):
                i = self.match[i] + 1
                prev_complete = True
                continue
            if x == "<":
                depth += 1
            elif x == ">":
                depth -= 1
            elif x == ">>":
                depth -= 2
            elif x == ">>>":
                depth -= 3
            if depth < 0:
                return i
            prev_complete = tk.kind in ("id", "num", "str") or x in (">", ">>", ">>>")
            if tk.kind == "id" and tk.text in ("keyof", "typeof", "readonly", "extends", "is", "infer", "new"):
                prev_complete = False
            if x in ("|", "&", "=>", ".", ",", "?", ":"):
                prev_complete = False
            i += 1

    def angle_end(self, i):
        """i at `<` in a position that can only hold type parameters: index past
        the matching `>`"""
        t = self.t
        depth, j = 0, i
        while True:
            x = t[j].text if t[j].kind == "p" else None
            if x in ("(", "[", "{"):
                j = self.match[j] + 1
                continue
            if x == "<":
                depth += 1
            elif x in (">", ">>", ">>>"):
                depth -= len(x)
                if depth <= 0:
                    return j + 1
            elif x == "=>" or x == ">=":
                pass
            j += 1

    def generic_end(self, i):
        """i at `<`: index past the matching `>` when the group looks like type
        arguments / parameters, else None"""
        t = self.t
        depth, j = 0, i
        while True:
            tk = t[j]
            if tk.kind == "eof":
                return None
            x = tk.text if tk.kind == "p" else None
            if x == "<":
                depth += 1
            elif x in (">", ">>", ">>>"):
                depth -= len(x)
                if depth <= 0:
                    return j + 1 if depth == 0 else None
            elif x in ("(", "[", "{"):
                j = self.match[j] + 1
                continue
            elif x in (";", "&&", "||", "+", "-", "*", "/", "%", "==", "===", "!=", "!==", "<=", ">=", "!", ")", "]",
                       "}", "=", "+=", "-="):
                return None
            elif tk.kind == "num":
                return None
            j += 1


def _cond_type(t, i):
    return False


# ---------------------------------------------------------------------------
# the eraser
# ---------------------------------------------------------------------------
class Eraser:
    def __init__(self, src_text, name):
        self.name = name
        self.s = Src(tokenize(src_text))
        self.t = self.s.t
        self.exports_hoisted = []   # function exports (hoisted)
        self.imports = {}           # local name -> (module var, imported name or None for namespace)
        self.modvars = {}           # module path -> var name
        self.reexports = []         # js lines
        self.class_bodies = set()
        self.params = {}            # `(` index -> is constructor params
        self.member_names = set()   # class-member / object-method name tokens (never import refs)

    # -- pass 1: imports / exports / declarations ------------------------------
    def stmt_start(self, i):
        p = self.s.prv(i)
        return p < 0 or self.s.is_p(p, ";", "}", "{") or self.s.is_id(p, "export", "declare")

    def modvar(self, path):
        if path not in self.modvars:
            base = re.sub(r"\W", "_", path.strip("'\"").split("/")[-1])
            self.modvars[path] = f"__m_{base}_{len(self.modvars)}"
        return self.modvars[path]

    def pass_modules(self):
        s, t = self.s, self.t
        i = 0
        while t[i].kind != "eof":
            tk = t[i]
            if tk.kind == "id" and tk.text == "import" and self.stmt_start(i) and not s.is_p(i + 1, "("):
                # import ... from "x";   import "x";
                j = i + 1
                if t[j].kind == "str":
                    end = j + 1 + (1 if s.is_p(j + 1, ";") else 0)
                    t[i].pre = f"require({t[j].text});"
                    s.drop(i, end)
                    i = end
                    continue
                while not (t[j].kind == "id" and t[j].text == "from"):
                    j += 1
                path = t[j + 1].text
                mv = self.modvar(path)
                k = i + 1
                if s.is_id(k, "type"):
                    k += 1
                while k < j:
                    if s.is_p(k, "*"):
                        self.imports[t[k + 2].text] = (mv, None)
                        k += 3
                    elif s.is_p(k, "{"):
                        e = s.match[k]
                        m = k + 1
                        while m < e:
                            if s.is_p(m, ","):
                                m += 1
                                continue
                            name = t[m].text
                            local = name
                            if s.is_id(m + 1, "as"):
                                local = t[m + 2].text
                                m += 3
                            else:
                                m += 1
                            self.imports[local] = (mv, name)
                        k = e + 1
                    elif t[k].kind == "id":
                        self.imports[t[k].text] = (mv, "default")
                        k += 1
                    else:
                        k += 1
                end = j + 2 + (1 if s.is_p(j + 2, ";") else 0)
                s.drop(i, end)
                i = end
                continue
            if tk.kind == "id" and tk.text == "export" and self.stmt_start(i):
                j = i + 1
                if s.is_p(j, "*"):
                    # export * from "x";
                    path = t[j + 2].text
                    self.reexports.append(f"__exportStar(require({path}));")
                    end = j + 3 + (1 if s.is_p(j + 3, ";") else 0)
                    s.drop(i, end)
                    i = end
                    continue
                if s.is_p(j, "{"):
                    e = s.match[j]
                    names = []
                    m = j + 1
                    while m < e:
                        if s.is_p(m, ","):
                            m += 1
                            continue
                        if s.is_id(m, "type"):
                            m += 1
                        name = t[m].text
                        alias = name
                        if s.is_id(m + 1, "as"):
                            alias = t[m + 2].text
                            m += 3
                        else:
                            m += 1
                        names.append((name, alias))
                    k = e + 1
                    if s.is_id(k, "from"):
                        path = t[k + 1].text
                        for name, alias in names:
                            self.reexports.append(
                                f"Object.defineProperty(exports, {alias!r}, {{enumerable: true, get: function () "
                                f"{{ return require({path})[{name!r}]; }}}});")
                        k += 2
                        end = k + (1 if s.is_p(k, ";") else 0)
                        s.drop(i, end)
                    else:
                        end = k + (1 if s.is_p(k, ";") else 0)
                        s.drop(i, end)
                        t[end - 1].post += "".join(
                            f" Object.defineProperty(exports, {alias!r}, {{enumerable: true, get: function () "
                            f"{{ return {name}; }}}});" for name, alias in names)
                    i = end
                    continue
                if s.is_id(j, "default"):
                    raise SyntaxError(f"{self.name}: export default")
                # export <declaration>
                t[i].drop = True
                k = j
                while s.is_id(k, "abstract", "declare", "async"):
                    k += 1
                kw = t[k].text
                if kw in ("interface", "type"):
                    i = j
                    continue
                if kw == "function":
                    name = t[k + 1].text if t[k + 1].kind == "id" else t[k + 2].text
                    self.exports_hoisted.append(name)
                elif kw in ("class", "enum"):
                    name = t[k + 1].text
                    e = k + 2
                    while not s.is_p(e, "{"):
                        e += 1 if not s.is_p(e, "(", "[") else (s.match[e] - e + 1)
                    e = s.match[e]
                    t[e].post += f" exports.{name} = {name};"
                elif kw in ("const", "let", "var"):
                    # exported names: simple declarators only
                    e = k + 1
                    names = []
                    expect_name = True
                    while not (s.is_p(e, ";") or t[e].kind == "eof"):
                        if s.is_p(e, "(", "[", "{"):
                            e = s.match[e] + 1
                            expect_name = False
                            continue
                        if expect_name and t[e].kind == "id":
                            names.append(t[e].text)
                            expect_name = False
                        elif s.is_p(e, ","):
                            expect_name = True
                        e += 1
                    t[e].post += "".join(f" exports.{nm} = {nm};" for nm in names)
                else:
                    raise SyntaxError(f"{self.name}: export {kw}")
                i = k
                continue
            i += 1

    def pass_decls(self):
        """interfaces, type aliases, enums, `declare`, abstract class keyword"""
        s, t = self.s, self.t
        i = 0
        while t[i].kind != "eof":
            tk = t[i]
            if tk.kind == "id" and not tk.drop and not s.is_p(s.prv(i), "."):
                if tk.text == "interface" and self.stmt_start(i) and t[i + 1].kind == "id":
                    j = i + 2
                    while not s.is_p(j, "{"):
                        j += 1
                    s.drop(i, s.match[j] + 1)
                    i = s.match[j] + 1
                    continue
                if tk.text == "type" and self.stmt_start(i) and t[i + 1].kind == "id" and s.is_p(i + 2, "=", "<"):
                    j = i + 2
                    depth = 0
                    while True:
                        if s.is_p(j, "(", "[", "{"):
                            j = s.match[j] + 1
                            continue
                        if s.is_p(j, "<"):
                            depth += 1
                        elif s.is_p(j, ">"):
                            depth -= 1
                        elif s.is_p(j, ">>"):
                            depth -= 2
                        if depth == 0 and s.is_p(j, ";"):
                            break
                        j += 1
                    s.drop(i, j + 1)
                    i = j + 1
                    continue
                if tk.text == "declare" and self.stmt_start(i):
                    j = i
                    while not s.is_p(j, ";"):
                        j = s.match[j] + 1 if s.is_p(j, "{", "(", "[") else j + 1
                    s.drop(i, j + 1)
                    i = j + 1
                    continue
                if tk.text == "enum" and self.stmt_start(i):
                    name = t[i + 1].text
                    j = i + 2
                    e = s.match[j]
                    members = []
                    m = j + 1
                    while m < e:
                        if s.is_p(m, ","):
                            m += 1
                            continue
                        key = t[m].text.strip("'\"")
                        m += 1
                        init = None
                        if s.is_p(m, "="):
                            a = m + 1
                            b = a
                            while b < e and not s.is_p(b, ","):
                                b += 1
                            init = " ".join(x.text for x in t[a:b])
                            m = b
                        members.append((key, init))
                    js = [f"var {name} = {{}};"]
                    auto = 0
                    for key, init in members:
                        if init is None:
                            val = str(auto)
                            auto += 1
                        else:
                            val = re.sub(r"\b(" + "|".join(re.escape(k) for k, _ in members) + r")\b",
                                         lambda mm: f"{name}.{mm.group(1)}", init)
                            try:
                                auto = int(eval(val.replace(f"{name}.", "0*"), {}, {})) + 1  # numeric init
                            except Exception:
                                pass
                        if init is not None and (init.startswith('"') or init.startswith("'")):
                            js.append(f"{name}[{key!r}] = {val};")
                        else:
                            js.append(f"{name}[{name}[{key!r}] = {val}] = {key!r};")
                    s.drop(i, e + 1)
                    t[i].pre = " ".join(js)
                    i = e + 1
                    continue
                if tk.text == "abstract" and s.is_id(i + 1, "class"):
                    tk.drop = True
            i += 1

    # -- pass 2: classes -------------------------------------------------------
    def pass_classes(self):
        s, t = self.s, self.t
        i = 0
        while t[i].kind != "eof":
            tk = t[i]
            if tk.kind == "id" and tk.text == "class" and not tk.drop and not s.is_p(s.prv(i), "."):
                j = i + 1
                if t[j].kind == "id" and t[j].text not in ("extends", "implements"):
                    j += 1
                if s.is_p(j, "<"):
                    e = s.angle_end(j)
                    s.drop(j, e)
                    j = e
                has_super = False
                while not s.is_p(j, "{"):
                    if s.is_id(j, "extends"):
                        has_super = True
                        j += 1
                        while not (s.is_p(j, "{") or s.is_id(j, "implements")):
                            if s.is_p(j, "<"):
                                e = s.angle_end(j)
                                if e:
                                    s.drop(j, e)
                                    j = e
                                    continue
                            if s.is_p(j, "(", "["):
                                j = s.match[j] + 1
                                continue
                            j += 1
                        continue
                    if s.is_id(j, "implements"):
                        k = j
                        while not s.is_p(k, "{"):
                            k = k + 1 if not s.is_p(k, "<") else s.angle_end(k)
                        s.drop(j, k)
                        j = k
                        continue
                    j += 1
                self.class_bodies.add(j)
                self.process_class_body(j, has_super)
                i = j + 1
                continue
            i += 1

    def process_class_body(self, b, has_super):
        s, t = self.s, self.t
        e = s.match[b]
        i = b + 1
        while i < e:
            if s.is_p(i, ";"):
                i += 1
                continue
            start = i
            # modifiers
            while t[i].kind == "id" and t[i].text in MODIFIERS | {"static", "async", "get", "set"} and \
                    (t[i + 1].kind == "id" or s.is_p(i + 1, "[", "#", "*")) and not s.is_p(i + 1, "(", "=", ":", ";"):
                if t[i].text in MODIFIERS:
                    t[i].drop = True
                i += 1
            if s.is_p(i, "["):  # computed name or index signature
                close = s.match[i]
                if s.is_p(i + 2, ":") and t[i + 1].kind == "id":  # index signature [k: T]: V;
                    j = close + 1
                    while not s.is_p(j, ";"):
                        j = s.match[j] + 1 if s.is_p(j, "(", "[", "{") else j + 1
                    s.drop(start, j + 1)
                    i = j + 1
                    continue
                i = close + 1
            elif s.is_p(i, "#"):
                i += 2
            else:
                name_tok = i
                self.member_names.add(i)
                i += 1
            optional = False
            if s.is_p(i, "?", "!"):
                optional = t[i].text == "?"
                t[i].drop = True
                i += 1
            if s.is_p(i, "<"):
                g = s.angle_end(i)
                s.drop(i, g)
                i = g
            if s.is_p(i, "("):
                ctor = t[start].text == "constructor" or (t[name_tok].text == "constructor" if 'name_tok' in dir() else False)
                pp = self.process_params(i, ctor=t[i - 1].text == "constructor")
                close = s.match[i]
                j = close + 1
                if s.is_p(j, ":"):
                    k = s.skip_type(j + 1, brace_ends=True)
                    s.drop(j, k)
                    j = k
                if s.is_p(j, ";") or s.is_p(j, "}") and j == e:  # overload / abstract
                    s.drop(start, j + (1 if s.is_p(j, ";") else 0))
                    i = j + 1
                    continue
                assert s.is_p(j, "{"), (self.name, t[j - 3:j + 3])
                if pp:
                    self.inject_param_props(j, pp, has_super)
                i = s.match[j] + 1
                continue
            # field
            j = i
            typed = False
            if s.is_p(j, ":"):
                k = s.skip_type(j + 1)
                s.drop(j, k)
                j = k
                typed = True
            if s.is_p(j, "="):
                k = j + 1
                while not (s.is_p(k, ";") or k >= e):
                    k = s.match[k] + 1 if s.is_p(k, "(", "[", "{") else k + 1
                i = k + 1 if s.is_p(k, ";") else k
                continue
            # no initializer: TS emits nothing for it
            end = j + 1 if s.is_p(j, ";") else j
            s.drop(start, end)
            i = end
            del typed, optional

    def inject_param_props(self, brace, names, has_super):
        s, t = self.s, self.t
        assigns = "".join(f" this.{n} = {n};" for n in names)
        if has_super:
            # after the super(...) call statement
            j = brace + 1
            e = s.match[brace]
            while j < e:
                if s.is_id(j, "super") and s.is_p(j + 1, "("):
                    k = s.match[j + 1] + 1
                    if s.is_p(k, ";"):
                        t[k].post += assigns
                    else:
                        t[k - 1].post += ";" + assigns
                    return
                j += 1
        t[brace].post += assigns

    # -- parameters --------------------------------------------------------------
    def process_params(self, p, ctor=False):
        """strip types / modifiers / `?` in a parameter list at `(` index p;
        returns the parameter-property names (constructors)."""
        s, t = self.s, self.t
        self.params[p] = ctor
        e = s.match[p]
        props = []
        i = p + 1
        while i < e:
            # one parameter
            pstart = i
            is_prop = False
            while t[i].kind == "id" and t[i].text in MODIFIERS and (t[i + 1].kind == "id" or s.is_p(i + 1, "{", "[")):
                t[i].drop = True
                is_prop = True
                i += 1
            if s.is_id(i, "this") and s.is_p(i + 1, ":"):
                k = s.skip_type(i + 2)
                s.drop(pstart, k + (1 if s.is_p(k, ",") else 0))
                i = k + 1
                continue
            if s.is_p(i, "..."):
                i += 1
            if s.is_p(i, "{", "["):
                self.process_pattern(i)
                i = s.match[i] + 1
            else:
                if is_prop:
                    props.append(t[i].text)
                i += 1
            if s.is_p(i, "?"):
                t[i].drop = True
                i += 1
            if s.is_p(i, ":"):
                k = s.skip_type(i + 1)
                s.drop(i, k)
                i = k
            if s.is_p(i, "="):
                # default value: an expression up to the next top-level comma
                i += 1
                while i < e and not s.is_p(i, ","):
                    i = s.match[i] + 1 if s.is_p(i, "(", "[", "{") else i + 1
            if s.is_p(i, ","):
                i += 1
        return props

    def process_pattern(self, i):
        """destructuring pattern: defaults may hold arrow functions etc.; nothing
        to strip inside for this code base"""
        return

    # -- pass 3: functions, arrows, declarations, expressions ----------------------
    def pass_code(self):
        s, t = self.s, self.t
        i = 0
        while t[i].kind != "eof":
            tk = t[i]
            if tk.drop:
                i += 1
                continue
            if tk.kind == "id" and tk.text == "function" and not s.is_p(s.prv(i), "."):
                j = i + 1
                if s.is_p(j, "*"):
                    j += 1
                if t[j].kind == "id":
                    j += 1
                if s.is_p(j, "<"):
                    g = s.angle_end(j)
                    s.drop(j, g)
                    j = g
                if s.is_p(j, "(") and j not in self.params:
                    self.process_params(j)
                    close = s.match[j]
                    k = close + 1
                    if s.is_p(k, ":"):
                        m = s.skip_type(k + 1, brace_ends=True)
                        s.drop(k, m)
                        k = m
                    if s.is_p(k, ";"):  # overload signature
                        st = i
                        pv = s.prv(i)
                        while pv >= 0 and s.is_id(pv, "export", "declare", "async"):
                            st = pv
                            pv = s.prv(pv)
                        s.drop(st, k + 1)
                        if t[st].text == "export" or any(x.text == "export" for x in t[st:i]):
                            pass
                        i = k + 1
                        continue
                i += 1
                continue
            if tk.kind == "p" and tk.text == "(" and i not in self.params:
                close = s.match[i]
                k = close + 1
                arrow = False
                if s.is_p(k, "=>"):
                    arrow = True
                elif s.is_p(k, ":") and not self._ternary_colon(i):
                    m = s.skip_type(k + 1, stop_arrow=True)
                    if s.is_p(m, "=>"):
                        arrow = True
                        s.drop(k, m)
                if arrow:
                    self.process_params(i)
                    pv = s.prv(i)
                    if s.is_p(pv, ">"):  # generic arrow <T>(...) =>
                        pass
                elif t[s.prv(i)].kind == "id" and t[s.prv(i)].text not in KEYWORDS_BEFORE_PAREN and \
                        s.is_p(s.prv(s.prv(i)), "{", ",") and self._in_object(s.prv(i)) and \
                        (s.is_p(k, "{") or s.is_p(k, ":")):
                    # object-literal method shorthand: name(params)[: R] { body }
                    self.member_names.add(s.prv(i))
                    self.process_params(i)
                    if s.is_p(k, ":"):
                        m = s.skip_type(k + 1, brace_ends=True)
                        s.drop(k, m)
                i += 1
                continue
            if tk.kind == "id" and tk.text in ("let", "const", "var") and not s.is_p(s.prv(i), "."):
                self.process_decl(i)
                i += 1
                continue
            if tk.kind == "id" and tk.text == "as" and not s.is_p(s.prv(i), ".") and self._expr_end(s.prv(i)):
                if s.is_id(i + 1, "const"):
                    s.drop(i, i + 2)
                    i += 2
                    continue
                k = s.skip_type(i + 1)
                s.drop(i, k)
                i = k
                continue
            if tk.kind == "p" and tk.text == "!" and self._expr_end(s.prv(i)) and "\n" not in tk.ws:
                tk.drop = True
                i += 1
                continue
            if tk.kind == "p" and tk.text == "<":
                pv = s.prv(i)
                if t[pv].kind == "id" and t[pv].text not in KEYWORDS_BEFORE_PAREN and not tk.ws:
                    g = s.generic_end(i)
                    if g is not None and s.is_p(g, "("):
                        s.drop(i, g)  # type arguments of a call / new
                        i = g
                        continue
                if not self._expr_end(pv):
                    g = s.generic_end(i)
                    if g is not None and t[i + 1].kind == "id":
                        s.drop(i, g)  # <T>expr cast
                        i = g
                        continue
            i += 1

    def _expr_end(self, j):
        if j < 0:
            return False
        tk = self.t[j]
        if tk.kind in ("num", "str", "tmpl", "regex"):
            return True
        if tk.kind == "id":
            return tk.text not in KEYWORDS_BEFORE_PAREN | {"typeof", "in", "of", "instanceof", "new", "delete",
                                                           "void", "else", "return", "case", "throw", "await"}
        return tk.text in (")", "]", "}")

    def _ternary_colon(self, i):
        """is the `:` after the group at i the else-branch of a conditional?
        Scan back for an unmatched `?` on this nesting level."""
        s, t = self.s, self.t
        j = s.prv(i)
        while j >= 0:
            tk = t[j]
            if tk.kind == "p":
                if tk.text in (")", "]", "}"):
                    j = s.prv(s.match[j])
                    continue
                if tk.text in ("(", "[", "{", ";", ","):
                    return False
                if tk.text == "?":
                    return True
                if tk.text == ":":
                    return False
            j = s.prv(j)
        return False

    def process_decl(self, i):
        """let/const/var declarators: drop `: T` and definite `!`"""
        s, t = self.s, self.t
        j = i + 1
        while True:
            if s.is_p(j, "{", "["):
                j = s.match[j] + 1
            elif t[j].kind == "id":
                j += 1
            else:
                return
            if s.is_p(j, "!"):
                t[j].drop = True
                j += 1
            if s.is_p(j, ":"):
                k = s.skip_type(j + 1)
                s.drop(j, k)
                j = k
            if s.is_id(j, "of", "in"):
                return
            if s.is_p(j, "="):
                j += 1
                while not (s.is_p(j, ",", ";", ")") or t[j].kind == "eof" or
                           (t[j].kind == "id" and t[j].text in ("of", "in") and False)):
                    if s.is_p(j, "(", "[", "{"):
                        j = s.match[j] + 1
                    else:
                        j += 1
            if s.is_p(j, ","):
                j += 1
                continue
            return

    # -- pass 4: identifiers of imports --------------------------------------------
    def pass_import_refs(self):
        s, t = self.s, self.t
        used = set()
        for i, tk in enumerate(t):
            if tk.drop or tk.kind != "id" or tk.text not in self.imports or i in self.member_names:
                continue
            pv = s.prv(i)
            if s.is_p(pv, ".", "?.") and not s.is_p(pv, "..."):
                continue
            nx = s.nxt(i)
            if s.is_p(pv, "{", ",") and s.is_p(nx, ":") and self._in_object(i):
                continue  # object key
            mv, name = self.imports[tk.text]
            used.add(mv)
            ref = mv if name is None else (f"{mv}.default" if name == "default" else f"{mv}.{name}")
            if s.is_p(pv, "{", ",") and s.is_p(nx, ",", "}") and self._in_object(i):
                tk.text = f"{tk.text}: {ref}"
            else:
                tk.text = ref
        return used

    def _in_object(self, i):
        """inside an object literal (not a block / pattern)?  Heuristic: the
        enclosing `{` follows `=`, `(`, `,`, `:`, `return` or `[`."""
        s, t = self.s, self.t
        depth = 0
        j = i - 1
        while j >= 0:
            if s.is_p(j, "}", ")", "]"):
                j = s.match[j] - 1
                continue
            if s.is_p(j, "{"):
                pv = s.prv(j)
                return pv >= 0 and (s.is_p(pv, "=", "(", ",", ":", "[", "?", "=>", "??", "||", "&&") or
                                    s.is_id(pv, "return"))
            if s.is_p(j, "(", "["):
                return False
            j -= 1
        return False

    # -- emit ----------------------------------------------------------------------
    def emit_ts_stripped(self):
        out = []
        for tk in self.t:
            out.append(tk.ws)
            out.append(tk.pre)
            if not tk.drop:
                out.append(tk.text)
            out.append(tk.post)
        return "".join(out)

    def run(self):
        self.pass_modules()
        self.pass_decls()
        self.pass_classes()
        self.pass_code()
        used = self.pass_import_refs()
        body = self.emit_ts_stripped()
        body = downlevel(body)
        head = ['"use strict";', 'Object.defineProperty(exports, "__esModule", { value: true });',
                "function __exportStar(m) { for (var k in m) if (k !== 'default' && !Object.prototype.hasOwnProperty"
                ".call(exports, k)) Object.defineProperty(exports, k, {enumerable: true, get: (function (k) "
                "{ return function () { return m[k]; }; })(k)}); }"]
        for name in self.exports_hoisted:
            head.append(f"exports.{name} = {name};")
        for path, mv in self.modvars.items():
            if mv in used:
                head.append(f"const {mv} = require({path});")
        head.extend(self.reexports)
        return "\n".join(head) + "\n" + body


# ---------------------------------------------------------------------------
# ?. ?? ??= -> ES2017
# ---------------------------------------------------------------------------
def downlevel(js):
    for _ in range(10000):
        toks = tokenize(js)
        s = Src(toks)
        k = next((i for i, tk in enumerate(toks) if tk.kind == "p" and tk.text in ("?.", "??", "??=")), None)
        if k is None:
            return js
        tk = toks[k]
        if tk.text == "?.":
            a = _chain_start(s, k)
            b = _chain_end(s, k)
            left = _text(toks, a, k)
            rest = _text(toks, k + 1, b)
            if toks[k + 1].kind == "p" and toks[k + 1].text in ("(", "["):
                rest_join = rest
            else:
                rest_join = "." + rest
            if _has_call(s, a, k):
                rep = f"(function (__t) {{ return __t == null ? void 0 : __t{rest_join}; }}).call(this, {left})"
            else:
                rep = f"({left} == null ? void 0 : {left}{rest_join})"
        elif tk.text == "??":
            a = _operand_start(s, k)
            b = _operand_end(s, k)
            left = _text(toks, a, k)
            right = _text(toks, k + 1, b)
            rep = f"(function (__t) {{ return __t != null ? __t : {right}; }}).call(this, {left})" \
                if _has_call(s, a, k) or "arguments" in right else \
                f"(({left}) != null ? ({left}) : {right})"
        else:  # ??=
            a = _chain_start(s, k)
            b = _operand_end(s, k)
            left = _text(toks, a, k)
            right = _text(toks, k + 1, b)
            rep = f"(({left}) != null ? ({left}) : ({left} = {right}))"
        js = _splice(toks, a, b, rep)
    raise RuntimeError("downlevel did not converge")


def _text(toks, a, b):
    return "".join((tk.ws if i > a else "") + tk.text for i, tk in enumerate(toks[a:b], start=a))


def _splice(toks, a, b, rep):
    out = []
    for i, tk in enumerate(toks):
        if i == a:
            out.append(tk.ws + rep)
        elif a < i < b:
            continue
        else:
            out.append(tk.ws + tk.text)
    return "".join(out)


def _chain_start(s, k):
    """first token of the member chain ending before k"""
    t = s.t
    j = k - 1
    while True:
        tk = t[j]
        if tk.kind == "p" and tk.text in (")", "]"):
            j = s.match[j] - 1
            # a call / index continues the chain to the left; a bare group starts it
            if j >= 0 and (t[j].kind == "id" and t[j].text not in KEYWORDS_BEFORE_PAREN or
                           t[j].kind == "p" and t[j].text in (")", "]")):
                continue
            return j + 1
        if tk.kind in ("id", "str", "num", "tmpl"):
            if j > 0 and t[j - 1].kind == "p" and t[j - 1].text in (".", "?."):
                j -= 2
                continue
            return j
        raise SyntaxError(f"?. after {tk!r}")


def _chain_end(s, k):
    """index past the optional chain starting at k (`?.`)"""
    t = s.t
    j = k + 1
    if t[j].kind == "id":
        j += 1
    elif t[j].kind == "p" and t[j].text in ("(", "["):
        j = s.match[j] + 1
    while True:
        tk = t[j]
        if tk.kind == "p" and tk.text in (".", "?.") and t[j + 1].kind == "id":
            j += 2
        elif tk.kind == "p" and tk.text == "?." and t[j + 1].text in ("(", "["):
            j = s.match[j + 1] + 1
        elif tk.kind == "p" and tk.text in ("(", "[") and not tk.ws.count("\n"):
            j = s.match[j] + 1
        else:
            return j


def _has_call(s, a, b):
    return any(tk.kind == "p" and tk.text == "(" for tk in s.t[a:b])


LOW = {"=", "+=", "-=", "*=", "/=", "%=", "||=", "&&=", "??=", "?", ":", ",", "(", "[", "{", ";", "=>", "||", "&&",
       "??", "...", "}", ")", "]"}


def _operand_start(s, k):
    t = s.t
    j = k - 1
    while j >= 0:
        tk = t[j]
        if tk.kind == "p" and tk.text in (")", "]", "}"):
            j = s.match[j] - 1
            continue
        if tk.kind == "p" and tk.text in LOW:
            return j + 1
        if tk.kind == "id" and tk.text in ("return", "case", "throw", "typeof", "await", "else", "yield", "of", "in"):
            return j + 1
        j -= 1
    return 0


def _operand_end(s, k):
    t = s.t
    j = k + 1
    while True:
        tk = t[j]
        if tk.kind == "eof":
            return j
        if tk.kind == "p" and tk.text in ("(", "[", "{"):
            j = s.match[j] + 1
            continue
        if tk.kind == "p" and tk.text in (")", "]", "}", ",", ";", "?", ":", "??", "||", "&&", "=>"):
            return j
        j += 1


# ---------------------------------------------------------------------------
def erase_file(path):
    src = open(path, encoding="utf-8").read()
    return Eraser(src, path).run()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=DEFAULT_SRC)
    ap.add_argument("--out", default=DEFAULT_OUT)
    ap.add_argument("files", nargs="*")
    args = ap.parse_args()
    if not os.path.isdir(args.src):
        sys.exit(f"reference sources not found: {args.src}")
    n = 0
    for root, dirs, files in os.walk(args.src):
        dirs[:] = [d for d in dirs if d != "test"]
        for f in files:
            if not f.endswith(".ts") or f.endswith(".d.ts"):
                continue
            rel = os.path.relpath(os.path.join(root, f), args.src)
            if args.files and rel not in args.files:
                continue
            try:
                js = erase_file(os.path.join(root, f))
            except Exception as ex:  # report and go on: one file at a time
                import traceback
                print(f"FAILED {rel}: {ex!r}")
                traceback.print_exc(limit=3)
                continue
            dst = os.path.join(args.out, rel[:-3] + ".js")
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            open(dst, "w", encoding="utf-8").write(js)
            n += 1
    # the packages the sources import: erased from the reference where their
    # values are used, the loggers / error classes / summary builder from
    # ref_stubs.js, the type-only ones empty
    stubs = os.path.join(HERE, "ref_stubs.js")
    nm = os.path.join(args.out, "node_modules", "@fluidframework")
    for pkg, mods in EXTERNAL.items():
        d = os.path.join(nm, pkg)
        os.makedirs(d, exist_ok=True)
        for name, rel in mods:
            open(os.path.join(d, name + ".js"), "w", encoding="utf-8").write(
                erase_file(os.path.join(REF_ROOT, rel)))
            n += 1
        for alias, target in INDEX_ALIASES.get(pkg, {}).items():
            open(os.path.join(d, alias + ".js"), "w").write(f"module.exports = require(\"./{target}\");\n")
        reqs = ", ".join(f"require(\"./{name}\")" for name, _ in mods)
        extra = f", require({stubs!r})" if pkg in STUB_EXTRA else ""
        open(os.path.join(d, "index.js"), "w").write(f"module.exports = Object.assign({{}}, {reqs}{extra});\n")
    for pkg in STUBBED:
        d = os.path.join(nm, pkg)
        os.makedirs(d, exist_ok=True)
        open(os.path.join(d, "index.js"), "w").write(f"module.exports = require({stubs!r});\n")
    seq_out = os.path.join(args.out, "sequence")
    os.makedirs(seq_out, exist_ok=True)
    for f in SEQUENCE_FILES:
        open(os.path.join(seq_out, f[:-3] + ".js"), "w", encoding="utf-8").write(
            erase_file(os.path.join(REF_ROOT, SEQUENCE_SRC, f)))
        n += 1
    d = os.path.join(nm, "merge-tree")
    os.makedirs(d, exist_ok=True)
    open(os.path.join(d, "index.js"), "w").write("module.exports = require(\"../../../index\");\n")
    d = os.path.join(args.out, "node_modules", "uuid")
    os.makedirs(d, exist_ok=True)
    open(os.path.join(d, "index.js"), "w").write(
        "module.exports = { v4() { throw new Error(\"uuid is not available offline: pass interval ids\"); } };\n")
    for pkg in TYPE_ONLY:
        d = os.path.join(nm, pkg)
        os.makedirs(d, exist_ok=True)
        open(os.path.join(d, "index.js"), "w").write("module.exports = {};\n")
    print(f"erased {n} files -> {args.out}")


if __name__ == "__main__":
    main()
