"""Type erasure for ts/verify.ts: TypeScript -> JavaScript that Node 12 runs (test infrastructure only).

Deno is absent from the image, so the TS binding is executed under Node 12 with a Deno.dlopen
shim (tests/ts_harness/deno_shim.js over the N-API addon deno_ffi.cc).  This module removes exactly the
TypeScript that verify.ts uses and nothing else; whatever it does not understand raises, so the binding is
kept inside an erasable subset instead of being silently mistranslated:
  * `import type ...;`, `interface X {...}`, `type X = ...;` statements;
  * `: Type` annotations of parameters (incl. `?` optional markers), return types, variables and class
    fields; `as Type` / `as const`; generic parameters `f<T>(` and type arguments `new Map<...>(`;
  * class member modifiers `readonly` / `private` / `public`; non-null assertions `x!`.
`export` is kept (the output is an ES module, .mjs).  The erasure keeps every newline, so line numbers of
errors match verify.ts.

    python erase_ts.py ts/verify.ts out.mjs
"""
from __future__ import annotations

import re
import sys

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<comment>//[^\n]*|/\*.*?\*/)
  | (?P<str>"(?:\\.|[^"\\])*"|'(?:\\.|[^'\\])*')
  | (?P<tmpl>`(?:\\.|[^`\\])*`)
  | (?P<num>\d[\d_]*n?|0x[0-9a-fA-F]+n?)
  | (?P<id>\#?[A-Za-z_$][\w$]*)
  | (?P<op>=>|\.\.\.|===|!==|==|!=|<=|>=|&&|\|\||\*\*|\?\?|\?\.|[-+*/%&|^!~?:;,.=<>(){}\[\]@])
""", re.S | re.X)

KEYWORDS_BEFORE_PAREN = {"if", "for", "while", "switch", "catch", "return", "await", "typeof", "new", "of",
                         "in", "void", "throw", "case", "else", "do"}


def tokenize(src: str):
    out, i = [], 0
    while i < len(src):
        m = _TOKEN.match(src, i)
        if not m:
            raise SyntaxError(f"erase_ts: cannot tokenize at line {src.count(chr(10), 0, i) + 1}: {src[i:i + 30]!r}")
        out.append((m.lastgroup, m.group()))
        i = m.end()
    return out


class Eraser:
    def __init__(self, src: str):
        self.t = tokenize(src)
        self.out = []
        self.i = 0

    # -- helpers -------------------------------------------------------------------------------------
    def sig(self, j: int) -> int:
        """Index of the first significant token at or after j."""
        while j < len(self.t) and self.t[j][0] in ("ws", "comment"):
            j += 1
        return j

    def val(self, j: int) -> str:
        return self.t[j][1] if j < len(self.t) else ""

    def blank(self, a: int, b: int) -> None:
        """Drop tokens [a, b), keeping their newlines."""
        for k in range(a, b):
            n = self.t[k][1].count("\n")
            self.t[k] = ("ws", "\n" * n if n else (" " if self.t[k][0] != "ws" else self.t[k][1]))

    def skip_type(self, j: int, stops) -> int:
        """End (exclusive) of a type expression starting at significant token j: stops at a token in `stops`
        at bracket depth 0 (`=>` belongs to function types and never stops it)."""
        depth = 0
        while j < len(self.t):
            kind, v = self.t[j]
            if kind in ("ws", "comment"):
                j += 1
                continue
            if depth == 0 and v in stops:
                return j
            if v in "([{<":
                depth += 1
            elif v in ")]}>":
                if depth == 0:
                    return j
                depth -= 1
            j += 1
        raise SyntaxError("erase_ts: unterminated type")

    def match_close(self, j: int) -> int:
        """Index of the bracket closing the one at j."""
        pairs = {"(": ")", "[": "]", "{": "}", "<": ">"}
        open_, close = self.t[j][1], pairs[self.t[j][1]]
        depth = 0
        while j < len(self.t):
            v = self.t[j][1]
            if self.t[j][0] not in ("ws", "comment", "str", "tmpl"):
                if v == open_:
                    depth += 1
                elif v == close:
                    depth -= 1
                    if depth == 0:
                        return j
            j += 1
        raise SyntaxError("erase_ts: unbalanced " + open_)

    # -- passes ---------------------------------------------------------------------------------------
    def statements(self) -> None:
        """Remove `import type`, `interface`, `type X =` statements."""
        j = 0
        while j < len(self.t):
            j = self.sig(j)
            if j >= len(self.t):
                break
            v = self.val(j)
            k = self.sig(j + 1)
            if v == "import" and self.val(k) == "type":
                e = j
                while self.val(e) != ";":
                    e += 1
                self.blank(j, e + 1)
                j = e + 1
                continue
            start = j
            if v == "export" and self.val(k) in ("interface", "type"):
                j, k = k, self.sig(k + 1)
                v = self.val(j)
            if v == "interface" and self.t[k][0] == "id":
                b = k
                while self.val(b) != "{":
                    b += 1
                e = self.match_close(b)
                self.blank(start, e + 1)
                j = e + 1
                continue
            if v == "type" and self.t[k][0] == "id" and self.val(self.sig(k + 1)) == "=":
                e = self.skip_type(self.sig(self.sig(k + 1) + 1), {";"})
                self.blank(start, e + 1)
                j = e + 1
                continue
            j = start + 1

    def annotations(self) -> None:
        """Erase annotations, casts, generics, modifiers and non-null assertions in one left-to-right walk."""
        t = self.t
        j = 0
        stack = []          # bracket kinds: "param" (a parameter list), "class" (a class body), other
        class_pending = False
        while j < len(t):
            kind, v = t[j]
            if kind in ("ws", "comment", "str", "tmpl", "num"):
                j += 1
                continue
            prev = self.prev_sig(j)
            pv = self.val(prev) if prev is not None else ""
            nxt = self.sig(j + 1)
            nv = self.val(nxt)
            if v == "class":
                class_pending = True
            if kind == "id" and v == "as" and prev is not None and (
                    pv in (")", "]", "}") or t[prev][0] in ("id", "str", "num")):
                e = self.skip_type(nxt, {",", ")", ";", "]", "}", "=", "||", "&&", "?", ":"})
                self.blank(j, e)
                j = e
                continue
            if kind == "id" and v in ("readonly", "private", "public", "protected") and stack and stack[-1] == "class":
                self.blank(j, j + 1)
                j += 1
                continue
            if v == "<" and t[j - 1][0] == "id" and t[j - 1][1] not in KEYWORDS_BEFORE_PAREN:
                # generic parameters / type arguments: directly attached to an identifier, followed by `(`
                e = self.match_close(j)
                if self.val(self.sig(e + 1)) == "(":
                    self.blank(j, e + 1)
                    j = e + 1
                    continue
            if v == "!" and pv in (")", "]") or (v == "!" and prev is not None and t[prev][0] == "id"
                                                 and prev == j - 1 and nv in (",", ")", ".", ";", "]")):
                if nv not in ("=", "=="):
                    self.blank(j, j + 1)
                    j += 1
                    continue
            if v == "(":
                stack.append("param" if self.is_param_list(j) else "(")
            elif v == "{":
                stack.append("class" if class_pending else "{")
                class_pending = False
            elif v == "[":
                stack.append("[")
            elif v in ")]}":
                top = stack.pop() if stack else None
                if v == ")" and top == "param":
                    k = self.sig(j + 1)
                    if self.val(k) == ":":                       # return type
                        e = self.skip_type(self.sig(k + 1), {"{", "=>", ";"})
                        self.blank(k, e)
                j += 1
                continue
            elif v == ":" and stack and stack[-1] == "param" and self.is_param_name(prev):
                e = self.skip_type(nxt, {",", ")", "="})
                if pv == "?":
                    self.blank(prev, prev + 1)
                self.blank(j, e)
                j = e
                continue
            elif v == ":" and stack and stack[-1] == "class" and self.is_member_name(prev):
                e = self.skip_type(nxt, {";", "="})
                if pv == "?":
                    self.blank(prev, prev + 1)
                self.blank(j, e)
                j = e
                continue
            elif v == ":" and self.is_var_decl(prev):
                e = self.skip_type(nxt, {"=", ";", ","})
                self.blank(j, e)
                j = e
                continue
            j += 1

    def prev_sig(self, j: int):
        k = j - 1
        while k >= 0 and self.t[k][0] in ("ws", "comment"):
            k -= 1
        return k if k >= 0 else None

    def is_param_list(self, j: int) -> bool:
        """`(` at j opens a parameter list: after `function name`, a method name in a class body or `constructor`,
        or it is an arrow function's parameter list (its `)` is followed by `=>` or `: T =>`)."""
        p = self.prev_sig(j)
        pv = self.val(p) if p is not None else ""
        if pv in KEYWORDS_BEFORE_PAREN:
            return False
        pp = self.prev_sig(p) if p is not None else None
        if pv == "function" or (p is not None and self.t[p][0] == "id" and self.val(pp) == "function"):
            return True
        if pv in ("constructor",):
            return True
        e = self.match_close(j)
        k = self.sig(e + 1)
        if self.val(k) == "=>":
            return True
        if self.val(k) == ":":
            # `(...): T =>` (an arrow with a return type) or a method `name(...): T {`
            end = self.skip_type(self.sig(k + 1), {"{", "=>", ";"})
            return self.val(end) in ("=>", "{") and (self.val(end) == "=>" or self.in_class_member(p))
        if self.val(k) == "{" and self.in_class_member(p):
            return True
        return False

    def in_class_member(self, p) -> bool:
        """Token p is a method name directly in a class body (preceded by `;`, `}`, `{`, `async` or a modifier)."""
        if p is None or self.t[p][0] != "id":
            return False
        q = self.prev_sig(p)
        while q is not None and self.val(q) in ("async", "private", "public", "protected", "static", "readonly"):
            q = self.prev_sig(q)
        return q is not None and self.val(q) in (";", "}", "{")

    def is_param_name(self, p) -> bool:
        if p is None:
            return False
        if self.val(p) == "?":
            p = self.prev_sig(p)
        q = self.prev_sig(p)
        return self.t[p][0] == "id" and self.val(q) in ("(", ",", "...")

    def is_member_name(self, p) -> bool:
        if p is None:
            return False
        if self.val(p) == "?":
            p = self.prev_sig(p)
        q = self.prev_sig(p)
        return self.t[p][0] == "id" and self.val(q) in (";", "{", "}")

    def is_var_decl(self, p) -> bool:
        if p is None or self.t[p][0] != "id":
            return False
        return self.val(self.prev_sig(p)) in ("let", "const", "var")

    def run(self) -> str:
        self.statements()
        self.annotations()
        return "".join(v for _, v in self.t)


def erase(src: str) -> str:
    return Eraser(src).run()


if __name__ == "__main__":
    src = open(sys.argv[1]).read()
    open(sys.argv[2], "w").write(erase(src))
