"""A small SQL expression parser for splink settings.

splink's settings carry SQL text: CASE expressions for comparison columns
(case_statements.py:62-277, or user-written) and join conditions for blocking rules
(blocking.py:95-160).  This module parses that text into an AST; splink_amd.compiler turns
the AST into device programs.  Anything outside the supported grammar raises ValueError.

Grammar (precedence low -> high):
    expr     := or
    or       := and (OR and)*
    and      := not (AND not)*
    not      := NOT not | cmp
    cmp      := add ((= | == | != | <> | < | <= | > | >=) add | IS [NOT] NULL)?
    add      := mul ((+ | -) mul)*
    mul      := unary ((* | / | %) unary)*
    unary    := - unary | primary
    primary  := number | 'string' | TRUE | FALSE | NULL | CASE ... END
              | CAST ( expr AS type ) | name ( args ) | name[.name] | ( expr )
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union


@dataclass(frozen=True)
class Lit:
    value: object  # int / float / str / bool / None


@dataclass(frozen=True)
class Col:
    name: str          # column name, lower-cased
    qualifier: str = ""  # "l" / "r" / "" (lower-cased)


@dataclass(frozen=True)
class Func:
    name: str
    args: Tuple["Node", ...]


@dataclass(frozen=True)
class Bin:
    op: str
    a: "Node"
    b: "Node"


@dataclass(frozen=True)
class Un:
    op: str  # "-" or "not"
    a: "Node"


@dataclass(frozen=True)
class IsNull:
    a: "Node"
    negated: bool = False


@dataclass(frozen=True)
class Case:
    whens: Tuple[Tuple["Node", "Node"], ...]
    else_: Optional["Node"] = None


Node = Union[Lit, Col, Func, Bin, Un, IsNull, Case]

_TOKEN = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?)
  | (?P<str>'(?:[^'\\]|\\.|'')*')
  | (?P<qid>`[^`]*`|"[^"]*")
  | (?P<id>[A-Za-z_][A-Za-z_0-9$]*)
  | (?P<op><=|>=|<>|!=|==|[=<>+\-*/%(),.])
""", re.VERBOSE | re.DOTALL)

KEYWORDS = {"case", "when", "then", "else", "end", "and", "or", "not", "is", "null", "true", "false", "as"}


_ESCAPES = {"0": "\u0000", "'": "'", '"': '"', "b": "\b", "n": "\n", "r": "\r", "t": "\t", "Z": "\u001A",
            "\\": "\\", "%": "\\%", "_": "\\_"}


def unescape_literal(quoted: str) -> str:
    """The value of a single-quoted SQL string literal (quotes included), as Spark's parser reads it
    (ParserUtils.unescapeSQLString, Spark 2.4): backslash escapes \\0 \\' \\" \\b \\n \\r \\t \\Z \\\\ (\\% and \\_
    keep their backslash, any other escaped character stands for itself), \\uXXXX and three-digit octal \\[01][0-7][0-7].
    A doubled quote '' stands for one quote (SQL-standard quoting, which the sqlite oracle and the reference's
    generated SQL use; Spark itself would read 'a''b' as two adjacent literals)."""
    b = quoted[1:-1]
    out = []
    i, n = 0, len(b)
    while i < n:
        c = b[i]
        if c == "'" and i + 1 < n and b[i + 1] == "'":
            out.append("'")
            i += 2
            continue
        if c != "\\" or i + 1 >= n:
            out.append(c)
            i += 1
            continue
        nxt = b[i + 1]
        if nxt == "u" and i + 5 < n and all(ch in "0123456789abcdefABCDEF" for ch in b[i + 2:i + 6]):
            out.append(chr(int(b[i + 2:i + 6], 16)))
            i += 6
        elif i + 3 < n and b[i + 1] in "01" and b[i + 2] in "01234567" and b[i + 3] in "01234567":
            out.append(chr(int(b[i + 1:i + 4], 8)))
            i += 4
        else:
            out.append(_ESCAPES.get(nxt, nxt))
            i += 2
    return "".join(out)


def tokenize(text: str):
    toks = []
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise ValueError(f"unexpected character {text[pos]!r} in SQL expression: {text!r}")
        pos = m.end()
        kind = m.lastgroup
        val = m.group(kind)
        if kind == "ws":
            continue
        if kind == "str":
            toks.append(("str", unescape_literal(val)))
        elif kind == "num":
            toks.append(("num", val))
        elif kind == "qid":
            toks.append(("id", val[1:-1]))
        elif kind == "id":
            low = val.lower()
            toks.append(("kw", low) if low in KEYWORDS else ("id", val))
        else:
            toks.append(("op", val))
    toks.append(("eof", None))
    return toks


class _Parser:
    def __init__(self, text: str):
        self.text = text
        self.toks = tokenize(text)
        self.i = 0

    def peek(self, k=0):
        return self.toks[self.i + k]

    def take(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, val=None):
        t = self.peek()
        if t[0] == kind and (val is None or t[1] == val):
            self.i += 1
            return t
        return None

    def expect(self, kind, val=None):
        t = self.accept(kind, val)
        if t is None:
            got = self.peek()
            raise ValueError(f"expected {val or kind}, got {got[1]!r} in SQL expression: {self.text!r}")
        return t

    def parse_expr(self):
        return self.parse_or()

    def parse_or(self):
        a = self.parse_and()
        while self.accept("kw", "or"):
            a = Bin("or", a, self.parse_and())
        return a

    def parse_and(self):
        a = self.parse_not()
        while self.accept("kw", "and"):
            a = Bin("and", a, self.parse_not())
        return a

    def parse_not(self):
        if self.accept("kw", "not"):
            return Un("not", self.parse_not())
        return self.parse_cmp()

    def parse_cmp(self):
        a = self.parse_add()
        t = self.peek()
        if t[0] == "op" and t[1] in ("=", "==", "!=", "<>", "<", "<=", ">", ">="):
            self.take()
            op = {"==": "=", "<>": "!="}.get(t[1], t[1])
            return Bin(op, a, self.parse_add())
        if self.accept("kw", "is"):
            neg = bool(self.accept("kw", "not"))
            self.expect("kw", "null")
            return IsNull(a, neg)
        return a

    def parse_add(self):
        a = self.parse_mul()
        while True:
            t = self.peek()
            if t[0] == "op" and t[1] in ("+", "-"):
                self.take()
                a = Bin(t[1], a, self.parse_mul())
            else:
                return a

    def parse_mul(self):
        a = self.parse_unary()
        while True:
            t = self.peek()
            if t[0] == "op" and t[1] in ("*", "/", "%"):
                self.take()
                a = Bin(t[1], a, self.parse_unary())
            else:
                return a

    def parse_unary(self):
        if self.accept("op", "-"):
            inner = self.parse_unary()
            if isinstance(inner, Lit) and isinstance(inner.value, (int, float)) and not isinstance(inner.value, bool):
                return Lit(-inner.value)
            return Un("-", inner)
        if self.accept("op", "+"):
            return self.parse_unary()
        return self.parse_primary()

    def parse_primary(self):
        t = self.take()
        kind, val = t
        if kind == "num":
            return Lit(float(val) if any(c in val for c in ".eE") else int(val))
        if kind == "str":
            return Lit(val)
        if kind == "kw":
            if val == "null":
                return Lit(None)
            if val == "true":
                return Lit(True)
            if val == "false":
                return Lit(False)
            if val == "case":
                return self.parse_case()
            raise ValueError(f"unexpected keyword {val!r} in SQL expression: {self.text!r}")
        if kind == "op" and val == "(":
            e = self.parse_expr()
            self.expect("op", ")")
            return e
        if kind == "id":
            if val.lower() == "cast" and self.peek()[0] == "op" and self.peek()[1] == "(":
                # CAST(expr AS type): Func("cast", (expr, Lit(type)))
                self.take()
                e = self.parse_expr()
                self.expect("kw", "as")
                typ = self.expect("id")[1].lower()
                self.expect("op", ")")
                return Func("cast", (e, Lit(typ)))
            if self.accept("op", "("):
                args = []
                if not self.accept("op", ")"):
                    args.append(self.parse_expr())
                    while self.accept("op", ","):
                        args.append(self.parse_expr())
                    self.expect("op", ")")
                return Func(val.lower(), tuple(args))
            if self.accept("op", "."):
                name = self.expect("id")[1]
                return Col(name.lower(), val.lower())
            return Col(val.lower(), "")
        raise ValueError(f"unexpected token {val!r} in SQL expression: {self.text!r}")

    def parse_case(self):
        whens = []
        operand = None
        if not (self.peek()[0] == "kw" and self.peek()[1] == "when"):
            operand = self.parse_expr()  # simple CASE x WHEN v THEN ...
        while self.accept("kw", "when"):
            cond = self.parse_expr()
            if operand is not None:
                cond = Bin("=", operand, cond)
            self.expect("kw", "then")
            whens.append((cond, self.parse_expr()))
        if not whens:
            raise ValueError(f"CASE without WHEN in SQL expression: {self.text!r}")
        else_ = None
        if self.accept("kw", "else"):
            else_ = self.parse_expr()
        self.expect("kw", "end")
        return Case(tuple(whens), else_)


def parse(text: str) -> Node:
    """Parse one SQL expression (an optional trailing `AS alias` is accepted and dropped)."""
    p = _Parser(text)
    e = p.parse_expr()
    if p.accept("kw", "as"):
        p.expect("id")
    p.accept("op", ";")
    if p.peek()[0] != "eof":
        raise ValueError(f"unexpected trailing text {p.peek()[1]!r} in SQL expression: {text!r}")
    return e


def conjuncts(node: Node) -> List[Node]:
    """Flatten a tree of ANDs."""
    if isinstance(node, Bin) and node.op == "and":
        return conjuncts(node.a) + conjuncts(node.b)
    return [node]
