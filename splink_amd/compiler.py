"""Compile splink's SQL settings into device programs.

* Comparison columns: each completed `case_expression` (a CASE over `<col>_l` / `<col>_r`,
  case_statements.py:62-277 or user-written) becomes a column program: WHEN branches whose
  predicates are RPN sequences of leaf tests (IS NULL, =, jaro_winkler_sim(..) cmp t,
  levenshtein(..)/((length(..)+length(..))/2) cmp t, abs(a-b) cmp t, abs(a-b)/abs(max) cmp t,
  substr / ifnull operands) combined with Kleene AND / OR / NOT.  An operand may be a Spark built-in
  over ONE record's columns (lower / upper / trim / ltrim / rtrim / concat / concat_ws / cast, nested,
  with substr / ifnull inside): a derived column (derived.py) evaluated once per row at ingest.
* Blocking rules (blocking.py:95-160): conjunctions of equalities between an l-side and an
  r-side key expression (a column, optionally under substr / lower / upper / trim).

Anything else raises ValueError naming the unsupported construct, rather than guessing.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from . import _native as N
from . import derived as D
from .sqlexpr import Bin, Case, Col, Func, IsNull, Lit, Un, conjuncts, parse

KLEENE_CONST = {False: 0, True: 1, None: 2}


# ---------------------------------------------------------------------------------------------
# comparison programs
# ---------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class OperandSpec:
    kind: str                      # "col" | "str" | "num"
    side: int = 0
    name: str = ""                 # canonical column name
    form: str = "str"              # device form of the column: "str" | "num"
    lit: Optional[str] = None      # string literal, or the ifnull default string
    num: float = 0.0               # number literal, or the ifnull default number
    has_num_default: bool = False
    substr: Optional[Tuple[int, int]] = None


@dataclass
class CompiledComparisons:
    programs: np.ndarray
    when_first: np.ndarray
    when_n: np.ndarray
    when_level: np.ndarray
    instrs: np.ndarray
    operands: List[OperandSpec]
    literals: List[str]
    n_levels: List[int]
    gamma_names: List[str]
    columns: List[Tuple[str, str]]   # (canonical name, form) the device tables must hold
    # derived columns (derived.py): name -> side-neutral expression of one record, evaluated once per row
    derived: Dict[str, object] = field(default_factory=dict)

    def native_operands(self, column_index: Dict[Tuple[str, str], int]):
        arr = np.zeros(len(self.operands), dtype=N.OPERAND_DTYPE)
        lit_index = {s: i for i, s in enumerate(self.literals)}
        for i, o in enumerate(self.operands):
            arr[i]["kind"] = {"col": 0, "str": 1, "num": 2}[o.kind]
            arr[i]["side"] = o.side
            arr[i]["col"] = column_index[(o.name, o.form)] if o.kind == "col" else 0
            arr[i]["lit"] = lit_index[o.lit] if o.lit is not None else -1
            arr[i]["num"] = o.num
            arr[i]["has_num_default"] = 1 if o.has_num_default else 0
            if o.substr is not None:
                arr[i]["substr_start"], arr[i]["substr_len"] = o.substr
                if arr[i]["substr_start"] == 0:  # Spark treats position 0 as 1
                    arr[i]["substr_start"] = 1
        return arr

    def literal_buffers(self):
        enc = [s.encode("utf-8", "surrogatepass") for s in self.literals]
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(b) for b in enc])
        data = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, np.uint8)
        return off, data


class Schema:
    """Column names of the input table(s), resolved case-insensitively, with their natural forms."""

    def __init__(self, forms: Dict[str, str]):
        self.forms = dict(forms)
        self._lower = {k.lower(): k for k in forms}

    def resolve(self, name: str) -> Optional[str]:
        return self._lower.get(name.lower())

    def form(self, canonical: str) -> str:
        return self.forms[canonical]


class _ProgramBuilder:
    def __init__(self, schema: Schema):
        self.schema = schema
        self.operands: List[OperandSpec] = []
        self.op_index: Dict[OperandSpec, int] = {}
        self.literals: List[str] = []
        self.instrs: List[tuple] = []
        self.whens: List[Tuple[int, int, int]] = []
        self.columns: Dict[Tuple[str, str], None] = {}
        self.derived: Dict[str, object] = {}

    # ---- operands -----------------------------------------------------------------------------
    def _column_ref(self, node: Col):
        if node.qualifier:
            raise ValueError(f"comparison expressions use <col>_l / <col>_r, not {node.qualifier}.{node.name}")
        name = node.name
        for suffix, side in (("_l", 0), ("_r", 1)):
            if name.endswith(suffix):
                canon = self.schema.resolve(name[:-2])
                if canon is not None:
                    return canon, side
        raise ValueError(f"column {node.name!r} in a case_expression does not match <input column>_l / _r")

    def operand(self, node, form_hint: Optional[str]) -> OperandSpec:
        """An operand node: column ref, literal, substr(x, a, b), ifnull / coalesce / nvl(x, literal)."""
        substr = None
        if isinstance(node, Func) and node.name in ("substr", "substring"):
            if len(node.args) not in (2, 3) or not all(isinstance(a, Lit) and isinstance(a.value, int)
                                                       for a in node.args[1:]):
                raise ValueError("substr() needs literal integer position / length")
            substr = (node.args[1].value, node.args[2].value if len(node.args) == 3 else 2 ** 31 - 1)
            node = node.args[0]
            form_hint = "str"
        default = None
        if isinstance(node, Func) and node.name in ("ifnull", "coalesce", "nvl"):
            if len(node.args) != 2 or not isinstance(node.args[1], Lit):
                raise ValueError(f"{node.name}() is supported with a column and a literal default")
            default = node.args[1].value
            node = node.args[0]
        if D.is_derived(node):
            return self._derived_operand(node, form_hint, substr, default)
        if isinstance(node, Lit):
            if substr is not None:
                raise ValueError("substr() of a literal is not supported")
            if isinstance(node.value, str):
                self._lit(node.value)
                return OperandSpec(kind="str", lit=node.value)
            if isinstance(node.value, (int, float)) and not isinstance(node.value, bool):
                return OperandSpec(kind="num", num=float(node.value), form="num")
            raise ValueError(f"unsupported literal {node.value!r} as a comparison operand")
        if not isinstance(node, Col):
            raise ValueError(f"unsupported comparison operand: {node}")
        name, side = self._column_ref(node)
        form = form_hint or self.schema.form(name)
        spec = dict(kind="col", side=side, name=name, form=form, substr=substr)
        if default is not None:
            if isinstance(default, str):
                spec["lit"] = default
                self._lit(default)
                spec["form"] = "str"
            elif isinstance(default, (int, float)) and not isinstance(default, bool):
                spec["num"] = float(default)
                spec["has_num_default"] = True
                spec["form"] = "num"
            else:
                raise ValueError(f"unsupported ifnull default {default!r}")
        o = OperandSpec(**spec)
        self.columns[(o.name, o.form)] = None
        return o

    def _derived_neutral(self, node):
        neutral, side = D.neutralise(node, self._column_ref)
        if side is None:
            raise ValueError(f"{D.render_any(node)} in a case_expression references no <col>_l / <col>_r column")
        return neutral, side

    def _derived_operand(self, node, form_hint, substr, default) -> OperandSpec:
        """A Spark built-in over one record's columns (lower / upper / trim / concat / cast ...): a derived
        column evaluated once per row at ingest (derived.py), read by the pair kernels like an input column.
        When the comparison needs the other form, Spark's implicit cast is folded into the expression."""
        neutral, side = self._derived_neutral(node)
        form = D.form_of(neutral, self.schema.form)
        want = "str" if substr is not None else (form_hint or form)
        if default is not None:
            want = "str" if isinstance(default, str) else "num"
        if want != form:
            neutral = Func("cast", (neutral, Lit("string" if want == "str" else "double")))
            form = want
        name = D.render(neutral)
        self.derived[name] = neutral
        spec = dict(kind="col", side=side, name=name, form=form, substr=substr)
        if default is not None:
            if isinstance(default, str):
                spec["lit"] = default
                self._lit(default)
            elif isinstance(default, (int, float)) and not isinstance(default, bool):
                spec["num"] = float(default)
                spec["has_num_default"] = True
            else:
                raise ValueError(f"unsupported ifnull default {default!r}")
        o = OperandSpec(**spec)
        self.columns[(o.name, o.form)] = None
        return o

    def _day_operand(self, node, shift: int) -> OperandSpec:
        """The day number (days since 1970-01-01, + shift) of a date operand of datediff: a string literal is
        parsed here (DateTimeUtils.stringToDate; NULL if it is not a date); a column or an expression of one record
        becomes the derived numeric column datediff(date_add(x, shift), '1970-01-01') (derived.py)."""
        if isinstance(node, Lit):
            day = D.spark_string_to_date(node.value) if isinstance(node.value, str) else None
            return OperandSpec(kind="num", num=float("nan") if day is None else float(day + shift), form="num")
        inner = node if shift == 0 else Func("date_add", (node, Lit(shift)))
        return self._derived_operand(Func("datediff", (inner, Lit("1970-01-01"))), "num", None, None)

    def _lit(self, s: str):
        if s not in self.literals:
            self.literals.append(s)

    def _op(self, spec: OperandSpec) -> int:
        if spec not in self.op_index:
            self.op_index[spec] = len(self.operands)
            self.operands.append(spec)
        return self.op_index[spec]

    # ---- predicates ----------------------------------------------------------------------------
    def emit(self, op, a=0, b=0, cmp=0, i0=0, t=0.0):
        self.instrs.append((N.OP[op], a, b, N.CMP[cmp] if isinstance(cmp, str) else cmp, i0, 0, float(t)))

    def predicate(self, node):
        if isinstance(node, Bin) and node.op in ("and", "or"):
            self.predicate(node.a)
            self.predicate(node.b)
            self.emit(node.op.upper())
        elif isinstance(node, Un) and node.op == "not":
            self.predicate(node.a)
            self.emit("NOT")
        elif isinstance(node, IsNull):
            o = self.operand(node.a, None)
            self.emit("NOTNULL" if node.negated else "ISNULL", a=self._op(o))
        elif isinstance(node, Lit) and (node.value is None or isinstance(node.value, bool)):
            self.emit("CONST", i0=KLEENE_CONST[node.value])
        elif isinstance(node, Bin) and node.op in ("=", "!=", "<", "<=", ">", ">="):
            self.comparison(node.op, node.a, node.b)
        else:
            raise ValueError(f"unsupported predicate in case_expression: {node}")

    _FLIP = {"=": "=", "!=": "!=", "<": ">", "<=": ">=", ">": "<", ">=": "<="}

    def comparison(self, op, lhs, rhs):
        lv, rv = _classify(lhs), _classify(rhs)
        if lv[0] != "operand" and _is_number(rhs):
            return self._value_test(op, lv, float(rhs.value))
        if rv[0] != "operand" and _is_number(lhs):
            return self._value_test(self._FLIP[op], rv, float(lhs.value))
        if lv[0] == "operand" and rv[0] == "operand":
            return self._operand_compare(op, lhs, rhs)
        raise ValueError(f"unsupported comparison in case_expression: {lhs} {op} {rhs}")

    def _value_test(self, op, v, t):
        kind = v[0]
        if kind == "jw":
            a, b = self.operand(v[1], "str"), self.operand(v[2], "str")
            self.emit("JW", self._op(a), self._op(b), op, t=t)
        elif kind in ("lev", "levratio"):
            a, b = self.operand(v[1], "str"), self.operand(v[2], "str")
            self.emit("LEV" if kind == "lev" else "LEVRATIO", self._op(a), self._op(b), op, t=t)
        elif kind == "len":
            a = self.operand(v[1], "str")
            self.emit("LEN", self._op(a), 0, op, t=t)
        elif kind in ("absdiff", "percdiff"):
            a, b = self.operand(v[1], "num"), self.operand(v[2], "num")
            self.emit("ABSDIFF" if kind == "absdiff" else "PERCDIFF", self._op(a), self._op(b), op, t=t)
        elif kind == "absdatediff":
            # abs(datediff(a, b)) cmp t = abs(day(a) - day(b)) cmp t over the operands' day numbers
            a, b = self._day_operand(v[1], 0), self._day_operand(v[2], 0)
            self.emit("ABSDIFF", self._op(a), self._op(b), op, t=t)
        elif kind == "datediff":
            # datediff(a, b) cmp t  <=>  day(a) cmp day(b) + t  (day numbers are integers: exact in fp64).  The shift
            # is folded into b's derived column (date_add); a non-integral t first becomes the integral threshold
            # with the same truth value for every integer
            if t != int(t):
                if op in ("=", "!="):
                    raise ValueError(f"datediff(...) {op} {t}: a non-integral day count")
                t = float(np.floor(t) if op in ("<=", ">") else np.ceil(t))
            a, b = self._day_operand(v[1], 0), self._day_operand(v[2], int(t))
            self.emit("NUM_CMP", self._op(a), self._op(b), op)
        else:
            raise ValueError(f"unsupported value expression {kind}")

    def _operand_compare(self, op, lhs, rhs):
        def natural(node):
            inner = node
            if isinstance(inner, Func) and inner.name in ("substr", "substring"):
                return "str"
            if D.is_derived(inner):
                return D.form_of(self._derived_neutral(inner)[0], self.schema.form)
            if isinstance(inner, Func):
                inner = inner.args[0]
                if D.is_derived(inner):
                    return D.form_of(self._derived_neutral(inner)[0], self.schema.form)
            if isinstance(inner, Lit):
                return "str" if isinstance(inner.value, str) else "num"
            name, _ = self._column_ref(inner)
            return self.schema.form(name)

        fl, fr = natural(lhs), natural(rhs)
        form = "str" if (fl == "str" and fr == "str") else "num"
        a, b = self.operand(lhs, form), self.operand(rhs, form)
        self.emit("STR_CMP" if form == "str" else "NUM_CMP", self._op(a), self._op(b), op)


def _is_number(node):
    return isinstance(node, Lit) and isinstance(node.value, (int, float)) and not isinstance(node.value, bool)


def _strip_abs_diff(node):
    if isinstance(node, Func) and node.name == "abs" and len(node.args) == 1 and isinstance(node.args[0], Bin) \
            and node.args[0].op == "-":
        return node.args[0].a, node.args[0].b
    return None


def _classify(node):
    """('jw'|'lev'|'levratio'|'len'|'absdiff'|'percdiff', ...) or ('operand',)."""
    if isinstance(node, Func):
        if node.name == "jaro_winkler_sim" and len(node.args) == 2:
            return ("jw", node.args[0], node.args[1])
        if node.name == "levenshtein" and len(node.args) == 2:
            return ("lev", node.args[0], node.args[1])
        if node.name in ("length", "char_length", "character_length") and len(node.args) == 1:
            return ("len", node.args[0])
        ad = _strip_abs_diff(node)
        if ad:
            return ("absdiff", ad[0], ad[1])
        if node.name == "datediff" and len(node.args) == 2:
            return ("datediff", node.args[0], node.args[1])
        if (node.name == "abs" and len(node.args) == 1 and isinstance(node.args[0], Func)
                and node.args[0].name == "datediff" and len(node.args[0].args) == 2):
            return ("absdatediff", node.args[0].args[0], node.args[0].args[1])
        if node.name in ("substr", "substring", "ifnull", "coalesce", "nvl") or D.is_derived(node):
            return ("operand",)
        raise ValueError(f"unsupported function {node.name}() in case_expression")
    if isinstance(node, Bin) and node.op == "/":
        # levenshtein(a, b) / ((length(a) + length(b)) / 2)
        if isinstance(node.a, Func) and node.a.name == "levenshtein" and len(node.a.args) == 2:
            a, b = node.a.args
            d = node.b
            if (isinstance(d, Bin) and d.op == "/" and _is_number(d.b) and float(d.b.value) == 2.0
                    and isinstance(d.a, Bin) and d.a.op == "+"
                    and isinstance(d.a.a, Func) and d.a.a.name == "length" and d.a.a.args == (a,)
                    and isinstance(d.a.b, Func) and d.a.b.name == "length" and d.a.b.args == (b,)):
                return ("levratio", a, b)
        # abs(a - b) / abs(case when a > b then a else b end)
        ad = _strip_abs_diff(node.a)
        if ad and isinstance(node.b, Func) and node.b.name == "abs" and len(node.b.args) == 1:
            c = node.b.args[0]
            a, b = ad
            if (isinstance(c, Case) and len(c.whens) == 1 and c.whens[0][0] == Bin(">", a, b)
                    and c.whens[0][1] == a and c.else_ == b):
                return ("percdiff", a, b)
        raise ValueError(f"unsupported arithmetic in case_expression: {node}")
    if isinstance(node, (Col, Lit)):
        return ("operand",)
    raise ValueError(f"unsupported expression in case_expression: {node}")


def _level(node, num_levels, what):
    if not (isinstance(node, Lit) and isinstance(node.value, int) and not isinstance(node.value, bool)):
        raise ValueError(f"{what} of a case_expression must be an integer literal, got {node}")
    v = node.value
    if not -1 <= v < num_levels:
        raise ValueError(f"{what} {v} is outside -1..{num_levels - 1} (num_levels = {num_levels})")
    return v


_NULL_EXACT = ("lower", "lcase", "upper", "ucase", "trim", "ltrim", "rtrim")


def _null_exact_of(node):
    """(F, column) when node = F(<column>) for a chain F of lower / upper / trim functions: F(x) is NULL
    exactly when x is (Spark's string functions of one argument)."""
    chain = []
    while isinstance(node, Func) and node.name in _NULL_EXACT and len(node.args) == 1:
        chain.append(node.name)
        node = node.args[0]
    return (tuple(chain), node) if chain and isinstance(node, Col) else None


def _guard_on_derived(tree: Case) -> Case:
    """`WHEN x_l IS NULL OR x_r IS NULL` followed by tests that read x only as F(x_l) / F(x_r), for one
    null-exact chain F (lower / upper / trim ...): the guard is rewritten onto F(x_l) / F(x_r) (the same
    truth value for every row), so the column keeps the templates' shape over the derived column and
    runs through the filter kernel (spk_gammas classify_simple) instead of the interpreter."""
    if not tree.whens:
        return tree
    cond, val = tree.whens[0]
    if not (isinstance(cond, Bin) and cond.op == "or" and isinstance(cond.a, IsNull) and isinstance(cond.b, IsNull)
            and not cond.a.negated and not cond.b.negated and isinstance(cond.a.a, Col) and isinstance(cond.b.a, Col)):
        return tree
    xs = {cond.a.a, cond.b.a}
    found = set()
    ok = [True]

    def walk(n):
        if isinstance(n, Col):
            if n in xs:
                ok[0] = False  # a bare reference to x
            return
        ne = _null_exact_of(n)
        if ne is not None and ne[1] in xs:
            found.add(ne[0])
            return
        if isinstance(n, Func):
            for a in n.args:
                walk(a)
        elif isinstance(n, Bin):
            walk(n.a)
            walk(n.b)
        elif isinstance(n, Un):
            walk(n.a)
        elif isinstance(n, IsNull):
            walk(n.a)
        elif isinstance(n, Case):
            for c, v in n.whens:
                walk(c)
                walk(v)
            if n.else_ is not None:
                walk(n.else_)

    for c, v in tree.whens[1:]:
        walk(c)
    if not ok[0] or len(found) != 1:
        return tree
    chain = found.pop()

    def wrap(col):
        for name in reversed(chain):
            col = Func(name, (col,))
        return col

    guard = Bin("or", IsNull(wrap(cond.a.a)), IsNull(wrap(cond.b.a)))
    return Case(((guard, val),) + tuple(tree.whens[1:]), tree.else_)


def compile_comparisons(settings: dict, schema: Schema) -> CompiledComparisons:
    b = _ProgramBuilder(schema)
    programs, names, n_levels = [], [], []
    for col in settings["comparison_columns"]:
        name = col["col_name"] if "col_name" in col else col["custom_name"]
        L = int(col["num_levels"])
        tree = parse(col["case_expression"])
        if not isinstance(tree, Case):
            raise ValueError(f"case_expression for {name} is not a CASE expression")
        tree = _guard_on_derived(tree)
        first_when = len(b.whens)
        for cond, val in tree.whens:
            start = len(b.instrs)
            b.predicate(cond)
            n = len(b.instrs) - start
            if n > 16:
                raise ValueError(f"a WHEN condition of {name} is too long for the device (max 16 terms)")
            b.whens.append((start, n, _level(val, L, "THEN value")))
        if tree.else_ is None:
            raise ValueError(f"case_expression for {name} has no ELSE branch")
        programs.append((L, _level(tree.else_, L, "ELSE value"), len(tree.whens), first_when))
        names.append(f"gamma_{name}")
        n_levels.append(L)
    prog = np.array(programs, dtype=N.PROGRAM_DTYPE)
    instrs = np.array(b.instrs, dtype=N.INSTR_DTYPE) if b.instrs else np.zeros(0, dtype=N.INSTR_DTYPE)
    wf = np.array([w[0] for w in b.whens], dtype=np.int32)
    wn = np.array([w[1] for w in b.whens], dtype=np.int32)
    wl = np.array([w[2] for w in b.whens], dtype=np.int32)
    return CompiledComparisons(prog, wf, wn, wl, instrs, b.operands, b.literals, n_levels, names, list(b.columns),
                               dict(b.derived))


# ---------------------------------------------------------------------------------------------
# blocking rules
# ---------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class KeyExpr:
    column: str                          # canonical column name
    transforms: Tuple[tuple, ...] = ()   # ("substr", pos, len) | ("lower",) | ("upper",) | ("trim",)


@dataclass
class RuleSpec:
    text: str
    terms: List[Tuple[KeyExpr, KeyExpr]]

    @property
    def symmetric(self) -> bool:
        return all(l == r for l, r in self.terms)


def _key_expr(node, schema: Schema):
    """(side, KeyExpr) for l.col / r.col under supported transforms."""
    transforms = []
    while isinstance(node, Func):
        if node.name in ("substr", "substring") and len(node.args) in (2, 3) and \
                all(isinstance(a, Lit) and isinstance(a.value, int) for a in node.args[1:]):
            transforms.append(("substr", node.args[1].value,
                               node.args[2].value if len(node.args) == 3 else 2 ** 31 - 1))
        elif node.name in ("lower", "upper", "trim") and len(node.args) == 1:
            transforms.append((node.name,))
        else:
            raise ValueError(f"unsupported function {node.name}() in a blocking rule")
        node = node.args[0]
    if not isinstance(node, Col) or node.qualifier not in ("l", "r"):
        raise ValueError("blocking rules compare l.<column> with r.<column> (optionally under substr / lower / "
                         f"upper / trim); got {node}")
    canon = schema.resolve(node.name)
    if canon is None:
        raise ValueError(f"column {node.name!r} used in a blocking rule is not in the input data")
    return node.qualifier, KeyExpr(canon, tuple(reversed(transforms)))


def compile_rule(text: str, schema: Schema) -> RuleSpec:
    terms = []
    for term in conjuncts(parse(text)):
        if not (isinstance(term, Bin) and term.op == "="):
            raise ValueError(f"blocking rule {text!r}: only conjunctions of equalities are supported on the device "
                             f"(found {term})")
        sa, ka = _key_expr(term.a, schema)
        sb, kb = _key_expr(term.b, schema)
        if sa == sb:
            raise ValueError(f"blocking rule {text!r}: each equality must compare an l.* with an r.* expression")
        terms.append((ka, kb) if sa == "l" else (kb, ka))
    return RuleSpec(text, terms)
