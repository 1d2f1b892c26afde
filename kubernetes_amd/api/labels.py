"""Label / field selectors.

Parity: `staging/src/k8s.io/apimachinery/pkg/labels/selector.go` (Requirement, Selector,
`Parse` string grammar), `staging/src/k8s.io/apimachinery/pkg/fields/selector.go`.

Extension over the reference (BASELINE config 5): `Gt`/`Lt` compare
*quantities*, not just integers, so a device selector such as
``amd.com/memory Gt 256Gi`` or ``amd.com/memory Gt 270000`` (MiB) both work. A plain
integer on both sides compares exactly like the reference's `strconv.ParseInt` path.
"""
from __future__ import annotations

import re
from typing import Iterable, Mapping

from .quantity import try_parse

IN, NOT_IN, EXISTS, DOES_NOT_EXIST = "in", "notin", "exists", "!"
EQUALS, DOUBLE_EQUALS, NOT_EQUALS, GT, LT = "=", "==", "!=", "gt", "lt"

# NodeSelectorOperator spellings used in PodSpec / ResourceSelector
NODE_OPS = {"In": IN, "NotIn": NOT_IN, "Exists": EXISTS, "DoesNotExist": DOES_NOT_EXIST, "Gt": GT, "Lt": LT}
LABEL_SELECTOR_OPS = {"In": IN, "NotIn": NOT_IN, "Exists": EXISTS, "DoesNotExist": DOES_NOT_EXIST}

_NAME_RE = re.compile(r"^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$")
_DNS1123_SUB = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")


class SelectorError(ValueError):
    pass


def is_qualified_name(key: str) -> bool:
    """`validation.IsQualifiedName`: optional DNS-1123 prefix + '/' + name (≤63)."""
    if not key:
        return False
    parts = key.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if not prefix or len(prefix) > 253 or not _DNS1123_SUB.match(prefix):
            return False
    else:
        return False
    return 0 < len(name) <= 63 and bool(_NAME_RE.match(name))


def is_valid_label_value(v: str) -> bool:
    return v == "" or (len(v) <= 63 and bool(_NAME_RE.match(v)))


def _num(v):
    """Quantity-aware numeric parse for Gt/Lt."""
    qv = try_parse(v)
    return None if qv is None else qv.value


class Requirement:
    __slots__ = ("key", "op", "values", "_num")

    def __init__(self, key: str, op: str, values: Iterable[str] = ()):
        values = [str(v) for v in (values or ())]
        if not is_qualified_name(key):
            raise SelectorError(f"invalid label key {key!r}")
        if op in (IN, NOT_IN):
            if not values:
                raise SelectorError("for 'in', 'notin' operators, values set can't be empty")
        elif op in (EQUALS, DOUBLE_EQUALS, NOT_EQUALS):
            if len(values) != 1:
                raise SelectorError("exact-match compatibility requires one single value")
        elif op in (EXISTS, DOES_NOT_EXIST):
            if values:
                raise SelectorError("values set must be empty for exists and does not exist")
        elif op in (GT, LT):
            if len(values) != 1:
                raise SelectorError("for 'Gt', 'Lt' operators, exactly one value is required")
            if _num(values[0]) is None:
                raise SelectorError(f"for 'Gt', 'Lt' operators, the value must be a number or quantity: {values[0]!r}")
        else:
            raise SelectorError(f"operator {op!r} is not recognized")
        self.key, self.op, self.values = key, op, values
        self._num = _num(values[0]) if op in (GT, LT) else None

    def matches(self, ls: Mapping[str, str]) -> bool:
        op = self.op
        if op in (IN, EQUALS, DOUBLE_EQUALS):
            return self.key in ls and ls[self.key] in self.values
        if op in (NOT_IN, NOT_EQUALS):
            return self.key not in ls or ls[self.key] not in self.values
        if op == EXISTS:
            return self.key in ls
        if op == DOES_NOT_EXIST:
            return self.key not in ls
        # GT / LT
        if self.key not in ls:
            return False
        v = _num(ls[self.key])
        if v is None:
            return False
        return v > self._num if op == GT else v < self._num

    def __str__(self):
        if self.op == EXISTS:
            return self.key
        if self.op == DOES_NOT_EXIST:
            return "!" + self.key
        if self.op in (IN, NOT_IN):
            return f"{self.key} {self.op} ({','.join(sorted(self.values))})"
        if self.op in (GT, LT):
            return f"{self.key}{'>' if self.op == GT else '<'}{self.values[0]}"
        return f"{self.key}{self.op}{self.values[0]}"


class Selector:
    __slots__ = ("reqs", "_nothing")

    def __init__(self, reqs=None, nothing=False):
        self.reqs = list(reqs or [])
        self._nothing = nothing

    def add(self, r: Requirement) -> "Selector":
        return Selector(self.reqs + [r])

    def matches(self, ls: Mapping[str, str] | None) -> bool:
        if self._nothing:
            return False
        ls = ls or {}
        for r in self.reqs:
            if not r.matches(ls):
                return False
        return True

    def empty(self) -> bool:
        return not self._nothing and not self.reqs

    def __str__(self):
        return ",".join(str(r) for r in self.reqs)


def everything() -> Selector:
    return Selector()


def nothing() -> Selector:
    return Selector(nothing=True)


def selector_from_set(s: Mapping[str, str] | None) -> Selector:
    return Selector([Requirement(k, EQUALS, [v]) for k, v in sorted((s or {}).items())])


_TOKEN = re.compile(r"\s*(!=|==|=|>|<|\(|\)|,|!|[^\s!=<>(),]+)")


def parse(s: str | None) -> Selector:
    """Parse the label selector string grammar (`labels.Parse`)."""
    if s is None or not s.strip():
        return everything()
    toks = []
    pos = 0
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise SelectorError(f"unable to parse selector {s!r}")
        toks.append(m.group(1))
        pos = m.end()
    reqs, i = [], 0

    def expect(tok):
        nonlocal i
        if i >= len(toks) or toks[i] != tok:
            raise SelectorError(f"expected {tok!r} in selector {s!r}")
        i += 1

    while i < len(toks):
        if toks[i] == "!":
            i += 1
            reqs.append(Requirement(toks[i], DOES_NOT_EXIST))
            i += 1
        else:
            key = toks[i]
            i += 1
            if i >= len(toks) or toks[i] == ",":
                reqs.append(Requirement(key, EXISTS))
            elif toks[i] in ("=", "==", "!="):
                op = toks[i]
                i += 1
                val = ""
                if i < len(toks) and toks[i] != ",":
                    val = toks[i]
                    i += 1
                reqs.append(Requirement(key, op, [val]))
            elif toks[i] in (">", "<"):
                op = GT if toks[i] == ">" else LT
                i += 1
                reqs.append(Requirement(key, op, [toks[i]]))
                i += 1
            elif toks[i].lower() in ("in", "notin"):
                op = toks[i].lower()
                i += 1
                expect("(")
                vals = []
                while i < len(toks) and toks[i] != ")":
                    if toks[i] != ",":
                        vals.append(toks[i])
                    i += 1
                expect(")")
                reqs.append(Requirement(key, op, vals))
            else:
                raise SelectorError(f"unexpected token {toks[i]!r} in selector {s!r}")
        if i < len(toks):
            expect(",")
    return Selector(reqs)


def node_selector_requirements_as_selector(reqs) -> Selector:
    """`NodeSelectorRequirementsAsSelector` / fork `ExtendedRequirementsAsSelector`
    (pkg/apis/core/v1/helper/helpers.go:465-498). Empty → Nothing (reference quirk kept:
    callers treat an empty affinity as match-all before calling)."""
    if not reqs:
        return nothing()
    out = []
    for r in reqs:
        op = NODE_OPS.get(r.get("operator"))
        if op is None:
            raise SelectorError(f"{r.get('operator')!r} is not a valid node selector operator")
        out.append(Requirement(r.get("key", ""), op, r.get("values") or []))
    return Selector(out)


def label_selector_as_selector(ls) -> Selector:
    """metav1.LabelSelectorAsSelector: nil → Nothing, {} → Everything."""
    if ls is None:
        return nothing()
    if not ls.get("matchLabels") and not ls.get("matchExpressions"):
        return everything()
    reqs = [Requirement(k, EQUALS, [v]) for k, v in sorted((ls.get("matchLabels") or {}).items())]
    for e in ls.get("matchExpressions") or []:
        op = LABEL_SELECTOR_OPS.get(e.get("operator"))
        if op is None:
            raise SelectorError(f"{e.get('operator')!r} is not a valid pod selector operator")
        reqs.append(Requirement(e["key"], op, e.get("values") or []))
    return Selector(reqs)


# ---------------------------------------------------------------------------
# field selectors (fields.ParseSelector): only =, ==, != on flat keys
class FieldSelector:
    __slots__ = ("terms",)

    def __init__(self, terms):
        self.terms = terms  # list of (key, op, value)

    def matches(self, fields: Mapping[str, str]) -> bool:
        for k, op, v in self.terms:
            fv = fields.get(k, "")
            if op == "!=":
                if fv == v:
                    return False
            elif fv != v:
                return False
        return True

    def empty(self):
        return not self.terms

    def requires(self, key):
        for k, op, v in self.terms:
            if k == key and op != "!=":
                return v
        return None


def parse_field_selector(s: str | None) -> FieldSelector:
    terms = []
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        for op in ("!=", "==", "="):
            if op in part:
                k, v = part.split(op, 1)
                terms.append((k.strip(), "!=" if op == "!=" else "=", v.strip()))
                break
        else:
            raise SelectorError(f"invalid field selector term {part!r}")
    return FieldSelector(terms)


def selector_to_string(sel) -> str:
    """A LabelSelector (or a plain label map, as RC selectors are) in the query-string form
    `metav1.FormatLabelSelector` prints (`a=b,c in (d,e),!f`)."""
    if not sel:
        return ""
    if "matchLabels" not in sel and "matchExpressions" not in sel:
        sel = {"matchLabels": sel}
    parts = [f"{k}={v}" for k, v in sorted((sel.get("matchLabels") or {}).items())]
    for e in sel.get("matchExpressions") or ():
        op = e.get("operator")
        vals = ",".join(e.get("values") or ())
        if op == "In":
            parts.append(f"{e['key']} in ({vals})")
        elif op == "NotIn":
            parts.append(f"{e['key']} notin ({vals})")
        elif op == "Exists":
            parts.append(e["key"])
        elif op == "DoesNotExist":
            parts.append(f"!{e['key']}")
    return ",".join(parts)
