"""resource.Quantity — exact fixed-point quantities with Kubernetes suffix rules.

Behavioural parity with the reference's `staging/src/k8s.io/apimachinery/pkg/api/resource/quantity.go`
(parse: `ParseQuantity`, canonical form: `CanonicalizeBytes`, `Value()` rounds up,
`MilliValue()`), re-implemented on Python `Fraction` so comparisons used by the
scheduler's device selectors (`Gt`/`Lt` on `amd.com/memory=288Gi`) are exact.

Formats:
  * BinarySI   — Ki Mi Gi Ti Pi Ei   (powers of 1024)
  * DecimalSI  — n u m "" k M G T P E (powers of 1000)
  * DecimalExponent — 1e3, 12E-3
"""
from __future__ import annotations

import math
import re
from fractions import Fraction
from functools import lru_cache, total_ordering

BINARY_SI = "BinarySI"
DECIMAL_SI = "DecimalSI"
DECIMAL_EXPONENT = "DecimalExponent"

_BIN = {"Ki": 1, "Mi": 2, "Gi": 3, "Ti": 4, "Pi": 5, "Ei": 6}
_DEC = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
_DEC_BY_EXP = {v: k for k, v in _DEC.items()}
_BIN_BY_EXP = {v: k for k, v in _BIN.items()}

_RE = re.compile(r"^([+-]?(?:\d+\.?\d*|\.\d+))((?:[eE][+-]?\d+)|Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E|)$")

# Quantities are rounded up to nano precision, like the reference's infDec path.
_NANO = Fraction(1, 10 ** 9)


class QuantityError(ValueError):
    pass


@total_ordering
class Quantity:
    __slots__ = ("value", "format")

    def __init__(self, value, fmt: str = DECIMAL_SI):
        if isinstance(value, Quantity):
            self.value, self.format = value.value, value.format
            return
        if isinstance(value, str):
            q = parse_quantity(value)
            self.value, self.format = q.value, q.format
            return
        v = Fraction(value)
        # round away from zero to nano precision
        if v.denominator != 1 and (v / _NANO).denominator != 1:
            scaled = v / _NANO
            v = Fraction(math.ceil(scaled) if v > 0 else math.floor(scaled)) * _NANO
        self.value = v
        self.format = fmt

    # -- accessors -----------------------------------------------------
    def int_value(self) -> int:
        """Value() in the reference: rounded up to the nearest integer."""
        return math.ceil(self.value)

    def milli_value(self) -> int:
        return math.ceil(self.value * 1000)

    def is_zero(self) -> bool:
        return self.value == 0

    def __float__(self):
        return float(self.value)

    # -- arithmetic ----------------------------------------------------
    # Quantity.Add / Sub: a zero receiver adopts the operand's format (0 + 1Gi prints "1Gi")
    def __add__(self, o):
        fmt = o.format if self.value == 0 and isinstance(o, Quantity) else self.format
        return Quantity(self.value + _val(o), fmt)

    def __sub__(self, o):
        fmt = o.format if self.value == 0 and isinstance(o, Quantity) else self.format
        return Quantity(self.value - _val(o), fmt)

    def __neg__(self):
        return Quantity(-self.value, self.format)

    def __eq__(self, o):
        try:
            return self.value == _val(o)
        except (QuantityError, TypeError):
            return NotImplemented

    def __lt__(self, o):
        return self.value < _val(o)

    def __hash__(self):
        return hash(self.value)

    def __repr__(self):
        return f"Quantity({str(self)!r})"

    def __str__(self):
        return canonical(self.value, self.format)


def _val(o) -> Fraction:
    if isinstance(o, Quantity):
        return o.value
    if isinstance(o, str):
        return parse_quantity(o).value
    return Fraction(o)


@lru_cache(maxsize=8192)
def parse_quantity(s: str) -> Quantity:
    if not isinstance(s, str) or not s:
        raise QuantityError(f"quantities must match the regular expression: {s!r}")
    m = _RE.match(s.strip())
    if not m:
        raise QuantityError(f"quantities must match the regular expression: {s!r}")
    num, suf = m.group(1), m.group(2)
    base = Fraction(num)
    if suf in _BIN:
        return Quantity(base * (1024 ** _BIN[suf]), BINARY_SI)
    if suf and suf[0] in "eE" and len(suf) > 1:
        return Quantity(base * Fraction(10) ** int(suf[1:]), DECIMAL_EXPONENT)
    return Quantity(base * Fraction(10) ** _DEC[suf], DECIMAL_SI)


def canonical(v: Fraction, fmt: str) -> str:
    """Canonical string (reference `CanonicalizeBytes`): largest suffix that keeps an integer mantissa."""
    if v == 0:
        return "0"
    sign = "-" if v < 0 else ""
    a = -v if v < 0 else v
    if fmt == BINARY_SI and a.denominator == 1 and a >= 1024:
        n = a.numerator
        exp = 0
        while exp < 6 and n % 1024 == 0:
            n //= 1024
            exp += 1
        if exp > 0:
            return f"{sign}{n}{_BIN_BY_EXP[exp]}"
        # not a multiple of 1024: fall through to decimal form
    # decimal: find the exponent (multiple of 3) for an integer mantissa
    exp = 0
    m = a
    while m.denominator != 1 and exp > -9:
        m *= 1000
        exp -= 3
    if m.denominator != 1:
        m = Fraction(math.ceil(m))
    n = m.numerator
    while exp < 18 and n % 1000 == 0 and n != 0:
        n //= 1000
        exp += 3
    if fmt == DECIMAL_EXPONENT:
        return f"{sign}{n}" + (f"e{exp}" if exp else "")
    return f"{sign}{n}{_DEC_BY_EXP[exp]}"


def q(s) -> Quantity:
    return s if isinstance(s, Quantity) else Quantity(s)


def try_parse(s) -> Quantity | None:
    try:
        return parse_quantity(s) if isinstance(s, str) else Quantity(s)
    except (QuantityError, ValueError, TypeError, ZeroDivisionError):
        return None
