"""Kubernetes protobuf wire / etcd storage format for every served kind, driven by the schema
table generated from the reference's `generated.proto` files (`hack/gen_proto_schema.py` ->
`api/generated/k8s_proto_schema.json`), including the fork's ResourceV2 fields.

Parity:
  * envelope: `staging/src/k8s.io/apimachinery/pkg/runtime/serializer/protobuf/protobuf.go:42`
    (magic `0x6b 0x38 0x73 0x00`) + `runtime.Unknown{typeMeta=1{apiVersion=1,kind=2}, raw=2,
    contentEncoding=3, contentType=4}` (`staging/src/k8s.io/apimachinery/pkg/runtime/types.go:112-124`);
  * field numbers and names: `staging/src/k8s.io/api/<group>/<version>/generated.proto` (e.g. the
    fork's Container 22, PodSpec 27, NodeStatus 11, ObjectReference 8 `extendedResourceBinding`);
    JSON names and inline embedding from the Go struct tags (`json:",inline"`: Volume.VolumeSource,
    Probe.Handler, ... whose fields appear at the parent's level in JSON);
  * value encodings (the types with custom JSON marshalling): meta/v1 Time / MicroTime
    `{seconds=1, nanos=2}` <-> RFC 3339, Duration `{duration=1}` <-> Go duration string,
    resource.Quantity `{string=1}`, intstr.IntOrString `{type=1, intVal=2, strVal=3}`,
    runtime.RawExtension / apiextensions JSON `{raw=1}` <-> any JSON value, the
    JSONSchemaPropsOr{Bool,Array,StringArray} unions, ExtraValue / Verbs string-slice wrappers,
    `bytes` <-> base64; maps as repeated entries in sorted key order, fields in field-number
    order (deterministic encoding).

Encoding is LOSSLESS OR AN ERROR: a field that is not in the kind's message raises
`ProtobufError` with its JSON path (the API server answers 422 instead of silently dropping it).
TypeMeta (`kind`, `apiVersion`) is not part of any message (Go's TypeMeta has no protobuf tag)
and travels in the envelope. Kinds without a message in the reference schema (custom resources,
`coordination.k8s.io` Leases) are stored as JSON, as the reference stores custom resources.

`encode_message` / `decode_message` here are the reference implementation; when the native
codec (`native/pbcodec/kamd_pbcodec.cc`, `_kamd_pbcodec`) is built the storage / wire entry
points use it — tests cross-check the two byte for byte.
"""
from __future__ import annotations

import base64
import datetime as _dt
import json
import os
import re

MAGIC = b"k8s\x00"
SCHEMA_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "generated", "k8s_proto_schema.json")

META = "k8s.io.apimachinery.pkg.apis.meta.v1."
TIME, MICROTIME, DURATION = META + "Time", META + "MicroTime", META + "Duration"
QUANTITY = "k8s.io.apimachinery.pkg.api.resource.Quantity"
INTORSTR = "k8s.io.apimachinery.pkg.util.intstr.IntOrString"
RAWEXT = "k8s.io.apimachinery.pkg.runtime.RawExtension"
_AX = "k8s.io.apiextensions_apiserver.pkg.apis.apiextensions.v1beta1."
JSONRAW, ORBOOL, ORARRAY, ORSTRARRAY = _AX + "JSON", _AX + "JSONSchemaPropsOrBool", _AX + "JSONSchemaPropsOrArray", \
    _AX + "JSONSchemaPropsOrStringArray"
# string-slice wrappers: `type ExtraValue []string` marshals as a JSON array
SLICES = {META + "Verbs"} | {f"k8s.io.api.{g}.ExtraValue" for g in (
    "authentication.v1", "authentication.v1beta1", "authorization.v1", "authorization.v1beta1", "certificates.v1beta1")}
SPECIAL = {TIME, MICROTIME, DURATION, QUANTITY, INTORSTR, RAWEXT, JSONRAW, ORBOOL, ORARRAY, ORSTRARRAY} | SLICES

# served kinds whose 1.9 message lives in another group/version of the same Go type
KIND_ALIASES = {"policy/v1beta1/PodSecurityPolicy": "extensions/v1beta1/PodSecurityPolicy",
                "policy/v1beta1/PodSecurityPolicyList": "extensions/v1beta1/PodSecurityPolicyList",
                "storage.k8s.io/v1beta1/VolumeAttachment": "storage.k8s.io/v1alpha1/VolumeAttachment",
                "storage.k8s.io/v1beta1/VolumeAttachmentList": "storage.k8s.io/v1alpha1/VolumeAttachmentList"}

VARINT_TYPES = {"bool", "int32", "int64", "uint32", "uint64"}


class ProtobufError(ValueError):
    def __init__(self, msg, path=""):
        super().__init__(f"{path}: {msg}" if path else msg)
        self.path = path


class _Field:
    __slots__ = ("json", "num", "label", "type", "key", "inline", "tag", "wt")

    def __init__(self, json_name, num, label, typ, key, inline):
        self.json, self.num, self.label, self.type, self.key, self.inline = json_name, num, label, typ, key, inline
        scalar_wt = 0 if typ in VARINT_TYPES else (1 if typ == "double" else 2)
        # packed repeated scalars are never used by the k8s protos (proto2, no [packed=true])
        self.wt = 2 if label == "map" else scalar_wt
        self.tag = _varint((num << 3) | self.wt)


class Schema:
    def __init__(self, path=SCHEMA_PATH):
        with open(path) as f:
            raw = json.load(f)
        self.kinds = dict(raw["kinds"])
        for alias, target in KIND_ALIASES.items():
            if target in self.kinds:
                self.kinds.setdefault(alias, self.kinds[target])
        self.fields: dict[str, list[_Field]] = {}
        for name, fs in raw["messages"].items():
            self.fields[name] = sorted((_Field(*f) for f in fs), key=lambda f: f.num)
        self.by_num = {m: {f.num: f for f in fs} for m, fs in self.fields.items()}
        # JSON key -> field (inline embedded messages contribute their keys to the parent)
        self.by_json: dict[str, dict[str, tuple]] = {}
        for m in self.fields:
            self.by_json[m] = self._json_map(m, ())

    def _json_map(self, m, chain):
        out = {}
        for f in self.fields[m]:
            if f.inline:
                for k, (ff, ch) in self._json_map(f.type, chain + (f,)).items():
                    out.setdefault(k, (ff, ch))
            else:
                out[f.json] = (f, chain)
        return out

    def message_for(self, api_version, kind):
        g = api_version if "/" in api_version else ("" if api_version == "v1" else api_version)
        key = f"{api_version}/{kind}" if g else f"v1/{kind}"
        return self.kinds.get(key)


_SCHEMA: Schema | None = None


def schema() -> Schema:
    global _SCHEMA
    if _SCHEMA is None:
        _SCHEMA = Schema()
    return _SCHEMA


# ---------------------------------------------------------------------------
# wire primitives
def _varint(n: int) -> bytes:
    if n < 0:
        n += 1 << 64
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(num, wt):
    return _varint((num << 3) | wt)


def _ld(num, payload: bytes) -> bytes:
    return _key(num, 2) + _varint(len(payload)) + payload


def _read_varint(buf, i):
    shift = n = 0
    while True:
        if i >= len(buf):
            raise ProtobufError("truncated varint")
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7
        if shift > 63:
            raise ProtobufError("varint too long")


def _fields(buf):
    i, n = 0, len(buf)
    while i < n:
        k, i = _read_varint(buf, i)
        num, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            v = buf[i:i + ln]
            if len(v) != ln:
                raise ProtobufError("truncated field")
            i += ln
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ProtobufError(f"unsupported wire type {wt}")
        yield num, wt, v


def _signed(v, bits=64):
    v &= (1 << 64) - 1
    if bits == 32:
        v &= 0xFFFFFFFF
        return v - (1 << 32) if v >= 1 << 31 else v
    return v - (1 << 64) if v >= 1 << 63 else v


# ---------------------------------------------------------------------------
# special types
_RFC3339 = re.compile(r"^(\d{4})-(\d{2})-(\d{2})[Tt ](\d{2}):(\d{2}):(\d{2})(\.\d+)?([Zz]|[+-]\d{2}:\d{2})$")


def parse_time(s, path=""):
    m = _RFC3339.match(s) if isinstance(s, str) else None
    if not m:
        raise ProtobufError(f"{s!r} is not an RFC 3339 time", path)
    y, mo, d, h, mi, se = (int(m.group(k)) for k in range(1, 7))
    frac = m.group(7) or ""
    nanos = int((frac[1:] + "000000000")[:9]) if frac else 0
    tz = m.group(8)
    off = 0 if tz in ("Z", "z") else (1 if tz[0] == "+" else -1) * (int(tz[1:3]) * 3600 + int(tz[4:6]) * 60)
    dt = _dt.datetime(y, mo, d, h, mi, se, tzinfo=_dt.timezone.utc)
    return int(dt.timestamp()) - off, nanos


def format_time(sec, nanos, micro=False):
    t = _dt.datetime.fromtimestamp(sec, _dt.timezone.utc)
    if micro:
        return t.strftime("%Y-%m-%dT%H:%M:%S") + f".{nanos // 1000:06d}Z"
    return t.strftime("%Y-%m-%dT%H:%M:%SZ")


_DUR = re.compile(r"(\d+(?:\.\d*)?|\.\d+)(ns|us|µs|ms|s|m|h)")
_DUR_NS = {"ns": 1, "us": 1000, "µs": 1000, "ms": 1_000_000, "s": 1_000_000_000, "m": 60_000_000_000, "h": 3_600_000_000_000}


def parse_duration(s, path=""):
    if not isinstance(s, str) or not s:
        raise ProtobufError(f"{s!r} is not a duration", path)
    neg = s.startswith("-")
    body = s.lstrip("+-")
    if body == "0":
        return 0
    pos, total = 0, 0
    for m in _DUR.finditer(body):
        if m.start() != pos:
            raise ProtobufError(f"{s!r} is not a duration", path)
        total += round(float(m.group(1)) * _DUR_NS[m.group(2)])
        pos = m.end()
    if pos != len(body):
        raise ProtobufError(f"{s!r} is not a duration", path)
    return -total if neg else total


def format_duration(ns):
    """Go's time.Duration.String()."""
    if ns == 0:
        return "0s"
    neg, ns = ns < 0, abs(ns)
    if ns < 1_000_000_000:
        for unit, div in (("ms", 1_000_000), ("µs", 1000), ("ns", 1)):
            if ns >= div:
                v = ns / div
                out = (f"{v:.9f}".rstrip("0").rstrip(".")) + unit
                return ("-" if neg else "") + out
    h, rem = divmod(ns, 3_600_000_000_000)
    m, rem = divmod(rem, 60_000_000_000)
    s = rem / 1e9
    out = (f"{h}h" if h else "") + (f"{m}m" if h or m else "") + (f"{s:.9f}".rstrip("0").rstrip(".") + "s")
    return ("-" if neg else "") + out


# ---------------------------------------------------------------------------
# encode
def _scalar(f: _Field, v, path):
    t = f.type
    if t == "string":
        if not isinstance(v, str):
            raise ProtobufError(f"expected a string, got {type(v).__name__}", path)
        b = v.encode()
        return f.tag + _varint(len(b)) + b
    if t == "bool":
        if not isinstance(v, bool):
            raise ProtobufError(f"expected a boolean, got {type(v).__name__}", path)
        return f.tag + (b"\x01" if v else b"\x00")
    if t in ("int32", "int64", "uint32", "uint64"):
        if isinstance(v, bool) or not isinstance(v, (int, float)) or (isinstance(v, float) and not v.is_integer()):
            raise ProtobufError(f"expected an integer, got {v!r}", path)
        return f.tag + _varint(int(v))
    if t == "bytes":
        if not isinstance(v, str):
            raise ProtobufError("expected a base64 string", path)
        try:
            b = base64.b64decode(v, validate=True)
        except ValueError:
            raise ProtobufError("invalid base64", path) from None
        return f.tag + _varint(len(b)) + b
    if t == "double":
        import struct
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            raise ProtobufError(f"expected a number, got {v!r}", path)
        return f.tag + struct.pack("<d", float(v))
    raise ProtobufError(f"unsupported scalar type {t}", path)


def _special(t, v, path) -> bytes:
    """The payload (message body) of a special-typed value."""
    if t in (TIME, MICROTIME):
        sec, nanos = parse_time(v, path)
        if t == TIME:
            nanos = 0      # metav1.Time is second-precision on the wire (RFC 3339 without fraction)
        out = _key(1, 0) + _varint(sec)
        if nanos:
            out += _key(2, 0) + _varint(nanos)
        return out
    if t == QUANTITY:
        if isinstance(v, bool) or not isinstance(v, (str, int, float)):
            raise ProtobufError(f"expected a quantity, got {v!r}", path)
        s = v if isinstance(v, str) else (str(int(v)) if float(v).is_integer() else repr(v))
        return _ld(1, s.encode())
    if t == INTORSTR:
        if isinstance(v, bool) or not isinstance(v, (int, str)):
            raise ProtobufError(f"expected an int or a string, got {v!r}", path)
        if isinstance(v, int):
            return _key(1, 0) + _varint(0) + _key(2, 0) + _varint(v) + _ld(3, b"")
        return _key(1, 0) + _varint(1) + _key(2, 0) + _varint(0) + _ld(3, v.encode())
    if t == DURATION:
        return _key(1, 0) + _varint(parse_duration(v, path))
    if t in (RAWEXT, JSONRAW):
        return _ld(1, json.dumps(v, separators=(",", ":"), ensure_ascii=False).encode())
    if t in SLICES:
        if not isinstance(v, list) or not all(isinstance(x, str) for x in v):
            raise ProtobufError("expected a list of strings", path)
        return b"".join(_ld(1, x.encode()) for x in v)
    if t == ORBOOL:
        if isinstance(v, bool):
            return _key(1, 0) + (b"\x01" if v else b"\x00")
        return _key(1, 0) + b"\x01" + _ld(2, encode_message(_AX + "JSONSchemaProps", v, path))
    if t == ORARRAY:
        if isinstance(v, list):
            return b"".join(_ld(2, encode_message(_AX + "JSONSchemaProps", x, f"{path}[{i}]")) for i, x in enumerate(v))
        return _ld(1, encode_message(_AX + "JSONSchemaProps", v, path))
    if t == ORSTRARRAY:
        if isinstance(v, list):
            return b"".join(_ld(2, str(x).encode()) for x in v)
        return _ld(1, encode_message(_AX + "JSONSchemaProps", v, path))
    raise ProtobufError(f"unsupported special type {t}", path)


def _value(f: _Field, v, path) -> bytes:
    t = f.type
    if t in SPECIAL:
        body = _special(t, v, path)
        return f.tag + _varint(len(body)) + body
    if "." in t:
        if not isinstance(v, dict):
            raise ProtobufError(f"expected an object, got {type(v).__name__}", path)
        body = encode_message(t, v, path)
        return f.tag + _varint(len(body)) + body
    return _scalar(f, v, path)


def _map_entry(f: _Field, k, v, path) -> bytes:
    kf = _Field("key", 1, "opt", f.key, "", False)
    vf = _Field("value", 2, "opt", f.type, "", False)
    if f.key in VARINT_TYPES:
        try:
            k = int(k)
        except ValueError:
            raise ProtobufError(f"map key {k!r} is not an integer", path) from None
    body = _scalar(kf, k, path) + _value(vf, v, f"{path}[{k}]")
    return f.tag + _varint(len(body)) + body


def encode_message(msg: str, obj: dict, path="") -> bytes:
    """obj (JSON form) -> message bytes. Raises ProtobufError on a field outside the schema."""
    s = schema()
    fields = s.fields.get(msg)
    if fields is None:
        raise ProtobufError(f"no protobuf message {msg}", path)
    jm = s.by_json[msg]
    # group the object's keys by the top-level field they encode into (inline chains)
    inline_parts: dict[int, dict] = {}
    direct = {}
    for k, v in obj.items():
        if v is None:
            continue
        ent = jm.get(k)
        if ent is None:
            if k in ("kind", "apiVersion"):
                continue          # TypeMeta: envelope only
            raise ProtobufError(f"field {k!r} is not part of {msg.rsplit('.', 1)[-1]} in the API schema",
                                f"{path}.{k}" if path else k)
        f, chain = ent
        if chain:
            inline_parts.setdefault(chain[0].num, {})[k] = v
        else:
            direct[f.num] = (f, v)
    out = bytearray()
    for f in fields:
        if f.inline:
            part = inline_parts.get(f.num)
            if part is not None:
                body = encode_message(f.type, part, path)
                out += f.tag + _varint(len(body)) + body
            continue
        ent = direct.get(f.num)
        if ent is None:
            continue
        _, v = ent
        p = f"{path}.{f.json}" if path else f.json
        if f.label == "rep":
            if not isinstance(v, list):
                raise ProtobufError(f"expected a list, got {type(v).__name__}", p)
            for i, x in enumerate(v):
                if x is None:
                    raise ProtobufError("null list element", f"{p}[{i}]")
                out += _value(f, x, f"{p}[{i}]")
        elif f.label == "map":
            if not isinstance(v, dict):
                raise ProtobufError(f"expected a map, got {type(v).__name__}", p)
            for k in sorted(v):
                if v[k] is None:
                    raise ProtobufError("null map value", f"{p}[{k}]")
                out += _map_entry(f, k, v[k], p)
        else:
            out += _value(f, v, p)
    return bytes(out)


# ---------------------------------------------------------------------------
# decode
def _decode_scalar(t, wt, v):
    if t == "string":
        return bytes(v).decode()
    if t == "bool":
        return bool(v)
    if t == "int32":
        return _signed(v, 32)
    if t in ("int64",):
        return _signed(v)
    if t in ("uint32", "uint64"):
        return v
    if t == "bytes":
        return base64.b64encode(bytes(v)).decode()
    if t == "double":
        import struct
        return struct.unpack("<d", bytes(v))[0]
    raise ProtobufError(f"unsupported scalar type {t}")


def _decode_special(t, v):
    if t in (TIME, MICROTIME):
        sec = nanos = 0
        for n, _, x in _fields(v):
            if n == 1:
                sec = _signed(x)
            elif n == 2:
                nanos = x
        return format_time(sec, nanos, t == MICROTIME)
    if t == QUANTITY:
        return next((bytes(x).decode() for n, _, x in _fields(v) if n == 1), "0")
    if t == INTORSTR:
        typ, iv, sv = 0, 0, ""
        for n, _, x in _fields(v):
            if n == 1:
                typ = x
            elif n == 2:
                iv = _signed(x, 32)
            elif n == 3:
                sv = bytes(x).decode()
        return iv if typ == 0 else sv
    if t == DURATION:
        return format_duration(next((_signed(x) for n, _, x in _fields(v) if n == 1), 0))
    if t in (RAWEXT, JSONRAW):
        raw = next((bytes(x) for n, _, x in _fields(v) if n == 1), b"")
        return json.loads(raw) if raw else None
    if t in SLICES:
        return [bytes(x).decode() for n, _, x in _fields(v) if n == 1]
    if t == ORBOOL:
        allows, sch = False, None
        for n, _, x in _fields(v):
            if n == 1:
                allows = bool(x)
            elif n == 2:
                sch = decode_message(_AX + "JSONSchemaProps", x)
        return sch if sch is not None else allows
    if t in (ORARRAY, ORSTRARRAY):
        sch, arr = None, []
        for n, _, x in _fields(v):
            if n == 1:
                sch = decode_message(_AX + "JSONSchemaProps", x)
            elif n == 2:
                arr.append(decode_message(_AX + "JSONSchemaProps", x) if t == ORARRAY else bytes(x).decode())
        return sch if sch is not None else arr
    raise ProtobufError(f"unsupported special type {t}")


def _decode_value(t, wt, v, depth=0):
    if t in SPECIAL:
        try:
            return _decode_special(t, v)
        except (TypeError, ValueError, UnicodeDecodeError) as e:
            if isinstance(e, ProtobufError):
                raise
            raise ProtobufError(f"malformed {t.rsplit('.', 1)[-1]}: {e}") from None
    if "." in t:
        return decode_message(t, v, None, depth + 1)
    try:
        return _decode_scalar(t, wt, v)
    except UnicodeDecodeError as e:
        raise ProtobufError(f"invalid UTF-8 in a string field: {e}") from None


MAX_DEPTH = 100    # nesting bound for untrusted input (recursive JSONSchemaProps, ...)


def _wire_of(t):
    return 0 if t in VARINT_TYPES else (1 if t == "double" else 2)


def _packed(t, wt, v):
    """A packed run of repeated varint / double scalars."""
    out, i = [], 0
    while i < len(v):
        if wt == 0:
            x, i = _read_varint(v, i)
        else:
            x = v[i:i + 8]
            if len(x) != 8:
                raise ProtobufError("truncated packed field")
            i += 8
        out.append(_decode_scalar(t, wt, x))
    return out


def decode_message(msg: str, buf, out=None, _depth=0) -> dict:
    """Decode one message. Every occurrence's wire type must match its field's type (a repeated
    varint/double field may also be packed): corrupt or hostile input raises ProtobufError, never
    a TypeError deeper down. Nesting is bounded by MAX_DEPTH."""
    if _depth > MAX_DEPTH:
        raise ProtobufError("protobuf nesting too deep")
    s = schema()
    byn = s.by_num.get(msg)
    if byn is None:
        raise ProtobufError(f"no protobuf message {msg}")
    out = {} if out is None else out
    for num, wt, v in _fields(buf):
        f = byn.get(num)
        if f is None:
            continue  # unknown field: skipped (forward compatible, as gogo-protobuf)
        if wt != f.wt and not (f.label == "rep" and wt == 2 and f.wt != 2):
            raise ProtobufError(f"wire type {wt} does not match the field's type", f.json)
        if f.inline:
            decode_message(f.type, v, out, _depth + 1)
        elif f.label == "rep":
            if wt == 2 and f.wt != 2:
                out.setdefault(f.json, []).extend(_packed(f.type, f.wt, v))
            else:
                out.setdefault(f.json, []).append(_decode_value(f.type, wt, v, _depth))
        elif f.label == "map":
            k = val = None
            kwt, ewt = _wire_of(f.key), (2 if "." in f.type else _wire_of(f.type))
            vwt = ewt
            for n2, w2, x in _fields(v):
                if (n2 == 1 and w2 != kwt) or (n2 == 2 and w2 != ewt):
                    raise ProtobufError("map entry: wrong wire type", f.json)
                if n2 == 1:
                    k = _decode_scalar(f.key, w2, x)
                elif n2 == 2:
                    val, vwt = x, w2
            if f.key in VARINT_TYPES:
                k = str(k)
            m = out.setdefault(f.json, {})
            if val is None:
                val = b"" if vwt == 2 else (bytes(8) if vwt == 1 else 0)
            m[k if k is not None else ""] = _decode_value(f.type, vwt, val, _depth)
        else:
            out[f.json] = _decode_value(f.type, wt, v, _depth)
    return out


# ---------------------------------------------------------------------------
# envelope
def encode_unknown(api_version: str, kind: str, raw: bytes) -> bytes:
    tm = _ld(1, api_version.encode()) + _ld(2, kind.encode())
    return MAGIC + _ld(1, tm) + _ld(2, raw) + _ld(3, b"") + _ld(4, b"")


def decode_unknown(data: bytes):
    if data[:4] != MAGIC:
        raise ProtobufError("missing k8s protobuf magic")
    api_version = kind = ""
    raw = b""
    for num, _, v in _fields(memoryview(data)[4:]):
        if num == 1:
            for n2, _, x in _fields(v):
                if n2 == 1:
                    api_version = bytes(x).decode()
                elif n2 == 2:
                    kind = bytes(x).decode()
        elif num == 2:
            raw = bytes(v)
    return api_version, kind, raw


def message_of(obj) -> str | None:
    return schema().message_for(obj.get("apiVersion", "v1") or "v1", obj.get("kind", ""))


_SUPPORTED: dict = {}


def supported(kind: str, api_version: str = "") -> bool:
    key = (kind, api_version)
    r = _SUPPORTED.get(key)
    if r is None:
        s = schema()
        if api_version:
            r = s.message_for(api_version, kind) is not None
        else:
            r = any(k.rsplit("/", 1)[-1] == kind for k in s.kinds)
        _SUPPORTED[key] = r
    return r


_NAT = []


def _native():
    if not _NAT:
        from ..native import pbcodec
        _NAT.append(pbcodec)
    return _NAT[0].codec()


def encode_object(obj: dict) -> bytes:
    kind, av = obj.get("kind", ""), obj.get("apiVersion", "v1") or "v1"
    msg = schema().message_for(av, kind)
    if msg is None:
        raise ProtobufError(f"no protobuf message for {av}/{kind}")
    nat = _native()
    if nat is not None:
        return nat.encode_object(obj, msg)
    return encode_unknown(av, kind, encode_message(msg, obj))


def decode_object(data: bytes) -> dict:
    nat = _native()
    if nat is not None:
        return nat.decode_object(data)
    api_version, kind, raw = decode_unknown(data)
    msg = schema().message_for(api_version, kind)
    if msg is None:
        raise ProtobufError(f"no protobuf message for {api_version}/{kind}")
    out = {"kind": kind, "apiVersion": api_version}
    out.update(decode_message(msg, raw))
    return out


# storage codec hooks (codec.StorageCodec)
def _alternates(obj):
    """Other versions of the object's kind in the reference schema, newest first: an object whose
    fields only exist in a later version (autoscaling/v1 HPA with v2beta1 `metrics`) is stored in
    that version's message, as the reference stores an HPA's metrics losslessly (its storage
    version carries them as an annotation; here the version that has the fields is chosen)."""
    from .meta import version_priority
    av, kind = obj.get("apiVersion", "v1") or "v1", obj.get("kind", "")
    group = av.rsplit("/", 1)[0] if "/" in av else ""
    out = []
    for key in schema().kinds:
        g, _, rest = key.rpartition("/")
        ver_group, _, ver = g.rpartition("/") if "/" in g else ("", "", g)
        if rest == kind and ver_group == group and f"{g}" != av:
            out.append((version_priority(ver), g))
    return [g for _, g in sorted(out, reverse=True)]


def encode_storage(obj):
    if message_of(obj) is None:
        from .codec import dumpb
        return dumpb(obj)          # custom resources / kinds outside the reference schema: JSON
    try:
        return encode_object(obj)
    except ProtobufError as first:
        for av in _alternates(obj):
            try:
                return encode_object(dict(obj, apiVersion=av))
            except ProtobufError:
                continue
        raise first


def decode_storage(data):
    obj = decode_object(data)
    from .meta import BY_KIND
    ri = BY_KIND.get(obj.get("kind", ""))
    if ri is not None and obj.get("apiVersion") != ri.group_version:
        obj["apiVersion"] = ri.group_version      # stored in another version of the same type
    return obj


# -- protobuf watch streams (`application/vnd.kubernetes.protobuf;stream=watch`) ----------------
WATCH_STREAM = "application/vnd.kubernetes.protobuf;stream=watch"


def envelope_with_rv(envelope: bytes, rv: str):
    """The stored envelope with metadata.resourceVersion set (etcd3 stores objects without
    it), or None when it is not a protobuf envelope of a known kind."""
    if envelope[:4] != MAGIC:
        return None
    nat = _native()
    if nat is not None:
        return nat.with_rv(envelope, rv)
    try:
        obj = decode_object(envelope)
    except ProtobufError:
        return None
    obj.setdefault("metadata", {})["resourceVersion"] = str(rv)
    api_version, kind, _ = decode_unknown(envelope)
    return encode_unknown(api_version, kind, encode_message(schema().message_for(api_version, kind), obj))


def to_json(envelope: bytes, rv) -> bytes:
    """A stored envelope as the object's JSON bytes with metadata.resourceVersion = rv."""
    nat = _native()
    if nat is not None:
        return nat.to_json(envelope, str(rv))
    from .codec import dumpb
    obj = decode_object(envelope)
    obj.setdefault("metadata", {})["resourceVersion"] = str(rv)
    return dumpb(obj)


def watch_frame(etype: str, raw: bytes) -> bytes:
    """One length-delimited metav1.WatchEvent frame (4-byte big-endian length) embedding `raw`
    (`runtime/serializer/protobuf/protobuf.go:436`, `endpoints/handlers/watch.go:166-226`)."""
    nat = _native()
    if nat is not None:
        return nat.watch_frame(etype, raw)
    ev = _ld(1, etype.encode()) + _ld(2, _ld(1, bytes(raw)))
    return len(ev).to_bytes(4, "big") + ev


MAX_WATCH_FRAME = 64 << 20


def decode_watch_frames(buf):
    """([(type, object)], bytes consumed) for the complete frames at the start of `buf`."""
    nat = _native()
    if nat is not None:
        return nat.decode_watch_frames(buf)
    from .meta import BY_KIND
    events, pos, n = [], 0, len(buf)
    mv = memoryview(buf)
    while n - pos >= 4:
        fl = int.from_bytes(bytes(mv[pos:pos + 4]), "big")
        if fl > MAX_WATCH_FRAME:
            raise ProtobufError("watch frame too large")
        if n - pos - 4 < fl:
            break
        etype, raw = None, b""
        for num, wt, v in _fields(mv[pos + 4:pos + 4 + fl]):
            if num == 1 and wt == 2:
                etype = bytes(v).decode()
            elif num == 2 and wt == 2:
                for n2, w2, x in _fields(v):
                    if n2 == 1 and w2 == 2:
                        raw = bytes(x)
        if etype is None:
            raise ProtobufError("malformed watch frame")
        if raw[:4] == MAGIC:
            obj = decode_object(raw)
            ri = BY_KIND.get(obj.get("kind", ""))
            if ri is not None:
                obj["apiVersion"] = ri.group_version     # the native codec's canonical version
        else:
            obj = json.loads(raw) if raw else None
        events.append((etype, obj))
        pos += 4 + fl
    return events, pos


def status_envelope(status: dict) -> bytes:
    """A metav1.Status as a protobuf envelope (`apiVersion: v1, kind: Status`), what client-go's
    protobuf stream decoder expects in an ERROR frame (watch.go:166-226 encodes the error
    object with the stream's serializer)."""
    return encode_object(dict(status, kind="Status", apiVersion="v1"))
