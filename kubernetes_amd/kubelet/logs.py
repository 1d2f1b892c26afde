"""Container log files in the CRI and docker-JSON formats (`pkg/kubelet/kuberuntime/logs/logs.go`).

A runtime behind the CRI (containerd, CRI-O) writes `<RFC3339Nano> <stdout|stderr> <tags> <log>`
lines, the tags a ':'-separated list whose first entry is `F` (full line) or `P` (partial: the
line continues in the next record, and carries no newline); dockershim wrote docker's JSON lines
`{"log", "stream", "time"}`. `read_logs` turns such a file back into what `kubectl logs` shows —
the log text of both streams, optionally prefixed by each record's timestamp, after `since`,
the last `tail` lines, at most `limit_bytes` bytes. The kubelet uses it when a container's log
file is in one of these formats; its own runtimes write the raw output.
"""
from __future__ import annotations

import calendar
import json
import re

STDOUT, STDERR = "stdout", "stderr"
_TS = re.compile(r"^(\d{4})-(\d\d)-(\d\d)T(\d\d):(\d\d):(\d\d)(?:\.(\d{1,9}))?(Z|[+-]\d\d:\d\d)$")


class LogFormatError(ValueError):
    pass


def parse_timestamp(s: str) -> float:
    """RFC3339Nano -> seconds since the epoch (nanosecond digits kept in the float)."""
    m = _TS.match(s)
    if not m:
        raise LogFormatError(f"unexpected timestamp format {s!r}")
    y, mo, d, h, mi, se, frac, tz = m.groups()
    t = calendar.timegm((int(y), int(mo), int(d), int(h), int(mi), int(se), 0, 0, 0))
    if frac:
        t += int(frac) / 10 ** len(frac)
    if tz != "Z":
        sign = 1 if tz[0] == "+" else -1
        t -= sign * (int(tz[1:3]) * 3600 + int(tz[4:6]) * 60)
    return t


def format_timestamp(s: str) -> str:
    """time.RFC3339Nano: the fraction without trailing zeros (none at all when zero)."""
    m = _TS.match(s)
    if not m or not m.group(7):
        return s
    frac = m.group(7).rstrip("0")
    head = s[:s.index(".")]
    return f"{head}.{frac}{m.group(8)}" if frac else f"{head}{m.group(8)}"


def parse_cri_log(line: bytes):
    """-> (timestamp string, stream, log bytes, partial)."""
    parts = line.split(b" ", 3)
    if len(parts) < 3:
        raise LogFormatError("timestamp, stream type or log tag is not found")
    ts = parts[0].decode(errors="replace")
    parse_timestamp(ts)
    stream = parts[1].decode(errors="replace")
    if stream not in (STDOUT, STDERR):
        raise LogFormatError(f"unexpected stream type {stream!r}")
    if len(parts) < 4:
        raise LogFormatError("log tag is not found")
    tags = parts[2].split(b":")
    partial = tags[0] == b"P"
    log = parts[3]
    if partial and log.endswith(b"\n"):
        log = log[:-1]
    return ts, stream, log, partial


def parse_docker_json_log(line: bytes):
    try:
        d = json.loads(line)
    except ValueError as e:
        raise LogFormatError(str(e)) from None
    if not isinstance(d, dict) or "log" not in d:
        raise LogFormatError("not a docker JSON log line")
    ts = str(d.get("time") or "")
    parse_timestamp(ts)
    return ts, str(d.get("stream") or ""), str(d["log"]).encode(), False


PARSERS = (parse_cri_log, parse_docker_json_log)


def get_parse_func(line: bytes):
    for p in PARSERS:
        try:
            p(line)
            return p
        except LogFormatError:
            continue
    raise LogFormatError(f"unsupported log format: {line[:80]!r}")


def read_logs(data: bytes, tail=None, since=None, timestamps=False, limit_bytes=None) -> bytes:
    """The `kubectl logs` bytes for a whole CRI / docker-JSON log file's content."""
    lines = data.splitlines(keepends=True)
    if not lines:
        return b""
    parse = get_parse_func(lines[0])
    if tail is not None and tail >= 0:
        lines = lines[len(lines) - tail:] if tail < len(lines) else lines
        if tail == 0:
            lines = []
    out, remain = [], (limit_bytes if limit_bytes and limit_bytes > 0 else None)
    for ln in lines:
        try:
            ts, _stream, log, _partial = parse(ln)
        except LogFormatError:
            continue
        if since is not None and parse_timestamp(ts) < since:
            continue
        chunk = (format_timestamp(ts).encode() + b" " + log) if timestamps else log
        if remain is not None:
            chunk = chunk[:remain]
            remain -= len(chunk)
        out.append(chunk)
        if remain is not None and remain <= 0:
            break
    return b"".join(out)


def is_structured(first_line: bytes) -> bool:
    try:
        get_parse_func(first_line)
        return True
    except LogFormatError:
        return False
