"""Container log parsing ported from `pkg/kubelet/kuberuntime/logs/logs_test.go` (TestParseLog,
TestWriteLogs, TestWriteLogsWithBytesLimit), plus ReadLogs over a whole CRI-format file."""
import pytest

from kubernetes_amd.kubelet.logs import (LogFormatError, format_timestamp, get_parse_func, parse_cri_log,
                                         parse_docker_json_log, parse_timestamp, read_logs)

TS = "2016-10-20T18:39:20.57606443Z"


@pytest.mark.parametrize("line,stream,log", [
    (b'{"log":"docker stdout test log","stream":"stdout","time":"' + TS.encode() + b'"}\n', "stdout",
     b"docker stdout test log"),
    (b'{"log":"docker stderr test log","stream":"stderr","time":"' + TS.encode() + b'"}\n', "stderr",
     b"docker stderr test log"),
    (TS.encode() + b" stdout F cri stdout test log\n", "stdout", b"cri stdout test log\n"),
    (TS.encode() + b" stderr F cri stderr test log\n", "stderr", b"cri stderr test log\n"),
    (TS.encode() + b" stdout P cri stdout partial test log\n", "stdout", b"cri stdout partial test log"),
    (TS.encode() + b" stdout P:TAG1:TAG2 cri stdout partial test log\n", "stdout", b"cri stdout partial test log"),
])
def test_parse_log(line, stream, log):
    ts, st, got, _ = get_parse_func(line)(line)
    assert (ts, st, got) == (TS, stream, log)


def test_unsupported_format():
    with pytest.raises(LogFormatError):
        get_parse_func(b"unsupported log format test log\n")
    with pytest.raises(LogFormatError):
        parse_cri_log(TS.encode() + b" stdin F x\n")
    with pytest.raises(LogFormatError):
        parse_docker_json_log(b'{"stream":"stdout"}')


def test_timestamps():
    assert parse_timestamp("1970-01-01T00:00:01.5Z") == 1.5
    assert parse_timestamp("1970-01-01T01:00:00+01:00") == 0
    assert format_timestamp("2016-10-20T18:39:20.500000000Z") == "2016-10-20T18:39:20.5Z"
    assert format_timestamp("2016-10-20T18:39:20.000000000Z") == "2016-10-20T18:39:20Z"


def _file(lines):
    return b"".join(f"1970-01-01T00:20:34.{i:09d}Z {s} F {t}\n".encode() for i, (s, t) in enumerate(lines))


def test_write_logs_streams_since_and_timestamps():
    data = _file([("stdout", "abcdefg"), ("stderr", "hijk")])
    assert read_logs(data) == b"abcdefg\nhijk\n"
    assert read_logs(data, since=1234 + 1) == b""                      # since after every record
    assert read_logs(data, timestamps=True) == (b"1970-01-01T00:20:34Z abcdefg\n"
                                                 b"1970-01-01T00:20:34.000000001Z hijk\n")


@pytest.mark.parametrize("n,limit,want", [(2, 1, b"a"), (2, 8, b"abcdefg\n"), (2, 10, b"abcdefg\nab"),
                                          (2, 100, b"abcdefg\nabcdefg\n")])
def test_write_logs_with_bytes_limit(n, limit, want):
    data = _file([("stdout", "abcdefg")] * n)
    assert read_logs(data, limit_bytes=limit) == want


def test_tail_lines():
    data = _file([("stdout", f"line{i}") for i in range(5)])
    assert read_logs(data, tail=2) == b"line3\nline4\n"
    assert read_logs(data, tail=0) == b""
