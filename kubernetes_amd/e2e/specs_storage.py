"""Storage conformance specs, the remaining `ConformanceIt` cases of the reference's
`test/e2e/common/empty_dir.go` (every (user, mode, medium) permutation and the volume-mode checks)
and `test/e2e/common/projected.go` (the secret, configMap and downwardAPI sources of a projected
volume: default/item modes, mappings, non-root readers with fsGroup, multiple volumes, optional
and live updates, resource fields). Helpers and conventions are those of `specs_common`.
"""
from __future__ import annotations

from .framework import conformance
from .specs_common import (SYNC_WAIT, _RES, _at, _b64, _cm, _lines, _log_contains, _mount, _pod, _res_item,
                           _run_and_log, _secret)

# ---------------------------------------------------------------------------------------------
# EmptyDir (empty_dir.go): (user, file mode, medium) permutations not in specs_common


def _ed_spec(tag, user, mode, medium):
    non_root = user == "non-root"

    async def spec(f):
        vol = _at("test-volume", "/test-volume", "test-file")
        cmd = (f"echo mount-tester new file > {vol} && chmod {mode} {vol} && stat -c %a {vol} && cat {vol} && "
               f"stat -c %a $(dirname {vol})")
        p = _pod(f"ed-{tag}", cmd, **({"securityContext": {"runAsUser": 1001}} if non_root else {}))
        _mount(p, "test-volume", {"emptyDir": {"medium": "Memory"} if medium == "tmpfs" else {}}, "/test-volume")
        out = _lines(await _run_and_log(f, p))
        assert out[:3] == [mode.lstrip("0"), "mount-tester new file", "777"], out
    spec.__name__ = f"emptydir_{tag}"
    return conformance(f"EmptyDir volumes should support ({user},{mode},{medium})")(spec)


for _i, (_u, _m, _md) in enumerate((("root", "0666", "default"), ("root", "0777", "default"),
                                    ("non-root", "0644", "default"), ("non-root", "0666", "default"),
                                    ("root", "0644", "tmpfs"), ("root", "0777", "tmpfs"),
                                    ("non-root", "0666", "tmpfs"), ("non-root", "0777", "tmpfs"))):
    _ed_spec(f"p{_i}", _u, _m, _md)


async def _ed_mode(f, name, medium):
    vol = _at("test-volume", "/test-volume", ".")
    p = _pod(name, f"stat -c %a {vol}; stat -f -c %T {vol}")
    _mount(p, "test-volume", {"emptyDir": {"medium": "Memory"} if medium else {}}, "/test-volume")
    return _lines(await _run_and_log(f, p))


@conformance("EmptyDir volumes volume on default medium should have the correct mode")
async def emptydir_default_mode(f):
    out = await _ed_mode(f, "edmode", None)
    assert out[0] == "777", out


@conformance("EmptyDir volumes volume on tmpfs should have the correct mode")
async def emptydir_tmpfs_mode(f):
    out = await _ed_mode(f, "edtmpfs", "Memory")
    # a memory-backed emptyDir is a tmpfs mount where the kubelet may mount (root); an
    # unprivileged kubelet falls back to a node-local directory of the same mode
    assert out[0] == "777", out
    pod = await f.client.get("pods", "edtmpfs", f.ns)
    assert pod["status"]["phase"] == "Succeeded"


# ---------------------------------------------------------------------------------------------
# Projected secret (projected.go:42-206)
def _psec(name, cmd, items=None, mode=None, secret="sec", **pod_extra):
    src = {"secret": {"name": secret}}
    if items:
        src["secret"]["items"] = items
    prj = {"sources": [src]}
    if mode is not None:
        prj["defaultMode"] = mode
    return _mount(_pod(name, cmd, **pod_extra), "p", {"projected": prj}, "/etc/projected-secret-volume")


def _pat(rel):
    return _at("p", "/etc/projected-secret-volume", rel)


@conformance("Projected secret should be consumable from pods in volume")
async def psec_volume(f):
    await _secret(f)
    assert _lines(await _run_and_log(f, _psec("psv", f"cat {_pat('data-1')}"))) == ["value-1"]


@conformance("Projected secret should be consumable from pods in volume with defaultMode set")
async def psec_default_mode(f):
    await _secret(f)
    out = _lines(await _run_and_log(f, _psec("psdm", f"stat -c %a {_pat('data-1')}; cat {_pat('data-1')}",
                                                 mode=0o400)))
    assert out == ["400", "value-1"], out


@conformance("Projected secret should be consumable from pods in volume as non-root with defaultMode and fsGroup set")
async def psec_non_root_fsgroup(f):
    await _secret(f)
    p = _psec("psnr", f"id -u; stat -c '%a %g' {_pat('data-1')}; cat {_pat('data-1')}", mode=0o440,
              securityContext={"runAsUser": 1000, "fsGroup": 1001})
    out = _lines(await _run_and_log(f, p))
    assert out == ["1000", "440 1001", "value-1"], out


@conformance("Projected secret should be consumable from pods in volume with mappings and Item Mode set")
async def psec_item_mode(f):
    await _secret(f)
    p = _psec("psim", f"stat -c %a {_pat('new-path-data-1')}; cat {_pat('new-path-data-1')}",
              items=[{"key": "data-1", "path": "new-path-data-1", "mode": 0o400}])
    assert _lines(await _run_and_log(f, p)) == ["400", "value-1"]


@conformance("Projected secret should be consumable in multiple volumes in a pod")
async def psec_multiple(f):
    await _secret(f)
    p = _pod("psmulti", f"cat {_at('a', '/etc/a', 'data-1')}; echo; cat {_at('b', '/etc/b', 'data-1')}")
    _mount(p, "a", {"projected": {"sources": [{"secret": {"name": "sec"}}]}}, "/etc/a")
    _mount(p, "b", {"projected": {"sources": [{"secret": {"name": "sec"}}]}}, "/etc/b")
    assert _lines(await _run_and_log(f, p)) == ["value-1", "value-1"]


async def _optional_updates(f, kind, name):
    """`optional updates should be reflected in volume`: one optional source is deleted, one is
    created after the pod started, one is updated; the volumes follow each change."""
    def obj(n, v):
        if kind == "secrets":
            return {"metadata": {"name": n}, "data": {"k": _b64(v)}}
        return {"metadata": {"name": n}, "data": {"k": v}}

    def src(n):
        return {"secret": {"name": n, "optional": True}} if kind == "secrets" else \
            {"configMap": {"name": n, "optional": True}}
    await f.client.create(kind, obj("del", "value-del"), f.ns)
    await f.client.create(kind, obj("upd", "value-upd-1"), f.ns)
    loop = "; ".join(f"cat {_at(v, '/etc/' + v, 'k')} 2>/dev/null || echo {v}-missing; echo"
                     for v in ("d", "u", "c"))
    p = _pod(name, f"while true; do {loop}; sleep 1; done", restart="Always")
    for v, n in (("d", "del"), ("u", "upd"), ("c", "create")):
        _mount(p, v, {"projected": {"sources": [src(n)]}}, "/etc/" + v)
    await f.client.create("pods", p, f.ns)
    await f.pod_phase(name, ("Running",))
    await _log_contains(f, name, "value-del", 30)
    await _log_contains(f, name, "c-missing", 30)
    await f.client.delete(kind, "del", f.ns)
    body = obj("upd", "value-upd-2")
    await f.client.patch(kind, "upd", {"data": body["data"]}, f.ns)
    await f.client.create(kind, obj("create", "value-create"), f.ns)
    await _log_contains(f, name, "value-create", SYNC_WAIT)
    await _log_contains(f, name, "value-upd-2", SYNC_WAIT)
    await _log_contains(f, name, "d-missing", SYNC_WAIT)


@conformance("Projected secret optional updates should be reflected in volume")
async def psec_optional_updates(f):
    await _optional_updates(f, "secrets", "psopt")


# ---------------------------------------------------------------------------------------------
# Projected configMap (projected.go:408-769)
def _pcm(name, cmd, items=None, mode=None, cm="cm", **pod_extra):
    src = {"configMap": {"name": cm}}
    if items:
        src["configMap"]["items"] = items
    prj = {"sources": [src]}
    if mode is not None:
        prj["defaultMode"] = mode
    return _mount(_pod(name, cmd, **pod_extra), "p", {"projected": prj}, "/etc/projected-configmap-volume")


def _cat(rel):
    return _at("p", "/etc/projected-configmap-volume", rel)


@conformance("Projected configMap should be consumable from pods in volume")
async def pcm_volume(f):
    await _cm(f)
    assert _lines(await _run_and_log(f, _pcm("pcv", f"cat {_cat('data-1')}"))) == ["value-1"]


@conformance("Projected configMap should be consumable from pods in volume as non-root")
async def pcm_non_root(f):
    await _cm(f)
    p = _pcm("pcnr", f"id -u; cat {_cat('data-1')}", securityContext={"runAsUser": 1000})
    assert _lines(await _run_and_log(f, p)) == ["1000", "value-1"]


@conformance("Projected configMap should be consumable from pods in volume with mappings")
async def pcm_mappings(f):
    await _cm(f)
    p = _pcm("pcmap", f"cat {_cat('path/to/data-2')}", items=[{"key": "data-2", "path": "path/to/data-2"}])
    assert _lines(await _run_and_log(f, p)) == ["value-2"]


@conformance("Projected configMap should be consumable from pods in volume with mappings and Item mode set")
async def pcm_item_mode(f):
    await _cm(f)
    p = _pcm("pcim", f"stat -c %a {_cat('path/to/data-2')}",
             items=[{"key": "data-2", "path": "path/to/data-2", "mode": 0o400}])
    assert _lines(await _run_and_log(f, p)) == ["400"]


@conformance("Projected configMap should be consumable from pods in volume with mappings as non-root")
async def pcm_mappings_non_root(f):
    await _cm(f)
    p = _pcm("pcmnr", f"id -u; cat {_cat('path/to/data-2')}", items=[{"key": "data-2", "path": "path/to/data-2"}],
             securityContext={"runAsUser": 1000})
    assert _lines(await _run_and_log(f, p)) == ["1000", "value-2"]


@conformance("Projected configMap optional updates should be reflected in volume")
async def pcm_optional_updates(f):
    await _optional_updates(f, "configmaps", "pcopt")


@conformance("Projected configMap should be consumable in multiple volumes in the same pod")
async def pcm_multiple(f):
    await _cm(f)
    p = _pod("pcmulti", f"cat {_at('a', '/etc/a', 'data-1')}; echo; cat {_at('b', '/etc/b', 'data-1')}")
    _mount(p, "a", {"projected": {"sources": [{"configMap": {"name": "cm"}}]}}, "/etc/a")
    _mount(p, "b", {"projected": {"sources": [{"configMap": {"name": "cm"}}]}}, "/etc/b")
    assert _lines(await _run_and_log(f, p)) == ["value-1", "value-1"]


# ---------------------------------------------------------------------------------------------
# Projected downwardAPI (projected.go:867-1092)
def _pdapi(name, items, cmd, mode=None, **pod_extra):
    prj = {"sources": [{"downwardAPI": {"items": items}}]}
    if mode is not None:
        prj["defaultMode"] = mode
    return _mount(_pod(name, cmd, **pod_extra), "podinfo", {"projected": prj}, "/etc/podinfo")


def _pinfo(rel):
    return _at("podinfo", "/etc/podinfo", rel)


@conformance("Projected downwardAPI should set DefaultMode on files")
async def pdapi_default_mode(f):
    p = _pdapi("pdmode", [{"path": "podname", "fieldRef": {"fieldPath": "metadata.name"}}],
               f"stat -c %a {_pinfo('podname')}", mode=0o400)
    assert _lines(await _run_and_log(f, p)) == ["400"]


@conformance("Projected downwardAPI should set mode on item file")
async def pdapi_item_mode(f):
    p = _pdapi("pdimode", [{"path": "podname", "fieldRef": {"fieldPath": "metadata.name"}, "mode": 0o400}],
               f"stat -c %a {_pinfo('podname')}")
    assert _lines(await _run_and_log(f, p)) == ["400"]


async def _pdapi_update(f, name, field):
    path = _pinfo(field)
    p = _pdapi(name, [{"path": field, "fieldRef": {"fieldPath": f"metadata.{field}"}}],
               f"while true; do cat {path}; echo; sleep 1; done", restart="Always")
    p["metadata"][field] = dict(p["metadata"].get(field) or {}, key1="value1")
    await f.client.create("pods", p, f.ns)
    await f.pod_phase(name, ("Running",))
    await _log_contains(f, name, 'key1="value1"', 30)
    await f.client.patch("pods", name, {"metadata": {field: {"key3": "value3"}}}, f.ns)
    await _log_contains(f, name, 'key3="value3"', SYNC_WAIT)


@conformance("Projected downwardAPI should update labels on modification")
async def pdapi_update_labels(f):
    await _pdapi_update(f, "pdlabels", "labels")


@conformance("Projected downwardAPI should update annotations on modification")
async def pdapi_update_annotations(f):
    await _pdapi_update(f, "pdannot", "annotations")


async def _pdapi_resource(f, name, resource, resources, divisor=None):
    p = _pdapi(name, [_res_item("v", resource, divisor)], f"cat {_pinfo('v')}")
    if resources:
        p["spec"]["containers"][0]["resources"] = resources
    return _lines(await _run_and_log(f, p))


@conformance("Projected downwardAPI should provide container's cpu limit")
async def pdapi_cpu_limit(f):
    assert await _pdapi_resource(f, "pdcpul", "limits.cpu", _RES, "1m") == ["1250"]


@conformance("Projected downwardAPI should provide container's memory limit")
async def pdapi_mem_limit(f):
    assert await _pdapi_resource(f, "pdmeml", "limits.memory", _RES, "1Mi") == ["64"]


@conformance("Projected downwardAPI should provide container's cpu request")
async def pdapi_cpu_request(f):
    assert await _pdapi_resource(f, "pdcpur", "requests.cpu", _RES, "1m") == ["250"]


@conformance("Projected downwardAPI should provide container's memory request")
async def pdapi_mem_request(f):
    assert await _pdapi_resource(f, "pdmemr", "requests.memory", _RES, "1Mi") == ["32"]


@conformance("Projected downwardAPI should provide node allocatable (cpu) as default cpu limit if the limit is not set")
async def pdapi_default_cpu(f):
    out = await _pdapi_resource(f, "pddefcpu", "limits.cpu", None)
    assert out and int(out[0]) >= 1, out


@conformance("Projected downwardAPI should provide node allocatable (memory) as default memory limit if the limit "
             "is not set")
async def pdapi_default_mem(f):
    out = await _pdapi_resource(f, "pddefmem", "limits.memory", None)
    assert out and int(out[0]) > 0, out
