"""More conformance specs: ports of `ConformanceIt` cases from the reference's
`test/e2e/common/{configmap_volume,secrets_volume,downward_api,downwardapi_volume,projected,
empty_dir,expansion,docker_containers,container_probe,pods,configmap}.go`,
`test/e2e/kubectl/kubectl.go`, `test/e2e/network/proxy.go` and
`test/e2e/scheduling/predicates.go`. Each runs in its own namespace (framework.Framework).

Volumes are read at their mount path when the container has a private mount namespace, else at
the host path the process runtime exports as `KUBERNETES_VOLUME_<NAME>` (see `_at`). Specs that
wait for the kubelet's periodic volume sync allow 150 s (the reference's `--sync-frequency`
is 1 m; the in-process test cluster syncs every second).
"""
from __future__ import annotations

import asyncio
import base64
import io

from ..api import core
from .framework import conformance

BUSYBOX = "busybox"
SYNC_WAIT = 150.0


def _b64(s):
    return base64.b64encode(s.encode()).decode()


def _at(vol, mount, rel):
    """Shell expression for file `rel` of volume `vol` mounted at `mount`."""
    env = "KUBERNETES_VOLUME_" + vol.upper().replace("-", "_")
    return f'$(if [ -e "{mount}/{rel}" ]; then echo "{mount}/{rel}"; else echo "${env}/{rel}"; fi)'


def _pod(name, cmd, restart="Never", **spec_extra):
    return {"metadata": {"name": name, "labels": {"app": name}},
            "spec": dict({"restartPolicy": restart, "containers": [{"name": "c", "image": BUSYBOX,
                                                                     "command": ["sh", "-c", cmd]}]}, **spec_extra)}


def _mount(p, vol, source, mount, **m):
    p["spec"].setdefault("volumes", []).append(dict({"name": vol}, **source))
    p["spec"]["containers"][0].setdefault("volumeMounts", []).append(dict({"name": vol, "mountPath": mount}, **m))
    return p


async def _run_and_log(f, p, timeout=60.0):
    await f.client.create("pods", p, f.ns)
    await f.pod_phase(p["metadata"]["name"], ("Succeeded",), timeout)
    return await f.logs(p["metadata"]["name"])


async def _log_contains(f, name, text, timeout=SYNC_WAIT):
    async def check():
        return text in await f.logs(name)
    await f.wait(check, timeout, f"{text!r} in the logs of {name}")


def _lines(out):
    return [ln.strip() for ln in out.splitlines() if ln.strip()]


# ---------------------------------------------------------------------------------------------
# ConfigMap volumes (configmap_volume.go)
async def _cm(f, name="cm", data=None):
    await f.client.create("configmaps", {"metadata": {"name": name}, "data": data or {"data-1": "value-1",
                                                                                     "data-2": "value-2"}}, f.ns)


@conformance("ConfigMap should be consumable from pods in volume with defaultMode set")
async def cm_default_mode(f):
    await _cm(f)
    p = _mount(_pod("cmmode", f"stat -c %a {_at('v', '/etc/cfg', 'data-1')}; cat {_at('v', '/etc/cfg', 'data-1')}"),
               "v", {"configMap": {"name": "cm", "defaultMode": 0o400}}, "/etc/cfg")
    out = _lines(await _run_and_log(f, p))
    assert out == ["400", "value-1"], out


@conformance("ConfigMap should be consumable from pods in volume with mappings")
async def cm_mappings(f):
    await _cm(f)
    p = _mount(_pod("cmmap", f"cat {_at('v', '/etc/cfg', 'path/to/data-2')}"),
               "v", {"configMap": {"name": "cm", "items": [{"key": "data-2", "path": "path/to/data-2"}]}}, "/etc/cfg")
    assert _lines(await _run_and_log(f, p)) == ["value-2"]


@conformance("ConfigMap should be consumable from pods in volume with mappings and Item mode set")
async def cm_item_mode(f):
    await _cm(f)
    p = _mount(_pod("cmitem", f"stat -c %a {_at('v', '/etc/cfg', 'path/to/data-2')}"),
               "v", {"configMap": {"name": "cm", "items": [{"key": "data-2", "path": "path/to/data-2", "mode": 0o400}]}},
               "/etc/cfg")
    assert _lines(await _run_and_log(f, p)) == ["400"]


@conformance("ConfigMap should be consumable from pods in volume as non-root")
async def cm_non_root(f):
    await _cm(f)
    p = _mount(_pod("cmnr", f"id -u; cat {_at('v', '/etc/cfg', 'data-1')}",
                    securityContext={"runAsUser": 1000}),
               "v", {"configMap": {"name": "cm"}}, "/etc/cfg")
    out = _lines(await _run_and_log(f, p))
    assert out == ["1000", "value-1"], out


@conformance("ConfigMap should be consumable in multiple volumes in the same pod")
async def cm_multiple_volumes(f):
    await _cm(f)
    p = _pod("cmmulti", f"cat {_at('v1', '/etc/cfg1', 'data-1')} {_at('v2', '/etc/cfg2', 'data-1')}")
    _mount(p, "v1", {"configMap": {"name": "cm"}}, "/etc/cfg1")
    _mount(p, "v2", {"configMap": {"name": "cm"}}, "/etc/cfg2")
    assert _lines(await _run_and_log(f, p)) == ["value-1value-1"] or \
        (await f.logs("cmmulti")).count("value-1") == 2


@conformance("ConfigMap updates should be reflected in volume")
async def cm_updates(f):
    await f.client.create("configmaps", {"metadata": {"name": "upd"}, "data": {"data-1": "value-1"}}, f.ns)
    path = _at("v", "/etc/cfg", "data-1")
    p = _mount(_pod("cmupd", f"while true; do cat {path}; echo; sleep 1; done", restart="Always"),
               "v", {"configMap": {"name": "upd"}}, "/etc/cfg")
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("cmupd", ("Running",))
    await _log_contains(f, "cmupd", "value-1", 30)
    await f.client.patch("configmaps", "upd", {"data": {"data-1": "value-2"}}, f.ns)
    await _log_contains(f, "cmupd", "value-2")


@conformance("ConfigMap optional updates should be reflected in volume")
async def cm_optional_updates(f):
    path = _at("v", "/etc/cfg", "data-1")
    p = _mount(_pod("cmopt", f"while true; do cat {path} 2>/dev/null || echo missing; sleep 1; done",
                    restart="Always"), "v", {"configMap": {"name": "later", "optional": True}}, "/etc/cfg")
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("cmopt", ("Running",))
    await _log_contains(f, "cmopt", "missing", 30)
    await f.client.create("configmaps", {"metadata": {"name": "later"}, "data": {"data-1": "appeared"}}, f.ns)
    await _log_contains(f, "cmopt", "appeared")


@conformance("ConfigMap should be consumable via environment variable (configMapKeyRef)")
async def cm_env(f):
    await _cm(f)
    p = _pod("cmenv", "echo CONFIG_DATA_1=$CONFIG_DATA_1")
    p["spec"]["containers"][0]["env"] = [{"name": "CONFIG_DATA_1",
                                          "valueFrom": {"configMapKeyRef": {"name": "cm", "key": "data-1"}}}]
    assert "CONFIG_DATA_1=value-1" in await _run_and_log(f, p)


# ---------------------------------------------------------------------------------------------
# Secret volumes (secrets_volume.go, secrets.go)
async def _secret(f, name="sec"):
    await f.client.create("secrets", {"metadata": {"name": name}, "data": {"data-1": _b64("value-1"),
                                                                           "data-2": _b64("value-2")}}, f.ns)


@conformance("Secrets should be consumable from pods in volume with defaultMode set")
async def secret_default_mode(f):
    await _secret(f)
    p = _mount(_pod("secmode", f"stat -c %a {_at('v', '/etc/sec', 'data-1')}; cat {_at('v', '/etc/sec', 'data-1')}"),
               "v", {"secret": {"secretName": "sec", "defaultMode": 0o400}}, "/etc/sec")
    assert _lines(await _run_and_log(f, p)) == ["400", "value-1"]


@conformance("Secrets should be consumable from pods in volume with mappings")
async def secret_mappings(f):
    await _secret(f)
    p = _mount(_pod("secmap", f"cat {_at('v', '/etc/sec', 'new-path-data-1')}"),
               "v", {"secret": {"secretName": "sec", "items": [{"key": "data-1", "path": "new-path-data-1"}]}},
               "/etc/sec")
    assert _lines(await _run_and_log(f, p)) == ["value-1"]


@conformance("Secrets should be consumable from pods in volume with mappings and Item Mode set")
async def secret_item_mode(f):
    await _secret(f)
    p = _mount(_pod("secitem", f"stat -c %a {_at('v', '/etc/sec', 'new-path-data-1')}"),
               "v", {"secret": {"secretName": "sec", "items": [{"key": "data-1", "path": "new-path-data-1",
                                                                "mode": 0o400}]}}, "/etc/sec")
    assert _lines(await _run_and_log(f, p)) == ["400"]


@conformance("Secrets should be consumable in multiple volumes in a pod")
async def secret_multiple_volumes(f):
    await _secret(f)
    p = _pod("secmulti", f"cat {_at('a', '/etc/a', 'data-1')}; echo; cat {_at('b', '/etc/b', 'data-2')}")
    _mount(p, "a", {"secret": {"secretName": "sec"}}, "/etc/a")
    _mount(p, "b", {"secret": {"secretName": "sec"}}, "/etc/b")
    assert _lines(await _run_and_log(f, p)) == ["value-1", "value-2"]


@conformance("Secrets optional updates should be reflected in volume")
async def secret_optional_updates(f):
    await f.client.create("secrets", {"metadata": {"name": "s-del"}, "data": {"k": _b64("to-be-deleted")}}, f.ns)
    p = _pod("secopt", "while true; do cat " + _at("d", "/etc/d", "k") + " 2>/dev/null || echo del-missing; echo; "
             "cat " + _at("c", "/etc/c", "k") + " 2>/dev/null || echo create-missing; echo; sleep 1; done",
             restart="Always")
    _mount(p, "d", {"secret": {"secretName": "s-del", "optional": True}}, "/etc/d")
    _mount(p, "c", {"secret": {"secretName": "s-create", "optional": True}}, "/etc/c")
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("secopt", ("Running",))
    await _log_contains(f, "secopt", "to-be-deleted", 30)
    await _log_contains(f, "secopt", "create-missing", 30)
    await f.client.delete("secrets", "s-del", f.ns)
    await f.client.create("secrets", {"metadata": {"name": "s-create"}, "data": {"k": _b64("created")}}, f.ns)
    await _log_contains(f, "secopt", "created")
    await _log_contains(f, "secopt", "del-missing")


@conformance("Secrets should be consumable via the environment (envFrom)")
async def secret_env_from(f):
    await _secret(f)
    # `env` itself, not a shell: POSIX shells drop variables whose names are not identifiers
    p = {"metadata": {"name": "secenv"}, "spec": {"restartPolicy": "Never", "containers": [
        {"name": "c", "image": BUSYBOX, "command": ["env"], "envFrom": [{"secretRef": {"name": "sec"}, "prefix": "p_"}]}]}}
    out = await _run_and_log(f, p)
    got = sorted(ln for ln in _lines(out) if ln.startswith("p_data"))
    assert got == ["p_data-1=value-1", "p_data-2=value-2"], out


# ---------------------------------------------------------------------------------------------
# Downward API env (downward_api.go)
@conformance("Downward API should provide pod name, namespace and IP address as env vars")
async def dapi_name_ns_ip(f):
    p = _pod("dapiip", "echo POD_NAME=$POD_NAME; echo POD_NAMESPACE=$POD_NAMESPACE; echo POD_IP=$POD_IP")
    p["spec"]["containers"][0]["env"] = [
        {"name": n, "valueFrom": {"fieldRef": {"fieldPath": fp}}}
        for n, fp in (("POD_NAME", "metadata.name"), ("POD_NAMESPACE", "metadata.namespace"), ("POD_IP", "status.podIP"))]
    out = await _run_and_log(f, p)
    pod = await f.client.get("pods", "dapiip", f.ns)
    assert "POD_NAME=dapiip" in out and f"POD_NAMESPACE={f.ns}" in out
    assert f"POD_IP={pod['status'].get('podIP')}" in out and pod["status"].get("podIP")


@conformance("Downward API should provide host IP as an env var")
async def dapi_host_ip(f):
    p = _pod("dapihost", "echo HOST_IP=$HOST_IP")
    p["spec"]["containers"][0]["env"] = [{"name": "HOST_IP", "valueFrom": {"fieldRef": {"fieldPath": "status.hostIP"}}}]
    out = await _run_and_log(f, p)
    pod = await f.client.get("pods", "dapihost", f.ns)
    assert pod["status"].get("hostIP") and f"HOST_IP={pod['status']['hostIP']}" in out


@conformance("Downward API should provide container's limits.cpu/memory and requests.cpu/memory as env vars")
async def dapi_resources_env(f):
    p = _pod("dapires", "echo CPU_LIMIT=$CPU_LIMIT MEMORY_LIMIT=$MEMORY_LIMIT CPU_REQUEST=$CPU_REQUEST "
             "MEMORY_REQUEST=$MEMORY_REQUEST")
    c = p["spec"]["containers"][0]
    c["resources"] = {"requests": {"cpu": "250m", "memory": "32Mi"}, "limits": {"cpu": "1250m", "memory": "64Mi"}}
    c["env"] = [{"name": n, "valueFrom": {"resourceFieldRef": {"resource": r}}}
                for n, r in (("CPU_LIMIT", "limits.cpu"), ("MEMORY_LIMIT", "limits.memory"),
                             ("CPU_REQUEST", "requests.cpu"), ("MEMORY_REQUEST", "requests.memory"))]
    out = await _run_and_log(f, p)
    assert "CPU_LIMIT=2 MEMORY_LIMIT=67108864 CPU_REQUEST=1 MEMORY_REQUEST=33554432" in out, out


@conformance("Downward API should provide default limits.cpu/memory from node allocatable")
async def dapi_default_limits(f):
    p = _pod("dapidef", "echo CPU_LIMIT=$CPU_LIMIT MEMORY_LIMIT=$MEMORY_LIMIT")
    p["spec"]["containers"][0]["env"] = [{"name": n, "valueFrom": {"resourceFieldRef": {"resource": r}}}
                                         for n, r in (("CPU_LIMIT", "limits.cpu"), ("MEMORY_LIMIT", "limits.memory"))]
    out = await _run_and_log(f, p)
    pod = await f.client.get("pods", "dapidef", f.ns)
    node = await f.client.get("nodes", pod["spec"]["nodeName"])
    from ..api.quantity import parse_quantity
    alloc = node["status"]["allocatable"]
    cpu = parse_quantity(str(alloc["cpu"])).value
    want_cpu = -(-cpu.numerator // cpu.denominator)
    assert f"CPU_LIMIT={want_cpu} " in out and f"MEMORY_LIMIT={int(parse_quantity(str(alloc['memory'])).value)}" in out, out


@conformance("Downward API should provide pod UID as env vars")
async def dapi_uid(f):
    p = _pod("dapiuid", "echo POD_UID=$POD_UID")
    p["spec"]["containers"][0]["env"] = [{"name": "POD_UID", "valueFrom": {"fieldRef": {"fieldPath": "metadata.uid"}}}]
    out = await _run_and_log(f, p)
    pod = await f.client.get("pods", "dapiuid", f.ns)
    assert f"POD_UID={pod['metadata']['uid']}" in out


# ---------------------------------------------------------------------------------------------
# Downward API volume (downwardapi_volume.go)
def _dapi_vol(name, items, cmd, mode=None, **pod_extra):
    src = {"downwardAPI": {"items": items}}
    if mode is not None:
        src["downwardAPI"]["defaultMode"] = mode
    return _mount(_pod(name, cmd, **pod_extra), "podinfo", src, "/etc/podinfo")


@conformance("Downward API volume should provide podname only")
async def dapiv_podname(f):
    p = _dapi_vol("dvname", [{"path": "podname", "fieldRef": {"fieldPath": "metadata.name"}}],
                  f"cat {_at('podinfo', '/etc/podinfo', 'podname')}")
    assert _lines(await _run_and_log(f, p)) == ["dvname"]


@conformance("Downward API volume should set DefaultMode on files")
async def dapiv_default_mode(f):
    p = _dapi_vol("dvmode", [{"path": "podname", "fieldRef": {"fieldPath": "metadata.name"}}],
                  f"stat -c %a {_at('podinfo', '/etc/podinfo', 'podname')}", mode=0o400)
    assert _lines(await _run_and_log(f, p)) == ["400"]


@conformance("Downward API volume should set mode on item file")
async def dapiv_item_mode(f):
    p = _dapi_vol("dvitem", [{"path": "podname", "fieldRef": {"fieldPath": "metadata.name"}, "mode": 0o400}],
                  f"stat -c %a {_at('podinfo', '/etc/podinfo', 'podname')}")
    assert _lines(await _run_and_log(f, p)) == ["400"]


@conformance("Downward API volume should update labels on modification")
async def dapiv_labels_update(f):
    path = _at("podinfo", "/etc/podinfo", "labels")
    p = _dapi_vol("dvlabels", [{"path": "labels", "fieldRef": {"fieldPath": "metadata.labels"}}],
                  f"while true; do cat {path}; echo; sleep 1; done", restart="Always")
    p["metadata"]["labels"] = {"key1": "value1", "key2": "value2"}
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("dvlabels", ("Running",))
    await _log_contains(f, "dvlabels", 'key1="value1"', 30)
    await f.client.patch("pods", "dvlabels", {"metadata": {"labels": {"key3": "value3"}}}, f.ns)
    await _log_contains(f, "dvlabels", 'key3="value3"')


@conformance("Downward API volume should update annotations on modification")
async def dapiv_annotations_update(f):
    path = _at("podinfo", "/etc/podinfo", "annotations")
    p = _dapi_vol("dvann", [{"path": "annotations", "fieldRef": {"fieldPath": "metadata.annotations"}}],
                  f"while true; do cat {path}; echo; sleep 1; done", restart="Always")
    p["metadata"]["annotations"] = {"builder": "bar"}
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("dvann", ("Running",))
    await _log_contains(f, "dvann", 'builder="bar"', 30)
    await f.client.patch("pods", "dvann", {"metadata": {"annotations": {"builder": "foo"}}}, f.ns)
    await _log_contains(f, "dvann", 'builder="foo"')


def _res_item(path, resource, divisor=None):
    ref = {"containerName": "c", "resource": resource}
    if divisor:
        ref["divisor"] = divisor
    return {"path": path, "resourceFieldRef": ref}


async def _dapiv_resource(f, name, resource, resources, divisor=None):
    p = _dapi_vol(name, [_res_item("v", resource, divisor)], f"cat {_at('podinfo', '/etc/podinfo', 'v')}")
    if resources:
        p["spec"]["containers"][0]["resources"] = resources
    return _lines(await _run_and_log(f, p))


_RES = {"requests": {"cpu": "250m", "memory": "32Mi"}, "limits": {"cpu": "1250m", "memory": "64Mi"}}


@conformance("Downward API volume should provide container's cpu limit")
async def dapiv_cpu_limit(f):
    assert await _dapiv_resource(f, "dvcpul", "limits.cpu", _RES, "1m") == ["1250"]


@conformance("Downward API volume should provide container's memory limit")
async def dapiv_mem_limit(f):
    assert await _dapiv_resource(f, "dvmeml", "limits.memory", _RES, "1Mi") == ["64"]


@conformance("Downward API volume should provide container's cpu request")
async def dapiv_cpu_request(f):
    assert await _dapiv_resource(f, "dvcpur", "requests.cpu", _RES, "1m") == ["250"]


@conformance("Downward API volume should provide container's memory request")
async def dapiv_mem_request(f):
    assert await _dapiv_resource(f, "dvmemr", "requests.memory", _RES, "1Mi") == ["32"]


@conformance("Downward API volume should provide node allocatable (cpu) as default cpu limit if the limit is not set")
async def dapiv_default_cpu(f):
    out = await _dapiv_resource(f, "dvdefcpu", "limits.cpu", None)
    assert out and int(out[0]) >= 1, out


@conformance("Downward API volume should provide node allocatable (memory) as default memory limit if the limit is not set")
async def dapiv_default_mem(f):
    out = await _dapiv_resource(f, "dvdefmem", "limits.memory", None)
    assert out and int(out[0]) > 0, out


# ---------------------------------------------------------------------------------------------
# Projected volumes (projected.go)
@conformance("Projected should be consumable from pods in volume with defaultMode set (configMap)")
async def projected_cm_mode(f):
    await _cm(f)
    p = _mount(_pod("prjmode", f"stat -c %a {_at('p', '/etc/prj', 'data-1')}; cat {_at('p', '/etc/prj', 'data-1')}"),
               "p", {"projected": {"defaultMode": 0o400, "sources": [{"configMap": {"name": "cm"}}]}}, "/etc/prj")
    assert _lines(await _run_and_log(f, p)) == ["400", "value-1"]


@conformance("Projected should be consumable from pods in volume with mappings (secret)")
async def projected_secret_map(f):
    await _secret(f)
    p = _mount(_pod("prjmap", f"cat {_at('p', '/etc/prj', 'new-path-data-1')}"),
               "p", {"projected": {"sources": [{"secret": {"name": "sec", "items": [
                   {"key": "data-1", "path": "new-path-data-1"}]}}]}}, "/etc/prj")
    assert _lines(await _run_and_log(f, p)) == ["value-1"]


@conformance("Projected should provide podname only (downwardAPI)")
async def projected_podname(f):
    p = _mount(_pod("prjname", f"cat {_at('p', '/etc/prj', 'podname')}"),
               "p", {"projected": {"sources": [{"downwardAPI": {"items": [
                   {"path": "podname", "fieldRef": {"fieldPath": "metadata.name"}}]}}]}}, "/etc/prj")
    assert _lines(await _run_and_log(f, p)) == ["prjname"]


@conformance("Projected updates should be reflected in volume (configMap)")
async def projected_updates(f):
    await f.client.create("configmaps", {"metadata": {"name": "pupd"}, "data": {"data-1": "value-1"}}, f.ns)
    path = _at("p", "/etc/prj", "data-1")
    p = _mount(_pod("prjupd", f"while true; do cat {path}; echo; sleep 1; done", restart="Always"),
               "p", {"projected": {"sources": [{"configMap": {"name": "pupd"}}]}}, "/etc/prj")
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("prjupd", ("Running",))
    await _log_contains(f, "prjupd", "value-1", 30)
    await f.client.patch("configmaps", "pupd", {"data": {"data-1": "value-2"}}, f.ns)
    await _log_contains(f, "prjupd", "value-2")


# ---------------------------------------------------------------------------------------------
# EmptyDir (empty_dir.go)
def _ed(name, medium, mode, non_root):
    f_ = _at("test-volume", "/test-volume", "test-file")
    d = f'$(dirname {f_})'
    cmd = (f"echo mount-tester new file > {f_} && chmod {mode} {f_} && stat -c %a {f_} && cat {f_} && "
           f"stat -c %a {d}")
    p = _pod(name, cmd, **({"securityContext": {"runAsUser": 1001}} if non_root else {}))
    return _mount(p, "test-volume", {"emptyDir": {"medium": medium} if medium else {}}, "/test-volume")


async def _ed_check(f, name, medium, mode, non_root):
    out = _lines(await _run_and_log(f, _ed(name, medium, mode, non_root)))
    assert out[0] == mode.lstrip("0") and out[1] == "mount-tester new file", out
    assert out[2] == "777", out          # the volume directory itself is world-writable


@conformance("EmptyDir volumes should support (root,0644,default)")
async def ed_root_0644(f):
    await _ed_check(f, "ed1", None, "0644", False)


@conformance("EmptyDir volumes should support (root,0666,tmpfs)")
async def ed_root_0666_tmpfs(f):
    await _ed_check(f, "ed2", "Memory", "0666", False)


@conformance("EmptyDir volumes should support (non-root,0777,default)")
async def ed_nonroot_0777(f):
    await _ed_check(f, "ed3", None, "0777", True)


@conformance("EmptyDir volumes should support (non-root,0644,tmpfs)")
async def ed_nonroot_0644_tmpfs(f):
    await _ed_check(f, "ed4", "Memory", "0644", True)


# ---------------------------------------------------------------------------------------------
# Variable expansion (expansion.go)
@conformance("Variable Expansion should allow composing env vars into new env vars")
async def expansion_compose(f):
    p = _pod("exp1", "env | grep -E '^(FOO|BAR|FOOBAR)=' | sort")
    p["spec"]["containers"][0]["env"] = [{"name": "FOO", "value": "foo-value"}, {"name": "BAR", "value": "bar-value"},
                                         {"name": "FOOBAR", "value": "$(FOO);;$(BAR)"}]
    assert _lines(await _run_and_log(f, p)) == ["BAR=bar-value", "FOO=foo-value", "FOOBAR=foo-value;;bar-value"]


@conformance("Variable Expansion should allow substituting values in a container's command")
async def expansion_command(f):
    p = {"metadata": {"name": "exp2"}, "spec": {"restartPolicy": "Never", "containers": [
        {"name": "c", "image": BUSYBOX, "command": ["sh", "-c", "echo test-value=$(TEST_VAR)"],
         "env": [{"name": "TEST_VAR", "value": "test-value"}]}]}}
    assert "test-value=test-value" in await _run_and_log(f, p)


@conformance("Variable Expansion should allow substituting values in a container's args")
async def expansion_args(f):
    p = {"metadata": {"name": "exp3"}, "spec": {"restartPolicy": "Never", "containers": [
        {"name": "c", "image": BUSYBOX, "command": ["sh", "-c"], "args": ["echo arg-value=$(TEST_VAR)"],
         "env": [{"name": "TEST_VAR", "value": "test-value"}]}]}}
    assert "arg-value=test-value" in await _run_and_log(f, p)


# ---------------------------------------------------------------------------------------------
# Docker containers: ENTRYPOINT / CMD (docker_containers.go)
TESTER = "kubernetes-amd/entrypoint-tester"


async def _ep(f, name, **c):
    p = {"metadata": {"name": name}, "spec": {"restartPolicy": "Never",
                                              "containers": [dict({"name": "c", "image": TESTER}, **c)]}}
    return _lines(await _run_and_log(f, p))


@conformance("Docker Containers should use the image defaults if command and args are blank")
async def docker_defaults(f):
    assert await _ep(f, "dk1") == ["entrypoint default arguments"]


@conformance("Docker Containers should be able to override the image's default arguments (docker cmd)")
async def docker_args(f):
    assert await _ep(f, "dk2", args=["override", "arguments"]) == ["entrypoint override arguments"]


@conformance("Docker Containers should be able to override the image's default command (docker entrypoint)")
async def docker_command(f):
    assert await _ep(f, "dk3", command=["/bin/echo", "override", "command"]) == ["override command"]


@conformance("Docker Containers should be able to override the image's default command and arguments")
async def docker_both(f):
    assert await _ep(f, "dk4", command=["/bin/echo", "cmd"], args=["and", "args"]) == ["cmd and args"]


# ---------------------------------------------------------------------------------------------
# Probes (container_probe.go)
@conformance("Probing container with readiness probe that fails should never be ready and never restart")
async def readiness_fails(f):
    p = _pod("rfail", "sleep 3600", restart="Always")
    p["spec"]["containers"][0]["readinessProbe"] = {"exec": {"command": ["/bin/false"]}, "periodSeconds": 1}
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("rfail", ("Running",))
    await asyncio.sleep(4)
    x = await f.client.get("pods", "rfail", f.ns)
    cs = (x["status"].get("containerStatuses") or [{}])[0]
    assert not cs.get("ready") and cs.get("restartCount", 0) == 0, cs
    assert core.get_condition(x["status"], "Ready")["status"] == "False"


@conformance("Probing container should *not* be restarted with a exec \"cat /tmp/health\" liveness probe")
async def liveness_ok(f):
    health = _at("tmp", "/tmp/h", "health")
    p = _mount(_pod("lok", f"echo ok > {health}; sleep 3600", restart="Always"), "tmp", {"emptyDir": {}}, "/tmp/h")
    p["spec"]["containers"][0]["livenessProbe"] = {"exec": {"command": ["sh", "-c", f"cat {health}"]},
                                                   "initialDelaySeconds": 1, "periodSeconds": 1, "failureThreshold": 1}
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("lok", ("Running",))
    await asyncio.sleep(5)
    x = await f.client.get("pods", "lok", f.ns)
    assert (x["status"].get("containerStatuses") or [{}])[0].get("restartCount", 0) == 0


@conformance("Probing container should be restarted with a exec \"cat /tmp/health\" liveness probe")
async def liveness_exec_restart(f):
    health = _at("tmp", "/tmp/h", "health")
    p = _mount(_pod("lexec", f"echo ok > {health}; sleep 3; rm -f {health}; sleep 3600", restart="Always"),
               "tmp", {"emptyDir": {}}, "/tmp/h")
    p["spec"]["containers"][0]["livenessProbe"] = {"exec": {"command": ["sh", "-c", f"cat {health}"]},
                                                   "initialDelaySeconds": 1, "periodSeconds": 1, "failureThreshold": 1}
    await f.client.create("pods", p, f.ns)

    async def restarted():
        x = await f.client.get("pods", "lexec", f.ns)
        return (x["status"].get("containerStatuses") or [{}])[0].get("restartCount", 0) >= 1
    await f.wait(restarted, 60, "a restart after the health file went away")


# ---------------------------------------------------------------------------------------------
# Pods (pods.go)
@conformance("Pods should be submitted and removed")
async def pods_submit_remove(f):
    lst = await f.client.list("pods", f.ns)
    w = await f.client.watch("pods", f.ns, lst["metadata"]["resourceVersion"], label_selector="e2e=submit")
    p = _pod("subm", "sleep 3600", restart="Always")
    p["metadata"]["labels"]["e2e"] = "submit"
    await f.client.create("pods", p, f.ns)
    seen = []
    async for typ, obj in w:
        seen.append(typ)
        if typ == "ADDED":
            break
    await f.pod_phase("subm", ("Running",))
    await f.client.delete("pods", "subm", f.ns, grace_period=1)
    async for typ, obj in w:
        seen.append(typ)
        if typ == "DELETED":
            assert obj["metadata"].get("deletionTimestamp")
            break
    w.close()
    assert seen[0] == "ADDED" and seen[-1] == "DELETED"


@conformance("Pods should allow activeDeadlineSeconds to be updated")
async def pods_active_deadline_update(f):
    await f.client.create("pods", _pod("adl", "sleep 3600", restart="Always"), f.ns)
    await f.pod_phase("adl", ("Running",))
    await f.client.patch("pods", "adl", {"spec": {"activeDeadlineSeconds": 5}}, f.ns)

    async def failed():
        x = await f.client.get("pods", "adl", f.ns)
        return x if x["status"].get("phase") == "Failed" and x["status"].get("reason") == "DeadlineExceeded" else None
    await f.wait(failed, 60, "DeadlineExceeded after the update")


@conformance("Pods should contain environment variables for services")
async def pods_service_env(f):
    await f.client.create("services", {"metadata": {"name": "fooservice"}, "spec": {
        "selector": {"name": "server"}, "ports": [{"port": 8765, "targetPort": 8080}]}}, f.ns)
    svc = await f.client.get("services", "fooservice", f.ns)
    out = await _run_and_log(f, _pod("envsvc", "env | grep ^FOOSERVICE_ | sort"))
    assert f"FOOSERVICE_SERVICE_HOST={svc['spec']['clusterIP']}" in out and "FOOSERVICE_SERVICE_PORT=8765" in out, out


@conformance("Pods should get a host IP")
async def pods_host_ip(f):
    await f.client.create("pods", _pod("hostip", "sleep 3600", restart="Always"), f.ns)
    p = await f.pod_phase("hostip", ("Running",))
    node = await f.client.get("nodes", p["spec"]["nodeName"])
    addrs = {a["address"] for a in node["status"].get("addresses") or ()}
    assert p["status"].get("hostIP") in addrs, (p["status"], addrs)


@conformance("Pods should be updated (an updated label is visible in the pod)")
async def pods_updated(f):
    await f.client.create("pods", _pod("updt", "sleep 3600", restart="Always"), f.ns)
    await f.pod_phase("updt", ("Running",))
    cur = await f.client.get("pods", "updt", f.ns)
    cur["metadata"]["labels"]["time"] = "value"
    await f.client.update("pods", cur, f.ns)
    lst = await f.client.list("pods", f.ns, label_selector="time=value")
    assert [x["metadata"]["name"] for x in lst["items"]] == ["updt"]


# ---------------------------------------------------------------------------------------------
# kubectl (kubectl.go) — the in-tree kubectl against the cluster under test
async def _kubectl(f, *args):
    from ..kubectl.cli import main as kubectl
    out = io.StringIO()

    def call():
        try:
            return kubectl(["-s", f.client.url, *args], out=out)
        except SystemExit as e:             # kubectl's error exits: a non-zero status, not a crash
            if e.code not in (None, 0) and not isinstance(e.code, int):
                out.write(str(e.code))
            return e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
    rc = await asyncio.to_thread(call)
    return rc, out.getvalue()


@conformance("Kubectl client Kubectl cluster-info should check if Kubernetes master services is included in cluster-info")
async def kubectl_cluster_info(f):
    rc, out = await _kubectl(f, "cluster-info")
    assert rc == 0 and "Kubernetes master" in out and "is running at" in out, out


@conformance("Kubectl client Kubectl api-versions should check if v1 is in available api versions")
async def kubectl_api_versions(f):
    rc, out = await _kubectl(f, "api-versions")
    assert rc == 0 and "v1" in out.split(), out


@conformance("Kubectl client Kubectl label should update the label on a resource")
async def kubectl_label(f):
    await f.client.create("pods", _pod("lbl", "sleep 3600", restart="Always"), f.ns)
    rc, out = await _kubectl(f, "label", "-n", f.ns, "pods", "lbl", "testing-label=testing-label-value")
    assert rc == 0, out
    x = await f.client.get("pods", "lbl", f.ns)
    assert x["metadata"]["labels"]["testing-label"] == "testing-label-value"
    rc, out = await _kubectl(f, "label", "-n", f.ns, "pods", "lbl", "testing-label-")
    assert rc == 0 and "testing-label" not in (await f.client.get("pods", "lbl", f.ns))["metadata"]["labels"]


@conformance("Kubectl client Kubectl describe should check if kubectl describe prints relevant information for rc and pods")
async def kubectl_describe(f):
    rc_obj = {"metadata": {"name": "redis-master", "labels": {"app": "redis"}}, "spec": {
        "replicas": 1, "selector": {"app": "redis"}, "template": {"metadata": {"labels": {"app": "redis"}}, "spec": {
            "containers": [{"name": "redis-master", "image": BUSYBOX, "command": ["sh", "-c", "sleep 3600"]}]}}}}
    await f.client.create("replicationcontrollers", rc_obj, f.ns)

    async def one_pod():
        pods = (await f.client.list("pods", f.ns, label_selector="app=redis"))["items"]
        return pods[0] if pods else None
    pod = await f.wait(one_pod, 60, "the rc's pod")
    rc, out = await _kubectl(f, "describe", "-n", f.ns, "pod", pod["metadata"]["name"])
    assert rc == 0 and "Name:" in out and pod["metadata"]["name"] in out and "app=redis" in out, out
    rc, out = await _kubectl(f, "describe", "-n", f.ns, "rc", "redis-master")
    assert rc == 0 and "redis-master" in out and "Replicas:" in out, out


@conformance("Kubectl client Kubectl run pod should create a pod from an image when restart is Never")
async def kubectl_run_pod(f):
    rc, out = await _kubectl(f, "run", "-n", f.ns, "e2e-test-pod", "--restart=Never", f"--image={BUSYBOX}",
                             "--command", "--", "sh", "-c", "echo run-pod-ok")
    assert rc == 0, out
    await f.pod_phase("e2e-test-pod", ("Succeeded",))
    assert "run-pod-ok" in await f.logs("e2e-test-pod")


@conformance("Kubectl client Kubectl run deployment should create a deployment from an image")
async def kubectl_run_deployment(f):
    rc, out = await _kubectl(f, "run", "-n", f.ns, "e2e-test-dep", f"--image={BUSYBOX}", "--command", "--",
                             "sh", "-c", "sleep 3600")
    assert rc == 0, out

    async def dep():
        try:
            d = await f.client.get("deployments", "e2e-test-dep", f.ns)
        except Exception:  # noqa: BLE001
            return None
        return d if (d.get("status") or {}).get("availableReplicas") == 1 else None
    await f.wait(dep, 60, "the deployment kubectl run created")


# ---------------------------------------------------------------------------------------------
# Proxy (network/proxy.go) and scheduling predicates (predicates.go)
@conformance("Proxy version v1 should proxy logs on node using proxy subresource")
async def proxy_node_logs(f):
    node = (await f.client.list("nodes"))["items"][0]["metadata"]["name"]
    st, body = await f.client.raw("GET", f"/api/v1/nodes/{node}/proxy/logs/")
    assert st == 200, (st, body[:200])


@conformance("SchedulerPredicates validates resource limits of pods that are allowed to run")
async def predicates_resource_limits(f):
    nodes = (await f.client.list("nodes"))["items"]
    from ..api.quantity import parse_quantity
    biggest = max(parse_quantity(str(n["status"]["allocatable"]["cpu"])).milli_value() for n in nodes)
    fits = _pod("fits", "sleep 3600", restart="Always")
    fits["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "100m"}}
    await f.client.create("pods", fits, f.ns)
    await f.pod_phase("fits", ("Running",))
    big = _pod("too-big", "sleep 3600", restart="Always")
    big["spec"]["containers"][0]["resources"] = {"requests": {"cpu": f"{biggest + 1000}m"}}
    await f.client.create("pods", big, f.ns)

    async def unsched():
        x = await f.client.get("pods", "too-big", f.ns)
        c = core.get_condition(x.get("status"), core.COND_POD_SCHEDULED)
        return c if c and c.get("status") == "False" and "Insufficient cpu" in (c.get("message") or "") else None
    await f.wait(unsched, 30, "PodScheduled=False for insufficient cpu")


@conformance("SchedulerPredicates validates that NodeSelector is respected if not matching")
async def predicates_selector_not_matching(f):
    await f.client.create("pods", _pod("restricted", "true", nodeSelector={"label": "nonempty"}), f.ns)

    async def unsched():
        x = await f.client.get("pods", "restricted", f.ns)
        c = core.get_condition(x.get("status"), core.COND_POD_SCHEDULED)
        return c if c and c.get("status") == "False" and "node selector" in (c.get("message") or "") else None
    await f.wait(unsched, 30, "PodScheduled=False (node selector)")
