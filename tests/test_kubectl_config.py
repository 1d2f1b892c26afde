"""`kubectl config` against kubeconfig files (no cluster needed).

Parity: `pkg/kubectl/cmd/config/*_test.go` — view redaction / --minify / --flatten, set-cluster
and set-credentials with embedded certificates, set-context --current, set / unset of dotted
property paths, delete-cluster / delete-context / rename-context, and KUBECONFIG merging.
"""
import base64
import io
import json

import pytest
import yaml

from kubernetes_amd.kubectl.cli import main as kubectl


def kc(path, *args):
    out = io.StringIO()
    rc = kubectl(["--kubeconfig", str(path), "config", *args], out=out)
    return rc, out.getvalue()


def test_config_set_view_and_edit(tmp_path):
    cfgp = tmp_path / "config"
    ca = tmp_path / "ca.crt"
    ca.write_text("-----BEGIN CERTIFICATE-----\nAAA\n-----END CERTIFICATE-----\n")
    assert kc(cfgp, "set-cluster", "mi", "--server", "https://10.0.0.1:6443", "--certificate-authority", str(ca),
              "--embed-certs")[1].strip() == 'Cluster "mi" set.'
    assert kc(cfgp, "set-credentials", "admin", "--token", "s3cret")[0] == 0
    assert kc(cfgp, "set-context", "prod", "--cluster", "mi", "--user", "admin", "--namespace", "ml")[1].strip() == \
        'Context "prod" created.'
    assert kc(cfgp, "use-context", "prod")[1].strip() == 'Switched to context "prod".'
    raw = yaml.safe_load(cfgp.read_text())
    assert base64.b64decode(raw["clusters"][0]["cluster"]["certificate-authority-data"]).decode() == ca.read_text()
    v = yaml.safe_load(kc(cfgp, "view")[1])
    assert v["clusters"][0]["cluster"]["certificate-authority-data"] == "DATA+OMITTED"
    assert v["users"][0]["user"]["token"] == "REDACTED"
    assert json.loads(kc(cfgp, "view", "--raw", "-o", "json")[1])["users"][0]["user"]["token"] == "s3cret"
    # a second context, then --minify keeps only the current one
    kc(cfgp, "set-cluster", "other", "--server", "http://127.0.0.1:8080")
    kc(cfgp, "set-context", "dev", "--cluster", "other", "--user", "admin")
    m = yaml.safe_load(kc(cfgp, "view", "--minify")[1])
    assert [c["name"] for c in m["contexts"]] == ["prod"] and [c["name"] for c in m["clusters"]] == ["mi"]
    assert kc(cfgp, "get-contexts", "-o", "name")[1].split() == ["prod", "dev"]
    rows = kc(cfgp, "get-contexts", "--no-headers")[1].splitlines()
    assert rows[0].split()[:2] == ["*", "prod"]
    assert kc(cfgp, "get-clusters")[1].split() == ["NAME", "mi", "other"]
    assert kc(cfgp, "set-context", "--current", "--namespace", "team")[1].strip() == 'Context "prod" modified.'
    assert yaml.safe_load(cfgp.read_text())["contexts"][0]["context"]["namespace"] == "team"
    # dotted set / unset (names may contain dots)
    kc(cfgp, "set-cluster", "a.b.c", "--server", "http://x")
    assert kc(cfgp, "set", "clusters.a.b.c.server", "http://y")[0] == 0
    assert [c for c in yaml.safe_load(cfgp.read_text())["clusters"] if c["name"] == "a.b.c"][0]["cluster"]["server"] == "http://y"
    assert kc(cfgp, "set", "users.admin.client-key-data", "PEM")[0] == 0
    assert yaml.safe_load(cfgp.read_text())["users"][0]["user"]["client-key-data"] == base64.b64encode(b"PEM").decode()
    assert kc(cfgp, "unset", "users.admin.token")[0] == 0
    assert "token" not in yaml.safe_load(cfgp.read_text())["users"][0]["user"]
    with pytest.raises(SystemExit, match="invalid"):
        kc(cfgp, "unset", "users.admin.nothing")
    assert kc(cfgp, "rename-context", "dev", "staging")[1].strip() == 'Context "dev" renamed to "staging".'
    assert "deleted context staging" in kc(cfgp, "delete-context", "staging")[1]
    assert "deleted cluster other" in kc(cfgp, "delete-cluster", "other")[1]
    with pytest.raises(SystemExit, match="no context exists"):
        kc(cfgp, "use-context", "gone")
    with pytest.raises(SystemExit, match="more than one authentication method"):
        kc(cfgp, "set-credentials", "x", "--token", "t", "--username", "u")


def test_config_flatten_and_kubeconfig_merge(tmp_path, monkeypatch):
    key = tmp_path / "client.key"
    key.write_text("KEY")
    a, b = tmp_path / "a", tmp_path / "b"
    a.write_text(yaml.safe_dump({"apiVersion": "v1", "kind": "Config", "current-context": "ctx-a",
                                 "clusters": [{"name": "c", "cluster": {"server": "http://a"}}],
                                 "users": [{"name": "u", "user": {"client-key": "client.key"}}],
                                 "contexts": [{"name": "ctx-a", "context": {"cluster": "c", "user": "u"}}]}))
    b.write_text(yaml.safe_dump({"apiVersion": "v1", "kind": "Config", "current-context": "ctx-b",
                                 "clusters": [{"name": "c", "cluster": {"server": "http://b"}},
                                              {"name": "d", "cluster": {"server": "http://d"}}],
                                 "contexts": [{"name": "ctx-b", "context": {"cluster": "d"}}]}))
    monkeypatch.setenv("KUBECONFIG", f"{a}:{b}")
    out = io.StringIO()
    assert kubectl(["config", "view", "--flatten", "--raw"], out=out) == 0
    v = yaml.safe_load(out.getvalue())
    assert v["current-context"] == "ctx-a"                       # first file wins
    assert {c["name"]: c["cluster"]["server"] for c in v["clusters"]} == {"c": "http://a", "d": "http://d"}
    assert base64.b64decode(v["users"][0]["user"]["client-key-data"]) == b"KEY"   # relative to its own file
    out = io.StringIO()
    kubectl(["config", "set-context", "ctx-b", "--namespace", "x"], out=out)
    assert yaml.safe_load(b.read_text())["contexts"][0]["context"]["namespace"] == "x"    # written where it lives
    assert "ctx-b" not in a.read_text()


def test_go_template_and_file_outputs(tmp_path):
    """`-o go-template=` / `template=` / `*-file=` (`pkg/printers/template.go`, customcolumn.go)."""
    from kubernetes_amd.kubectl.gotemplate import TemplateError, render as gt
    from kubernetes_amd.kubectl.printers import render
    pods = [{"kind": "Pod", "metadata": {"name": "a", "labels": {"app": "x"}}, "status": {"phase": "Running"}},
            {"kind": "Pod", "metadata": {"name": "b"}, "status": {"phase": "Pending"}}]
    lst = {"kind": "List", "items": pods}
    assert render(pods, 'go-template={{range .items}}{{.metadata.name}}{{"\\n"}}{{end}}', list_obj=lst) == "a\nb\n"
    t = ('{{range $i, $p := .items}}{{if eq $p.status.phase "Running"}}{{$i}}:up{{else if eq $p.status.phase "Pending"}}'
         '{{$i}}:wait{{else}}?{{end}} {{end}}')
    assert gt(t, lst) == "0:up 1:wait "
    assert gt('{{(index .items 0).metadata.labels}} {{len .items}} {{printf "%s=%d" "n" 2}}', lst) == "map[app:x] 2 n=2"
    assert gt('{{.data.pw | base64decode}}{{with .nope}}x{{else}}-none{{end}} {{.missing}}', {"data": {"pw": "aGk="}}) == \
        "hi-none <no value>"
    assert gt('{{- range .items -}}\n  {{ .metadata.name }}\n{{- end }}', lst) == "ab"
    with pytest.raises(TemplateError):
        gt("{{if .x}}unterminated", {})
    f = tmp_path / "t.tmpl"
    f.write_text("{{range .items}}<{{.metadata.name}}>{{end}}")
    assert render(pods, f"go-template-file={f}", list_obj=lst) == "<a><b>"
    cc = tmp_path / "cols"
    cc.write_text("NAME PHASE\n.metadata.name .status.phase\n")
    out = render(pods, f"custom-columns-file={cc}").splitlines()
    assert out[0].split() == ["NAME", "PHASE"] and out[1].split() == ["a", "Running"]
    jp = tmp_path / "jp"
    jp.write_text("{.items[*].metadata.name}")
    assert render(pods, f"jsonpath-file={jp}", list_obj=lst) == "a b"


def test_rollout_status_viewers():
    """DeploymentStatusViewer / DaemonSetStatusViewer / StatefulSetStatusViewer messages."""
    from kubernetes_amd.kubectl.cli import rollout_status
    md = {"name": "x", "generation": 2}
    d = {"kind": "Deployment", "metadata": md, "spec": {"replicas": 3},
         "status": {"observedGeneration": 1}}
    assert rollout_status(d) == ("Waiting for deployment spec update to be observed...", False)
    d["status"] = {"observedGeneration": 2, "updatedReplicas": 3, "replicas": 4, "availableReplicas": 3}
    assert rollout_status(d) == ("Waiting for rollout to finish: 1 old replicas are pending termination...", False)
    d["status"]["replicas"] = 3
    assert rollout_status(d) == ('deployment "x" successfully rolled out', True)
    ds = {"kind": "DaemonSet", "metadata": md, "spec": {"updateStrategy": {"type": "RollingUpdate"}},
          "status": {"observedGeneration": 2, "desiredNumberScheduled": 4, "updatedNumberScheduled": 4, "numberAvailable": 2}}
    assert rollout_status(ds)[0].endswith("2 of 4 updated pods are available...")
    ss = {"kind": "StatefulSet", "metadata": md,
          "spec": {"replicas": 3, "updateStrategy": {"type": "RollingUpdate", "rollingUpdate": {"partition": 1}}},
          "status": {"observedGeneration": 2, "readyReplicas": 3, "updatedReplicas": 2}}
    assert rollout_status(ss) == ("partitioned roll out complete: 2 new pods have been updated...", True)
    ss["spec"]["updateStrategy"] = {"type": "OnDelete"}
    with pytest.raises(SystemExit, match="OnDelete updateStrategy does not have a Status"):
        rollout_status(ss)


def test_env_file_parsing(tmp_path, monkeypatch):
    from kubernetes_amd.kubectl.extra import _env_file
    f = tmp_path / "e.env"
    f.write_text("# comment\n\nA=1\n  B=two words \nFROM_ENV\nC=x=y\n")
    monkeypatch.setenv("FROM_ENV", "inherited")
    assert _env_file(str(f)) == {"A": "1", "B": "two words ", "FROM_ENV": "inherited", "C": "x=y"}
    f.write_text("1bad key=v\n")
    with pytest.raises(SystemExit, match="not a valid key name"):
        _env_file(str(f))
