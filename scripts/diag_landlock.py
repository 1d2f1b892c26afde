"""GPU-box diagnostic for the Landlock isolation tier: what `kamd-runc features` reports, and
whether the HIP vector_add payload runs (a) directly and (b) inside a Landlock-tier container
whose /dev/dri is limited to one render node. Every step has its own time limit."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "kubernetes_amd", "native", "bin")


def run(cmd, timeout=60, **kw):
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, **kw)
        return r.returncode, (r.stdout + r.stderr)[-3000:]
    except subprocess.TimeoutExpired as e:
        return "timeout", ((e.stdout or b"").decode(errors="replace") + (e.stderr or b"").decode(errors="replace"))[-3000:]


def main():
    out = {"uid": os.getuid()}
    out["features"] = run([os.path.join(BIN, "kamd-runc"), "features"], 30)
    out["dev_dri"] = sorted(os.listdir("/dev/dri")) if os.path.isdir("/dev/dri") else None
    renders = sorted(n for n in (out["dev_dri"] or []) if n.startswith("renderD"))
    out["direct"] = run([os.path.join(BIN, "hip-vector-add")], 60)
    if renders:
        mine = "/dev/dri/" + renders[0]
        d = tempfile.mkdtemp(prefix="kamd-ll-diag-")
        spec = {"process": {"args": [os.path.join(BIN, "hip-vector-add")],
                            "env": [f"{k}={v}" for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES",)],
                            "cwd": "/"},
                "root": {"path": "/"}, "mounts": [],
                "annotations": {"kamd.io/isolation-tier": "landlock"},
                "linux": {"devices": [{"path": "/dev/kfd"}, {"path": mine}], "namespaces": []}}
        with open(os.path.join(d, "config.json"), "w") as f:
            json.dump(spec, f)
        out["landlock_run"] = run([os.path.join(BIN, "kamd-runc"), "run", "--bundle", d], 90)
        try:
            out["isolation_json"] = open(os.path.join(d, "isolation.json")).read()
        except OSError as e:
            out["isolation_json"] = str(e)
        probe = ("for n in /dev/dri/*; do if [ -c \"$n\" ]; then if (exec 3<>\"$n\") 2>/dev/null; "
                 "then echo OPEN $n; else echo DENIED $n; fi; fi; done")
        spec["process"]["args"] = ["/bin/sh", "-c", probe]
        with open(os.path.join(d, "config.json"), "w") as f:
            json.dump(spec, f)
        out["landlock_probe"] = run([os.path.join(BIN, "kamd-runc"), "run", "--bundle", d], 30)
        out["host_probe"] = run(["/bin/sh", "-c", probe], 30)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.exit(main())
