"""Reference-doc generators for every component's command line.

Parity: `cmd/gendocs` (markdown), `cmd/genman` (man pages), `cmd/genyaml` (kubectl YAML docs) and
`cmd/genkubedocs`. The parsers are captured from each entry point without running it: the
entry point's `parse_args` is intercepted and the ArgumentParser (with every sub-command) is
walked.

    python -m kubernetes_amd.cmd.gendocs --format md --out docs/cli
"""
from __future__ import annotations

import argparse
import datetime
import importlib
import os
import sys

import yaml

COMPONENTS = {"kube-apiserver": "apiserver", "kube-controller-manager": "controller_manager",
              "kube-scheduler": "scheduler", "kubelet": "kubelet", "kube-proxy": "proxy", "kubectl": "kubectl",
              "kubeadm": "kubeadm", "kube-dns": "dns", "kube-addon-manager": "addon_manager", "kamd-cri": "cri",
              "amd-gpu-device-plugin": "device_plugin", "csi-hostpath": "csi_hostpath",
              "node-problem-detector": "npd", "log-shipper": "log_shipper", "amd-smi-exporter": "amd_smi_exporter"}


class _Captured(Exception):
    def __init__(self, parser):
        super().__init__("captured")
        self.parser = parser


def capture_parser(module_name):
    """The ArgumentParser an entry point builds, captured at its first parse_args call."""
    mod = importlib.import_module(f"kubernetes_amd.cmd.{module_name}")
    if module_name == "kubectl":
        from ..kubectl.cli import build_parser
        return build_parser()
    orig = argparse.ArgumentParser.parse_args

    def grab(self, *a, **kw):
        raise _Captured(self)
    argparse.ArgumentParser.parse_args = grab
    try:
        mod.main([])
    except _Captured as c:
        return c.parser
    except SystemExit:
        pass
    finally:
        argparse.ArgumentParser.parse_args = orig
    raise RuntimeError(f"{module_name}: no parser captured")


def _options(parser):
    out = []
    for act in parser._actions:  # noqa: SLF001 - argparse has no public walker
        if isinstance(act, (argparse._HelpAction, argparse._SubParsersAction)) or not act.option_strings:  # noqa: SLF001
            continue
        if act.help == argparse.SUPPRESS:
            continue
        default = None if act.default in (None, argparse.SUPPRESS, False, [], "") else act.default
        out.append({"name": ", ".join(act.option_strings), "default": default, "usage": act.help or ""})
    return out


def _positionals(parser):
    return [a.dest for a in parser._actions if not a.option_strings and not isinstance(a, argparse._SubParsersAction)]  # noqa: SLF001


def walk(parser, path):
    """Yield (command path, parser) for the parser and every sub-command, depth first."""
    yield path, parser
    for act in parser._actions:  # noqa: SLF001
        if isinstance(act, argparse._SubParsersAction):  # noqa: SLF001
            seen = set()
            for name, sub in act.choices.items():
                if id(sub) in seen:          # aliases share a parser
                    continue
                seen.add(id(sub))
                yield from walk(sub, path + [name])


def to_markdown(path, parser):
    title = " ".join(path)
    lines = [f"## {title}", "", parser.description or "", "", "```", parser.format_usage().strip(), "```", ""]
    pos = _positionals(parser)
    if pos:
        lines += ["Arguments: " + ", ".join(f"`{p}`" for p in pos), ""]
    opts = _options(parser)
    if opts:
        lines += ["| option | default | description |", "|---|---|---|"]
        for o in opts:
            d = "" if o["default"] is None else f"`{o['default']}`"
            lines.append(f"| `{o['name']}` | {d} | {o['usage'].replace('|', '/')} |")
        lines.append("")
    return "\n".join(lines)


def to_man(path, parser):
    title = "-".join(path).upper()
    date = datetime.date.today().isoformat()
    out = [f'.TH "{title}" "1" "{date}" "kubernetes-amd" "Kubernetes on MI355X"', ".SH NAME",
           f"{' '.join(path)}", ".SH SYNOPSIS", parser.format_usage().strip().replace("-", "\\-"), ".SH OPTIONS"]
    for o in _options(parser):
        out += [".TP", f"\\fB{o['name'].replace('-', chr(92) + '-')}\\fP",
                (o["usage"] or "").replace("-", "\\-") + (f" (default {o['default']})" if o["default"] is not None else "")]
    return "\n".join(out) + "\n"


def to_yaml(path, parser):
    return {"name": " ".join(path), "synopsis": (parser.description or "").strip(),
            "usage": parser.format_usage().strip(), "options": _options(parser)}


def parsers():
    """{"component sub command": parser} for every component and sub-command (hack/verify.py's
    flag checks walk these)."""
    out = {}
    for comp, mod in COMPONENTS.items():
        for path, sp in walk(capture_parser(mod), [comp]):
            out[" ".join(path)] = sp
    return out


def generate(out_dir, fmt="md", components=None):
    os.makedirs(out_dir, exist_ok=True)
    written = []
    for comp, mod in COMPONENTS.items():
        if components and comp not in components:
            continue
        parser = capture_parser(mod)
        parser.prog = comp
        entries = list(walk(parser, [comp]))
        if fmt == "md":
            p = os.path.join(out_dir, f"{comp}.md")
            with open(p, "w") as f:
                f.write(f"# {comp}\n\n" + "\n".join(to_markdown(path, sp) for path, sp in entries))
            written.append(p)
        elif fmt == "man":
            for path, sp in entries:
                p = os.path.join(out_dir, "-".join(path) + ".1")
                with open(p, "w") as f:
                    f.write(to_man(path, sp))
                written.append(p)
        else:
            p = os.path.join(out_dir, f"{comp}.yaml")
            with open(p, "w") as f:
                yaml.safe_dump([to_yaml(path, sp) for path, sp in entries], f, sort_keys=False)
            written.append(p)
    return written


def main(argv=None):
    ap = argparse.ArgumentParser("gendocs")
    ap.add_argument("--format", choices=["md", "man", "yaml"], default="md")
    ap.add_argument("--out", default="docs/cli")
    ap.add_argument("components", nargs="*")
    a = ap.parse_args(argv)
    files = generate(a.out, a.format, a.components or None)
    print(f"wrote {len(files)} files to {a.out}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
