"""`-o go-template=` / `-o template=` (`pkg/printers/template.go`): Go text/template over the
object's JSON form.

Supported: `{{.a.b}}` field chains, `$` (the root) and variables (`{{$x := ...}}`,
`{{range $i, $e := ...}}`), `range` / `if` / `else if` / `else` / `with` / `end`, `{{- -}}`
whitespace trimming, string / number / bool literals, pipelines (`x | printf "%s"`), and the
functions templates in the wild use: index, len, printf, print, println, eq, ne, lt, le, gt,
ge, and, or, not, plus kubectl's `base64decode`. Map iteration is in sorted key order, as in
Go. A missing field renders `<no value>` like Go's default.
"""
from __future__ import annotations

import base64
import json
import re

_TOKEN = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)
_ARG = re.compile(r'\s*("(?:[^"\\]|\\.)*"|`[^`]*`|\(|\)|\||:=|[^\s()|]+)')


class TemplateError(ValueError):
    pass


def _parse_tokens(text):
    """-> list of ("text", str) / ("action", str), with trim markers applied."""
    out, pos = [], 0
    for mt in _TOKEN.finditer(text):
        lit = text[pos:mt.start()]
        if mt.group(1):
            lit = lit.rstrip()
        out.append(["text", lit])
        out.append(["action", mt.group(2).strip(), bool(mt.group(3))])
        pos = mt.end()
    out.append(["text", text[pos:]])
    for i, t in enumerate(out):        # right-trim marker strips the following text's leading space
        if t[0] == "action" and t[2] and i + 1 < len(out):
            out[i + 1][1] = out[i + 1][1].lstrip()
    return [(t[0], t[1]) for t in out if t[0] == "action" or t[1]]


def _build(tokens, i=0, stop=("end",)):
    """-> (node list, index of the stopping token, its text)."""
    nodes = []
    while i < len(tokens):
        kind, s = tokens[i]
        if kind == "text":
            nodes.append(("text", s))
            i += 1
            continue
        word = s.split(None, 1)[0] if s else ""
        if word in ("end", "else") or s.startswith("else "):
            return nodes, i, s
        if s.startswith("/*"):
            i += 1
            continue
        if word in ("range", "if", "with"):
            node, j = _branch(tokens, i + 1, word, s[len(word):].strip())
            nodes.append(node)
            i = j + 1
            continue
        nodes.append(("action", s))
        i += 1
    return nodes, i, ""


def _branch(tokens, i, word, cond):
    """-> (node, index of the closing {{end}}); `else if` nests an if sharing that end."""
    body, j, end = _build(tokens, i)
    alt = []
    if end.startswith("else"):
        rest = end[4:].strip()
        if rest.startswith("if ") and word == "if":
            node, j = _branch(tokens, j + 1, "if", rest[3:].strip())
            return (word, cond, body, [node]), j
        alt, j, end = _build(tokens, j + 1)
    if end != "end":
        raise TemplateError(f"unexpected EOF: {word} has no {{{{end}}}}")
    return (word, cond, body, alt), j


def _truth(v):
    return not (v is None or v is False or v == 0 or v == "" or v == [] or v == {})


def _fmt(fmt, args):
    conv = iter(args)

    def sub(mt):
        spec = mt.group(0)
        if spec == "%%":
            return "%"
        v = next(conv, None)
        if spec[-1] == "v":
            return _str(v)
        if spec[-1] == "q":
            return json.dumps(_str(v))
        if spec[-1] == "d":
            return (spec[:-1] + "d") % int(v)
        if spec[-1] in "fegs":
            return spec % (v if spec[-1] != "s" else _str(v))
        return _str(v)
    return re.sub(r"%[-+# 0-9.]*[a-zA-Z%]", sub, fmt)


def _str(v):
    if v is None:
        return "<no value>"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, (dict, list)):
        return _go_repr(v)
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)


def _go_repr(v):
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_repr(x)}" for k, x in sorted(v.items())) + "]"
    if isinstance(v, list):
        return "[" + " ".join(_go_repr(x) for x in v) + "]"
    return _str(v)


def _cmp(a, b):
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return (a > b) - (a < b)
    a, b = str(a), str(b)
    return (a > b) - (a < b)


FUNCS = {
    "len": lambda x: len(x or ()),
    "index": lambda x, *ks: _index(x, ks),
    "printf": lambda f, *a: _fmt(f, a),
    "print": lambda *a: "".join(_str(x) for x in a),
    "println": lambda *a: " ".join(_str(x) for x in a) + "\n",
    "eq": lambda a, *bs: any(a == b for b in bs),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: _cmp(a, b) < 0,
    "le": lambda a, b: _cmp(a, b) <= 0,
    "gt": lambda a, b: _cmp(a, b) > 0,
    "ge": lambda a, b: _cmp(a, b) >= 0,
    "not": lambda a: not _truth(a),
    "and": lambda *a: next((x for x in a if not _truth(x)), a[-1]),
    "or": lambda *a: next((x for x in a if _truth(x)), a[-1]),
    "base64decode": lambda s: base64.b64decode(s or "").decode(errors="replace"),
    "html": lambda s: _str(s).replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;"),
    "js": lambda s: json.dumps(_str(s))[1:-1],
    "urlquery": lambda *a: __import__("urllib.parse").parse.quote_plus("".join(_str(x) for x in a)),
}


def _index(x, keys):
    for k in keys:
        if x is None:
            return None
        if isinstance(x, list):
            x = x[int(k)] if -len(x) <= int(k) < len(x) else None
        else:
            x = x.get(k) if isinstance(x, dict) else None
    return x


class _Ctx:
    def __init__(self, root):
        self.vars = [{"$": root}]

    def get(self, name):
        for scope in reversed(self.vars):
            if name in scope:
                return scope[name]
        raise TemplateError(f"undefined variable: {name}")

    def set(self, name, v, declare=True):
        if declare:
            self.vars[-1][name] = v
            return
        for scope in reversed(self.vars):
            if name in scope:
                scope[name] = v
                return
        raise TemplateError(f"undefined variable: {name}")


def _field(v, path):
    for part in [p for p in path.split(".") if p]:
        if isinstance(v, dict):
            v = v.get(part)
        else:
            return None
    return v


def _tokenize_args(s):
    out, pos = [], 0
    while pos < len(s):
        mt = _ARG.match(s, pos)
        if not mt or not mt.group(1):
            break
        tok = mt.group(1)
        if out and out[-1] == ")" and mt.start(1) == pos and tok.startswith("."):
            tok = "@" + tok          # `(pipeline).field`: a field of the group's value
        out.append(tok)
        pos = mt.end()
    return out


def _operand(tok, dot, ctx, toks):
    if tok == "(":
        depth, inner = 1, []
        while toks:
            t = toks.pop(0)
            if t == "(":
                depth += 1
            elif t == ")":
                depth -= 1
                if depth == 0:
                    break
            inner.append(t)
        v = _pipeline(inner, dot, ctx)
        while toks and toks[0].startswith("@."):
            v = _field(v, toks.pop(0)[1:])
        return v
    if tok.startswith('"'):
        return json.loads(tok)
    if tok.startswith("`"):
        return tok[1:-1]
    if tok in ("true", "false"):
        return tok == "true"
    if tok == "nil":
        return None
    if re.fullmatch(r"-?\d+", tok):
        return int(tok)
    if re.fullmatch(r"-?\d+\.\d*", tok):
        return float(tok)
    if tok == ".":
        return dot
    if tok.startswith("."):
        return _field(dot, tok)
    if tok.startswith("$"):
        name, _, rest = tok.partition(".")
        return _field(ctx.get(name), rest)
    raise TemplateError(f"function {tok!r} not defined")


def _command(toks, dot, ctx, piped=None, has_piped=False):
    if not toks:
        raise TemplateError("empty command")
    head = toks[0]
    if head in FUNCS:
        rest = list(toks[1:])
        args = []
        while rest:
            args.append(_operand(rest.pop(0), dot, ctx, rest))
        if has_piped:
            args.append(piped)
        try:
            return FUNCS[head](*args)
        except (TypeError, ValueError, IndexError, KeyError) as e:
            raise TemplateError(f"error calling {head}: {e}") from e
    rest = list(toks)
    v = _operand(rest.pop(0), dot, ctx, rest)
    if rest or has_piped:
        raise TemplateError(f"can't give argument to non-function {head}")
    return v


def _pipeline(toks, dot, ctx):
    decl = None
    if len(toks) >= 2 and toks[0].startswith("$") and toks[1] in (":=", "="):
        decl, toks = (toks[0], toks[1] == ":="), toks[2:]
    cmds, cur = [], []
    for t in toks:
        if t == "|":
            cmds.append(cur)
            cur = []
        else:
            cur.append(t)
    cmds.append(cur)
    v, has = None, False
    for c in cmds:
        v = _command(c, dot, ctx, v, has)
        has = True
    if decl:
        ctx.set(decl[0], v, decl[1])
        return _NOPRINT
    return v


_NOPRINT = object()


def _exec(nodes, dot, ctx, out):
    for n in nodes:
        kind = n[0]
        if kind == "text":
            out.append(n[1])
        elif kind == "action":
            v = _pipeline(_tokenize_args(n[1]), dot, ctx)
            if v is not _NOPRINT:
                out.append(_str(v))
        elif kind in ("if", "with"):
            v = _pipeline(_tokenize_args(n[1]), dot, ctx)
            ctx.vars.append({})
            try:
                if _truth(v):
                    _exec(n[2], v if kind == "with" else dot, ctx, out)
                else:
                    _exec(n[3], dot, ctx, out)
            finally:
                ctx.vars.pop()
        elif kind == "range":
            toks = _tokenize_args(n[1])
            kvar = evar = None
            if ":=" in toks:
                names = [t.rstrip(",") for t in toks[:toks.index(":=")] if t != ","]
                toks = toks[toks.index(":=") + 1:]
                if len(names) == 2:
                    kvar, evar = names
                else:
                    evar = names[0]
            v = _pipeline(toks, dot, ctx)
            items = sorted(v.items()) if isinstance(v, dict) else list(enumerate(v or ()))
            if not items:
                _exec(n[3], dot, ctx, out)
                continue
            for k, e in items:
                ctx.vars.append({})
                if kvar:
                    ctx.set(kvar, k)
                if evar:
                    ctx.set(evar, e)
                try:
                    _exec(n[2], e, ctx, out)
                finally:
                    ctx.vars.pop()


def render(template: str, obj) -> str:
    nodes, i, end = _build(_parse_tokens(template))
    if end:
        raise TemplateError(f"unexpected {{{{{end}}}}}")
    out = []
    _exec(nodes, obj, _Ctx(obj), out)
    return "".join(out)
