"""Go `text/template` subset for Ollama Modelfile TEMPLATE layers and the
prompt assembly of /api/generate and /api/chat.

Supported: {{ }} actions with `-` trim markers, comments, field chains (.A.B, $.A, $v.A),
variables ($x := / =), if / else if / else / end, range (with `$i, $v :=`), with, pipelines with
`|`, parenthesised calls, literals, and the functions eq ne lt le gt ge and or not len index slice
print printf println json.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass
from typing import Any

RESPONSE_MARK = "\x00__OMX_RESPONSE__\x00"


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------------------------------------
# lexing: split into text and {{ action }} pieces, applying trim markers
_ACTION = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)


def _split(src: str) -> list[tuple[str, str]]:
    out: list[tuple[str, str]] = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        out.append(("text", text))
        body = m.group(2).strip()
        out.append(("act", body))
        pos = m.end()
        if m.group(3):
            rest = src[pos:]
            pos += len(rest) - len(rest.lstrip())
    out.append(("text", src[pos:]))
    return [p for p in out if not (p[0] == "text" and p[1] == "")]


_TOK = re.compile(r'''\s*(?:(?P<str>"(?:[^"\\]|\\.)*"|`[^`]*`)|(?P<num>-?\d+(?:\.\d+)?)|(?P<decl>:=)|(?P<asg>=)|'''
                  r'''(?P<sym>[()|,])|(?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)|(?P<field>(?:\.[A-Za-z0-9_]+)+|\.)|'''
                  r'''(?P<ident>[A-Za-z_][A-Za-z0-9_]*))''')


def _tokens(s: str) -> list[tuple[str, str]]:
    out = []
    pos = 0
    s = s.rstrip()
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            raise TemplateError(f"bad token in {{{{ {s} }}}} at {pos}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        pos = m.end()
    return out


# ------------------------------------------------------------------------------------------------
# AST
@dataclass
class Text:
    s: str


@dataclass
class Action:
    pipe: Any  # Pipeline


@dataclass
class If:
    branches: list  # [(pipeline, nodes)]
    else_: list


@dataclass
class Range:
    decl: list
    pipe: Any
    body: list
    else_: list


@dataclass
class With:
    pipe: Any
    body: list
    else_: list


@dataclass
class Pipeline:
    decl: list          # variable names declared (:=) or assigned (=)
    assign: bool
    cmds: list          # list of commands; each command = list of args


class Parser:
    def __init__(self, src: str):
        self.parts = _split(src)
        self.i = 0

    def parse(self) -> list:
        nodes, end = self._list(())
        if end is not None:
            raise TemplateError(f"unexpected {{{{ {end} }}}}")
        return nodes

    def _list(self, stops: tuple) -> tuple[list, str | None]:
        nodes: list = []
        while self.i < len(self.parts):
            kind, body = self.parts[self.i]
            self.i += 1
            if kind == "text":
                nodes.append(Text(body))
                continue
            if body.startswith("/*"):
                continue
            word = body.split(None, 1)[0] if body else ""
            if word in stops:
                return nodes, body
            if word == "if":
                nodes.append(self._if(body[2:].strip()))
            elif word == "range":
                nodes.append(self._range(body[5:].strip()))
            elif word == "with":
                p = parse_pipeline(body[4:].strip())
                b, e = self._list(("else", "end"))
                els: list = []
                if e and e.startswith("else"):
                    els, _ = self._list(("end",))
                nodes.append(With(p, b, els))
            elif word in ("end", "else"):
                raise TemplateError(f"unexpected {{{{ {body} }}}}")
            elif word in ("define", "template", "block"):
                raise TemplateError(f"{word} is not supported")
            else:
                nodes.append(Action(parse_pipeline(body)))
        return nodes, None

    def _if(self, cond: str) -> If:
        branches = []
        p = parse_pipeline(cond)
        while True:
            body, end = self._list(("else", "end"))
            branches.append((p, body))
            if end is None:
                raise TemplateError("unterminated if")
            if end == "end":
                return If(branches, [])
            rest = end[4:].strip()
            if rest.startswith("if "):
                p = parse_pipeline(rest[3:].strip())
                continue
            els, end2 = self._list(("end",))
            if end2 is None:
                raise TemplateError("unterminated if/else")
            return If(branches, els)

    def _range(self, spec: str) -> Range:
        p = parse_pipeline(spec)
        body, end = self._list(("else", "end"))
        els: list = []
        if end and end.startswith("else"):
            els, _ = self._list(("end",))
        elif end is None:
            raise TemplateError("unterminated range")
        return Range(p.decl, Pipeline([], False, p.cmds), body, els)


def parse_pipeline(s: str) -> Pipeline:
    toks = _tokens(s)
    decl: list = []
    assign = False
    # `$a, $b :=` / `$a :=` / `$a =`
    j = 0
    names = []
    while j < len(toks) and toks[j][0] == "var":
        names.append(toks[j][1])
        if j + 1 < len(toks) and toks[j + 1] == ("sym", ","):
            j += 2
            continue
        j += 1
        break
    if names and j < len(toks) and toks[j][0] in ("decl", "asg"):
        decl = names
        assign = toks[j][0] == "asg"
        toks = toks[j + 1:]
    cmds, rest = _parse_cmds(toks, 0)
    if rest != len(toks):
        raise TemplateError(f"trailing tokens in {s!r}")
    return Pipeline(decl, assign, cmds)


def _parse_cmds(toks, i):
    cmds = []
    cur: list = []
    while i < len(toks):
        k, v = toks[i]
        if (k, v) == ("sym", ")"):
            break
        if (k, v) == ("sym", "|"):
            cmds.append(cur)
            cur = []
            i += 1
            continue
        if (k, v) == ("sym", "("):
            sub, i = _parse_cmds(toks, i + 1)
            if i >= len(toks) or toks[i] != ("sym", ")"):
                raise TemplateError("unbalanced parenthesis")
            cur.append(("pipe", Pipeline([], False, sub)))
            i += 1
            continue
        cur.append((k, v))
        i += 1
    cmds.append(cur)
    return cmds, i


# ------------------------------------------------------------------------------------------------
# evaluation
def truthy(v: Any) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, tuple, dict)):
        return len(v) > 0
    return True


def _field(obj: Any, name: str) -> Any:
    if obj is None:
        return None
    if isinstance(obj, dict):
        if name in obj:
            return obj[name]
        low = {k.lower(): v for k, v in obj.items()}
        return low.get(name.lower())
    return getattr(obj, name, None)


def _cmp(a, b):
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return (a > b) - (a < b)
    a, b = str(a), str(b)
    return (a > b) - (a < b)


def _printf(fmt, *args):
    out = re.sub(r"%(?:\d+)?[vdsqf]", "{}", fmt)
    vals = [json.dumps(a) if fmt.count("%q") else a for a in args]
    try:
        return out.format(*vals)
    except (IndexError, KeyError):
        return fmt


FUNCS = {
    "eq": lambda a, *bs: any(a == b for b in bs),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: _cmp(a, b) < 0,
    "le": lambda a, b: _cmp(a, b) <= 0,
    "gt": lambda a, b: _cmp(a, b) > 0,
    "ge": lambda a, b: _cmp(a, b) >= 0,
    "not": lambda a: not truthy(a),
    "len": lambda a: len(a) if a is not None else 0,
    "index": lambda a, *ks: _index(a, ks),
    "slice": lambda a, *ix: a[ix[0]:(ix[1] if len(ix) > 1 else None)] if a is not None else a,
    "print": lambda *a: "".join(str(x) for x in a),
    "println": lambda *a: " ".join(str(x) for x in a) + "\n",
    "printf": _printf,
    "json": lambda a: json.dumps(a),
    "toJson": lambda a: json.dumps(a),
}


def _index(a, ks):
    for k in ks:
        a = a[k] if a is not None else None
    return a


class Renderer:
    def __init__(self, root: Any):
        self.root = root
        self.vars: list[dict] = [{"$": root}]

    def lookup(self, name: str):
        for scope in reversed(self.vars):
            if name in scope:
                return scope[name]
        raise TemplateError(f"undefined variable {name}")

    def set_var(self, name, value, declare):
        if declare:
            self.vars[-1][name] = value
            return
        for scope in reversed(self.vars):
            if name in scope:
                scope[name] = value
                return
        raise TemplateError(f"undefined variable {name}")

    def arg(self, tok, dot):
        k, v = tok
        if k == "str":
            return json.loads(v) if v.startswith('"') else v[1:-1]
        if k == "num":
            return float(v) if "." in v else int(v)
        if k == "field":
            if v == ".":
                return dot
            o = dot
            for part in v.split(".")[1:]:
                o = _field(o, part)
            return o
        if k == "var":
            parts = v.split(".")
            o = self.lookup(parts[0])
            for part in parts[1:]:
                o = _field(o, part)
            return o
        if k == "pipe":
            return self.pipeline(v, dot)
        if k == "ident":
            if v == "true":
                return True
            if v == "false":
                return False
            if v == "nil":
                return None
            if v in FUNCS:
                return FUNCS[v]()
            raise TemplateError(f"unknown function {v}")
        raise TemplateError(f"bad argument {v}")

    def command(self, cmd, dot, prev=None, has_prev=False):
        if not cmd:
            raise TemplateError("empty command")
        head = cmd[0]
        if head[0] == "ident" and head[1] in FUNCS and head[1] not in ("true", "false", "nil"):
            args = [self.arg(t, dot) for t in cmd[1:]]
            if has_prev:
                args.append(prev)
            if head[1] == "and":
                pass
            return FUNCS[head[1]](*args)
        if head[0] == "ident" and head[1] in ("and", "or"):
            vals = [self.arg(t, dot) for t in cmd[1:]] + ([prev] if has_prev else [])
            if head[1] == "and":
                for x in vals:
                    if not truthy(x):
                        return x
                return vals[-1] if vals else None
            for x in vals:
                if truthy(x):
                    return x
            return vals[-1] if vals else None
        if len(cmd) > 1:
            raise TemplateError(f"cannot call non-function {head[1]}")
        return self.arg(head, dot)

    def pipeline(self, p: Pipeline, dot):
        val = None
        has = False
        for cmd in p.cmds:
            val = self.command(cmd, dot, val, has)
            has = True
        if p.decl:
            self.set_var(p.decl[-1], val, not p.assign)
        return val

    def render(self, nodes, dot, out: list):
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Action):
                v = self.pipeline(n.pipe, dot)
                if not n.pipe.decl:
                    out.append(_fmt(v))
            elif isinstance(n, If):
                for p, body in n.branches:
                    if truthy(self.pipeline(p, dot)):
                        self.scoped(body, dot, out)
                        break
                else:
                    self.scoped(n.else_, dot, out)
            elif isinstance(n, With):
                v = self.pipeline(n.pipe, dot)
                if truthy(v):
                    self.scoped(n.body, v, out)
                else:
                    self.scoped(n.else_, dot, out)
            elif isinstance(n, Range):
                seq = self.pipeline(n.pipe, dot)
                items = list(seq.items()) if isinstance(seq, dict) else list(enumerate(seq or []))
                if not items:
                    self.scoped(n.else_, dot, out)
                for k, v in items:
                    self.vars.append({})
                    if len(n.decl) == 1:
                        self.vars[-1][n.decl[0]] = v
                    elif len(n.decl) == 2:
                        self.vars[-1][n.decl[0]] = k
                        self.vars[-1][n.decl[1]] = v
                    self.render(n.body, v, out)
                    self.vars.pop()

    def scoped(self, nodes, dot, out):
        self.vars.append({})
        self.render(nodes, dot, out)
        self.vars.pop()


def _fmt(v) -> str:
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (list, dict)):
        return json.dumps(v)
    return str(v)


class Template:
    def __init__(self, src: str):
        self.src = src
        self.nodes = Parser(src).parse()

    def render(self, data: dict) -> str:
        out: list[str] = []
        Renderer(data).render(self.nodes, data, out)
        return "".join(out)

    @property
    def uses_messages(self) -> bool:
        return ".Messages" in self.src


DEFAULT_TEMPLATE = "{{ .Prompt }}"


def _msg(m: dict) -> dict:
    return {"Role": m.get("role", ""), "Content": m.get("content", ""), "Images": m.get("images"),
            "ToolCalls": m.get("tool_calls")}


def render_generate(template: str | None, prompt: str, system: str | None, suffix: str | None = None) -> str:
    t = Template(template or DEFAULT_TEMPLATE)
    if t.uses_messages:
        msgs = ([{"role": "system", "content": system}] if system else []) + [{"role": "user", "content": prompt}]
        return render_chat(template, msgs, None)
    out = t.render({"System": system or "", "Prompt": prompt, "Response": RESPONSE_MARK, "Suffix": suffix or ""})
    return out.split(RESPONSE_MARK, 1)[0]


def render_chat(template: str | None, messages: list[dict], default_system: str | None,
                tools: list | None = None) -> str:
    """Ollama chat prompt: `.Messages` templates render once; legacy System/Prompt/Response
    templates render turn by turn, the final turn cut at `{{ .Response }}`."""
    t = Template(template or DEFAULT_TEMPLATE)
    msgs = list(messages)
    if default_system and not any(m.get("role") == "system" for m in msgs):
        msgs.insert(0, {"role": "system", "content": default_system})
    if t.uses_messages:
        sys_txt = "\n\n".join(m.get("content", "") for m in msgs if m.get("role") == "system")
        data = {"Messages": [_msg(m) for m in msgs], "System": sys_txt, "Prompt": "", "Response": "",
                "Tools": tools or []}
        return t.render(data)
    out = []
    system, prompt = "", None
    for m in msgs:
        role, content = m.get("role"), m.get("content", "")
        if role == "system":
            system = (system + "\n\n" + content) if system else content
        elif role == "user":
            if prompt is not None:
                out.append(t.render({"System": system, "Prompt": prompt, "Response": ""}))
                system = ""
            prompt = content
        elif role in ("assistant", "tool"):
            out.append(t.render({"System": system, "Prompt": prompt or "", "Response": content}))
            system, prompt = "", None
    if prompt is not None or system:
        last = t.render({"System": system, "Prompt": prompt or "", "Response": RESPONSE_MARK})
        out.append(last.split(RESPONSE_MARK, 1)[0])
    return "".join(out)
