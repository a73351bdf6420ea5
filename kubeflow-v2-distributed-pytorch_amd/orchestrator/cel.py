"""Tiny evaluator for the CEL subset kfp v2 emits in ``triggerPolicy.condition``.

Grammar (enough for ``dsl.Condition`` comparisons and their conjunctions)::

    expr   := or
    or     := and ('||' and)*
    and    := unary ('&&' unary)*
    unary  := '!' unary | cmp
    cmp    := atom (('=='|'!='|'<'|'<='|'>'|'>=') atom)?
    atom   := '(' expr ')' | NUMBER | STRING | 'true' | 'false'
            | inputs.parameters['NAME'].(int_value|double_value|string_value|bool_value)

No ``eval``: the condition string comes from a job-spec file.
"""
from __future__ import annotations

import json
import re
from typing import Any, Callable, Dict, List, Tuple

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<ref>inputs\.parameters\[(?P<q>['"])(?P<name>.+?)(?P=q)\]\.(?P<acc>int_value|double_value|string_value|bool_value|number_value))
  | (?P<num>-?\d+(\.\d*)?([eE][-+]?\d+)?)
  | (?P<str>"(\\.|[^"\\])*"|'(\\.|[^'\\])*')
  | (?P<op>==|!=|<=|>=|<|>|&&|\|\||!|\(|\))
  | (?P<kw>true|false)
""", re.VERBOSE)


def _tokenize(s: str) -> List[Tuple[str, Any]]:
    pos, out = 0, []
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise ValueError(f"bad condition near {s[pos:pos+20]!r}")
        pos = m.end()
        if m.group("ws"):
            continue
        if m.group("ref"):
            out.append(("ref", (m.group("name"), m.group("acc"))))
        elif m.group("num") is not None and m.group("num") != "":
            t = m.group("num")
            out.append(("lit", float(t) if any(c in t for c in ".eE") else int(t)))
        elif m.group("str"):
            raw = m.group("str")
            out.append(("lit", json.loads('"' + raw[1:-1].replace('"', '\\"') + '"')
                        if raw[0] == "'" else json.loads(raw)))
        elif m.group("op"):
            out.append(("op", m.group("op")))
        elif m.group("kw"):
            out.append(("lit", m.group("kw") == "true"))
    return out


def evaluate(condition: str, params: Dict[str, Dict[str, Any]]) -> bool:
    """``params``: name -> IR value dict (``{"doubleValue": 1.0}`` ...)."""
    toks = _tokenize(condition)
    i = [0]

    def peek():
        return toks[i[0]] if i[0] < len(toks) else (None, None)

    def take():
        t = peek()
        i[0] += 1
        return t

    def value_of(name: str, acc: str):
        if name not in params:
            raise KeyError(f"condition references unknown input {name!r}")
        v = params[name]
        if "doubleValue" in v:
            x: Any = float(v["doubleValue"])
        elif "intValue" in v:
            x = int(v["intValue"])
        else:
            x = v.get("stringValue", "")
        if acc == "double_value" or acc == "number_value":
            return float(x)
        if acc == "int_value":
            return int(float(x))
        if acc == "bool_value":
            return str(x).lower() in ("true", "1")
        return str(x)

    def atom():
        kind, v = take()
        if kind == "op" and v == "(":
            r = expr()
            if take() != ("op", ")"):
                raise ValueError("missing ')'")
            return r
        if kind == "lit":
            return v
        if kind == "ref":
            return value_of(*v)
        raise ValueError(f"unexpected token {v!r}")

    ops: Dict[str, Callable[[Any, Any], bool]] = {
        "==": lambda a, b: a == b, "!=": lambda a, b: a != b, "<": lambda a, b: a < b,
        "<=": lambda a, b: a <= b, ">": lambda a, b: a > b, ">=": lambda a, b: a >= b}

    def cmp():
        a = atom()
        kind, v = peek()
        if kind == "op" and v in ops:
            take()
            b = atom()
            return ops[v](a, b)
        return a

    def unary():
        if peek() == ("op", "!"):
            take()
            return not unary()
        return cmp()

    def and_():
        r = unary()
        while peek() == ("op", "&&"):
            take()
            r = unary() and r
        return r

    def expr():
        r = and_()
        while peek() == ("op", "||"):
            take()
            r = and_() or r
        return r

    result = expr()
    if i[0] != len(toks):
        raise ValueError(f"trailing tokens in condition {condition!r}")
    return bool(result)
