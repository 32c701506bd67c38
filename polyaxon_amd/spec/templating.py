"""``{{ expression }}`` rendering for Polyaxonfiles.

The reference renders specs with Jinja over ``declarations`` + the matrix sample (external
polyaxon_schemas; documented in docs/templates/polyaxonfile_specification/sections.md:750-801 and used in
every example, e.g. ``--lr={{ lr }}``).  Jinja is not a dependency here, so expressions are evaluated by a
small, side-effect-free AST interpreter: names, ``a.b`` / ``a['b']`` / ``a[0]`` lookups, literals,
arithmetic, comparisons, boolean ops, conditional expressions, and the ``int/float/str/round/len/min/max/
abs/join`` helpers (``|`` filters of the form ``{{ x | int }}`` are also accepted).

A string that is exactly one ``{{ ... }}`` keeps the native type of its value (so ``lr: "{{ lr }}"``
renders to a float); otherwise values are substituted with ``str()``.
"""
from __future__ import annotations

import ast
import operator
import re
from typing import Any, Dict

_TEMPLATE = re.compile(r"{{\s*(.+?)\s*}}")


class TemplateError(ValueError):
    pass


_BIN = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv,
        ast.FloorDiv: operator.floordiv, ast.Mod: operator.mod, ast.Pow: operator.pow}
_CMP = {ast.Eq: operator.eq, ast.NotEq: operator.ne, ast.Lt: operator.lt, ast.LtE: operator.le, ast.Gt: operator.gt,
        ast.GtE: operator.ge, ast.In: lambda a, b: a in b, ast.NotIn: lambda a, b: a not in b}
_FUNCS = {"int": int, "float": float, "str": str, "round": round, "len": len, "min": min, "max": max, "abs": abs,
          "bool": bool, "join": lambda seq, sep=",": sep.join(str(s) for s in seq), "list": list,
          "lower": lambda s: str(s).lower(), "upper": lambda s: str(s).upper()}


class _Missing:
    pass


def _eval(node: ast.AST, ctx: Dict[str, Any]) -> Any:
    if isinstance(node, ast.Expression):
        return _eval(node.body, ctx)
    if isinstance(node, ast.Constant):
        return node.value
    if isinstance(node, ast.Name):
        if node.id in ctx:
            return ctx[node.id]
        if node.id in _FUNCS:
            return _FUNCS[node.id]
        if node.id in ("true", "True"):
            return True
        if node.id in ("false", "False"):
            return False
        if node.id in ("none", "None", "null"):
            return None
        raise TemplateError(f"undefined template variable `{node.id}`")
    if isinstance(node, ast.Attribute):
        base = _eval(node.value, ctx)
        if isinstance(base, dict) and node.attr in base:
            return base[node.attr]
        raise TemplateError(f"`{node.attr}` not found")
    if isinstance(node, ast.Subscript):
        base = _eval(node.value, ctx)
        key = _eval(node.slice, ctx)
        try:
            return base[key]
        except (KeyError, IndexError, TypeError) as e:
            raise TemplateError(f"bad subscript {key!r}: {e}") from None
    if isinstance(node, ast.BinOp) and type(node.op) in _BIN:
        return _BIN[type(node.op)](_eval(node.left, ctx), _eval(node.right, ctx))
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.BitOr):  # jinja-style filter: x | int
        val = _eval(node.left, ctx)
        f = node.right
        if isinstance(f, ast.Name) and f.id in _FUNCS:
            return _FUNCS[f.id](val)
        if isinstance(f, ast.Call) and isinstance(f.func, ast.Name) and f.func.id in _FUNCS:
            return _FUNCS[f.func.id](val, *[_eval(a, ctx) for a in f.args])
        raise TemplateError("unknown filter")
    if isinstance(node, ast.UnaryOp):
        v = _eval(node.operand, ctx)
        if isinstance(node.op, ast.USub):
            return -v
        if isinstance(node.op, ast.UAdd):
            return +v
        if isinstance(node.op, ast.Not):
            return not v
    if isinstance(node, ast.BoolOp):
        vals = [_eval(v, ctx) for v in node.values]
        return all(vals) if isinstance(node.op, ast.And) else any(vals)
    if isinstance(node, ast.Compare):
        left = _eval(node.left, ctx)
        for op, comp in zip(node.ops, node.comparators):
            right = _eval(comp, ctx)
            if not _CMP[type(op)](left, right):
                return False
            left = right
        return True
    if isinstance(node, ast.IfExp):
        return _eval(node.body, ctx) if _eval(node.test, ctx) else _eval(node.orelse, ctx)
    if isinstance(node, (ast.List, ast.Tuple)):
        return [_eval(e, ctx) for e in node.elts]
    if isinstance(node, ast.Dict):
        return {_eval(k, ctx): _eval(v, ctx) for k, v in zip(node.keys, node.values)}
    if isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id in _FUNCS:
        return _FUNCS[node.func.id](*[_eval(a, ctx) for a in node.args])
    raise TemplateError(f"unsupported template expression: {ast.dump(node)[:80]}")


def evaluate(expr: str, ctx: Dict[str, Any]) -> Any:
    try:
        tree = ast.parse(expr.strip(), mode="eval")
    except SyntaxError as e:
        raise TemplateError(f"invalid template expression `{expr}`: {e}") from None
    return _eval(tree, ctx)


def render_str(s: str, ctx: Dict[str, Any]) -> Any:
    m = _TEMPLATE.fullmatch(s.strip())
    if m:
        return evaluate(m.group(1), ctx)
    return _TEMPLATE.sub(lambda mm: str(evaluate(mm.group(1), ctx)), s)


def render(obj: Any, ctx: Dict[str, Any]) -> Any:
    """Recursively render every string in a parsed YAML/JSON object."""
    if isinstance(obj, str):
        return render_str(obj, ctx) if "{{" in obj else obj
    if isinstance(obj, list):
        return [render(v, ctx) for v in obj]
    if isinstance(obj, dict):
        return {k: render(v, ctx) for k, v in obj.items()}
    return obj


def has_template(obj: Any) -> bool:
    if isinstance(obj, str):
        return bool(_TEMPLATE.search(obj))
    if isinstance(obj, list):
        return any(has_template(v) for v in obj)
    if isinstance(obj, dict):
        return any(has_template(v) for v in obj.values())
    return False
