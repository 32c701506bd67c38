"""Query DSL → SQL for the tracking store.

Grammar (docs/templates/query_syntax/introduction.md; reference parser polyaxon/query/parser.py:6-255 and
builder query/builder.py:16-266): comma-separated conditions ``field:expr`` (all must hold);
``~`` negates; value conditions ``a|b|c``; scalar conditions ``>v >=v <v <=v v``; datetime conditions
with the scalar operators or a ``start .. end`` range.  Field proxies as in
query/managers/experiment.py:21-91: ``metric.<name>`` → ``last_metric``, ``declarations.<name>``,
``status``, ``group``, ``project``, ``commit``, ``tags``, ``independent``...

Sorting: comma-separated fields, ``-`` prefix for descending, ``metric.<name>`` allowed.
"""
from __future__ import annotations

import datetime as _dt
import re
from dataclasses import dataclass
from typing import Any, List, Optional, Tuple


class QueryError(ValueError):
    pass


@dataclass
class Condition:
    field: str
    subfield: Optional[str]
    negation: bool
    op: str  # "=", "!=", ">", ">=", "<", "<=", "in", "range"
    value: Any


_NEG_OPS = {"=": "!=", ">": "<=", ">=": "<", "<": ">=", "<=": ">", "in": "not in", "range": "not range"}


def split_query(query: str) -> List[Tuple[str, str]]:
    out = []
    for part in [p for p in query.split(",") if p.strip()]:
        if ":" not in part:
            raise QueryError(f"query condition `{part.strip()}` needs the form field:value")
        field, expr = part.split(":", 1)
        field, expr = field.strip(), expr.strip()
        if not field or not expr:
            raise QueryError(f"query condition `{part.strip()}` is incomplete")
        out.append((field, expr))
    return out


def _parse_number(s: str):
    try:
        return int(s)
    except ValueError:
        try:
            return float(s)
        except ValueError:
            raise QueryError(f"expected a number, got `{s}`") from None


def parse_datetime(s: str) -> float:
    s = s.strip()
    for fmt in ("%Y-%m-%d %H:%M:%S", "%Y-%m-%d %H:%M", "%Y-%m-%dT%H:%M:%S", "%Y-%m-%d"):
        try:
            return _dt.datetime.strptime(s, fmt).replace(tzinfo=_dt.timezone.utc).timestamp()
        except ValueError:
            continue
    raise QueryError(f"invalid datetime `{s}` (YYYY-MM-DD[ HH:MM[:SS]])")


def parse_comparison(expr: str) -> Tuple[Optional[str], str]:
    """Leading comparison operator (reference parse_comparison_operation, query/parser.py:25-41): ``<=``/``=<``,
    ``>=``/``=>``, ``<``, ``>``; None when there is none."""
    e = expr.strip()
    if e[:2] in ("<=", "=<"):
        return "<=", e[2:].strip()
    if e[:2] in (">=", "=>"):
        return ">=", e[2:].strip()
    if e[:1] in ("<", ">"):
        return e[:1], e[1:].strip()
    if e[:1] == "=":
        return "=", e[1:].strip()
    return None, e


def parse_scalar(expr: str, number=True) -> Tuple[bool, str, Any]:
    """Scalar condition: ``[~][op]value``.  ``|`` and ``..`` are not allowed (reference query/parser.py:104-109)."""
    if not expr.strip():
        raise QueryError("empty scalar condition")
    if number:
        if "|" in expr:
            raise QueryError(f"`|` is not allowed for scalar operations: `{expr}`")
        if ".." in expr:
            raise QueryError(f"`..` is not allowed for scalar operations: `{expr}`")
    neg = expr.startswith("~")
    if neg:
        expr = expr[1:].strip()
    op, raw = parse_comparison(expr)
    op = op or "="
    if not raw:
        raise QueryError("empty scalar condition")
    val = _parse_number(raw) if number else raw
    return neg, op, val


def parse_value(expr: str) -> Tuple[bool, str, Any]:
    neg = expr.startswith("~")
    if neg:
        expr = expr[1:].strip()
    vals = [v.strip() for v in expr.split("|") if v.strip()]
    if not vals:
        raise QueryError("empty value condition")
    return (neg, "in", vals) if len(vals) > 1 else (neg, "=", vals[0])


def parse_datetime_op(expr: str) -> Tuple[bool, str, Any]:
    """Datetime condition (reference parse_datetime_operation): a comparison or an ``a .. b`` range; ``|`` is not
    allowed and a range takes exactly two bounds."""
    if "|" in expr:
        raise QueryError(f"`|` is not allowed for datetime operations: `{expr}`")
    neg = expr.startswith("~")
    if neg:
        expr = expr[1:].strip()
    if ".." in expr:
        parts = [p.strip() for p in expr.split("..") if p.strip()]
        if len(parts) != 2:
            raise QueryError(f"a datetime range needs exactly 2 bounds: `{expr}`")
        return neg, "range", (parse_datetime(parts[0]), parse_datetime(parts[1]))
    op, raw = parse_comparison(expr)
    if not raw:
        raise QueryError("empty datetime condition")
    return neg, op or "=", parse_datetime(raw)


class BaseQuery:
    TABLE_ALIAS = "e"
    FIELDS = {}  # name -> (kind, sql column or callable)
    PROXIES = {}

    def parse(self, query: str) -> List[Condition]:
        conds = []
        for field, expr in split_query(query):
            name, _, sub = field.partition(".")
            name = self.PROXIES.get(name, name)
            if name not in self.FIELDS:
                raise QueryError(f"unknown query field `{name}`")
            kind = self.FIELDS[name][0]
            if kind in ("json_scalar",):
                if not sub:
                    raise QueryError(f"`{name}` needs a key, e.g. {name}.loss")
                neg, op, val = parse_scalar(expr)
            elif kind == "json_value":
                if not sub:
                    raise QueryError(f"`{name}` needs a key")
                neg, op, val = parse_value(expr)
            elif kind == "datetime":
                neg, op, val = parse_datetime_op(expr)
            elif kind == "scalar":
                neg, op, val = parse_scalar(expr)
            else:
                neg, op, val = parse_value(expr)
            conds.append(Condition(name, sub or None, neg, op, val))
        return conds

    def _column(self, c: Condition) -> Tuple[str, List[Any]]:
        kind, col = self.FIELDS[c.field][:2]
        a = self.TABLE_ALIAS
        if kind in ("json_scalar", "json_value"):
            return f"json_extract({a}.{col}, ?)", [f'$."{c.subfield}"']
        return f"{a}.{col}", []

    def where(self, query: str) -> Tuple[List[str], List[Any]]:
        clauses, params = [], []
        for c in self.parse(query):
            kind = self.FIELDS[c.field][0]
            op = _NEG_OPS[c.op] if c.negation else c.op
            if c.negation and c.op == "!=":
                op = "="
            if kind == "tags":
                vals = c.value if isinstance(c.value, list) else [c.value]
                sub = (f"EXISTS (SELECT 1 FROM json_each({self.TABLE_ALIAS}.tags) WHERE value IN "
                       f"({', '.join('?' * len(vals))}))")
                clauses.append(("NOT " if c.negation else "") + sub)
                params.extend(vals)
                continue
            if kind == "bool":
                truth = str(c.value).lower() in ("1", "true", "yes")
                if c.negation:
                    truth = not truth
                clauses.append(self.FIELDS[c.field][1] if truth else f"NOT ({self.FIELDS[c.field][1]})")
                continue
            if kind == "subquery":
                sql_tmpl = self.FIELDS[c.field][1]
                vals = c.value if isinstance(c.value, list) else [c.value]
                sub = sql_tmpl.format(ph=", ".join("?" * len(vals)))
                clauses.append(("NOT " if c.negation else "") + sub)
                params.extend(vals)
                continue
            col, cparams = self._column(c)
            if op in ("in", "not in"):
                vals = [_coerce(v) for v in c.value]
                clauses.append(f"{col} {op.upper()} ({', '.join('?' * len(vals))})")
                params.extend(cparams + vals)
            elif op in ("range", "not range"):
                lo, hi = c.value
                expr = f"{col} BETWEEN ? AND ?"
                clauses.append(expr if op == "range" else f"NOT ({expr})")
                params.extend(cparams + [lo, hi])
            else:
                sql_op = {"=": "=", "!=": "!="}.get(op, op)
                if kind == "datetime" and op in ("=", "!="):
                    # equality on a date means "within that second/day"
                    lo = c.value
                    hi = lo + 86400 if _is_midnight(lo) else lo + 1
                    expr = f"({col} >= ? AND {col} < ?)"
                    clauses.append(expr if op == "=" else f"NOT {expr}")
                    params.extend(cparams + [lo] + cparams + [hi])
                    continue
                clauses.append(f"{col} {sql_op} ?")
                params.extend(cparams + [_coerce(c.value)])
        return clauses, params

    def order_by(self, sort: str) -> str:
        parts = []
        for s in [p.strip() for p in sort.split(",") if p.strip()]:
            desc = s.startswith("-")
            s = s.lstrip("-").strip()
            name, _, sub = s.partition(".")
            name = self.PROXIES.get(name, name)
            if name not in self.FIELDS:
                raise QueryError(f"unknown sort field `{name}`")
            kind, col = self.FIELDS[name][:2]
            a = self.TABLE_ALIAS
            if kind in ("json_scalar", "json_value"):
                if not sub or not re.fullmatch(r"[A-Za-z0-9_\-]+", sub):
                    raise QueryError(f"invalid sort key `{s}`")
                expr = f"json_extract({a}.{col}, '$.\"{sub}\"')"
            elif kind in ("tags", "bool", "subquery"):
                raise QueryError(f"cannot sort by `{name}`")
            else:
                expr = f"{a}.{col}"
            # metrics: a missing or non-finite value (a string, store/db.py _json_safe) sorts last either way
            last = f"typeof({expr}) NOT IN ('integer', 'real')" if col == "last_metric" else f"{expr} IS NULL"
            parts.append(f"{last}, {expr} {'DESC' if desc else 'ASC'}")
        parts.append(f"{self.TABLE_ALIAS}.id ASC")
        return ", ".join(parts)


def _is_midnight(ts: float) -> bool:
    return ts % 86400 == 0


def _coerce(v):
    if isinstance(v, str):
        try:
            return int(v)
        except ValueError:
            try:
                return float(v)
            except ValueError:
                return v
    return v


class ExperimentQuery(BaseQuery):
    PROXIES = {"metric": "metric", "metrics": "metric", "group": "group", "experiment_group": "group"}
    FIELDS = {
        "id": ("value", "id"),
        "created_at": ("datetime", "created_at"),
        "updated_at": ("datetime", "updated_at"),
        "started_at": ("datetime", "started_at"),
        "finished_at": ("datetime", "finished_at"),
        "name": ("value", "name"),
        "user": ("value", "user"),
        "status": ("value", "status"),
        "group": ("value", "group_id"),
        "build": ("value", "build_job_id"),
        "framework": ("value", "framework"),
        "project": ("subquery", "e.project_id IN (SELECT id FROM projects WHERE name IN ({ph}))"),
        "commit": ("subquery", "e.code_reference_id IN (SELECT id FROM code_references WHERE commit_sha IN ({ph}))"),
        "declarations": ("json_value", "declarations"),
        "tags": ("tags", "tags"),
        "metric": ("json_scalar", "last_metric"),
        "independent": ("bool", "e.group_id IS NULL"),
    }


class GroupQuery(BaseQuery):
    FIELDS = {
        "id": ("value", "id"),
        "created_at": ("datetime", "created_at"),
        "updated_at": ("datetime", "updated_at"),
        "started_at": ("datetime", "started_at"),
        "finished_at": ("datetime", "finished_at"),
        "name": ("value", "name"),
        "user": ("value", "user"),
        "status": ("value", "status"),
        "search_algorithm": ("value", "search_algorithm"),
        "concurrency": ("scalar", "concurrency"),
        "tags": ("tags", "tags"),
    }


class JobQuery(BaseQuery):
    FIELDS = {
        "id": ("value", "id"),
        "created_at": ("datetime", "created_at"),
        "updated_at": ("datetime", "updated_at"),
        "started_at": ("datetime", "started_at"),
        "finished_at": ("datetime", "finished_at"),
        "name": ("value", "name"),
        "user": ("value", "user"),
        "status": ("value", "status"),
        "kind": ("value", "kind"),
        "tags": ("tags", "tags"),
    }
