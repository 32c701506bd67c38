"""Query DSL parser and SQL builder, golden cases.

Adapted from the reference's tests/test_query/test_parser.py and test_builder.py (the grammar of
query/parser.py:6-255: `field:value`, `~` negation, `a|b` membership, `a..b` ranges, scalar comparisons,
datetime operations).  Differences kept on purpose: datetimes may carry a time of day (`HH:MM[:SS]`), so
`field:value` splits on the FIRST colon only."""
import pytest

from polyaxon_amd.store.query import (ExperimentQuery, GroupQuery, JobQuery, QueryError, parse_datetime,
                                      parse_datetime_op, parse_scalar, parse_value, split_query)


@pytest.mark.parametrize("bad", ["foo", "fff:", ":dsf", ":", " : ", "a:1, b"])
def test_split_rejects_incomplete_conditions(bad):
    with pytest.raises(QueryError):
        split_query(bad)


def test_split_strips_whitespace():
    assert split_query("foo:bar") == [("foo", "bar")]
    assert split_query(" foo: bar ") == [("foo", "bar")]
    assert split_query("foo :>=bar ") == [("foo", ">=bar")]
    assert split_query(" foo :bar|moo|boo") == [("foo", "bar|moo|boo")]
    assert split_query(" foo : bar..moo ") == [("foo", "bar..moo")]
    assert split_query(" foo : ~bar ") == [("foo", "~bar")]
    assert split_query("a:1, b:2,,") == [("a", "1"), ("b", "2")]
    assert split_query("created_at:2020-01-01 10:00") == [("created_at", "2020-01-01 10:00")]


@pytest.mark.parametrize("expr,expected", [
    ("1", (False, "=", 1)),
    ("0.5", (False, "=", 0.5)),
    (">=1", (False, ">=", 1)),
    ("<0.1", (False, "<", 0.1)),
    ("~>=0.1", (True, ">=", 0.1)),
    ("~ <= 3", (True, "<=", 3)),
    ("-2", (False, "=", -2)),
    ("1e-3", (False, "=", 1e-3)),
])
def test_scalar_operations(expr, expected):
    assert parse_scalar(expr) == expected


@pytest.mark.parametrize("bad", ["1|12", "0.1..0.2", ">=f", "~ <=f1", "~ > bbb", "~", ""])
def test_scalar_rejects(bad):
    with pytest.raises(QueryError):
        parse_scalar(bad)


@pytest.mark.parametrize("expr,expected", [
    ("foo", (False, "=", "foo")),
    ("~foo", (True, "=", "foo")),
    ("foo|boo", (False, "in", ["foo", "boo"])),
    ("~ foo|boo", (True, "in", ["foo", "boo"])),
    ("foo| |boo|", (False, "in", ["foo", "boo"])),
])
def test_value_operations(expr, expected):
    assert parse_value(expr) == expected


@pytest.mark.parametrize("bad", ["|", "~", "~ | "])
def test_value_rejects_empty(bad):
    with pytest.raises(QueryError):
        parse_value(bad)


def test_datetime_operations():
    d1, d2 = parse_datetime("2018-01-01"), parse_datetime("2018-02-01")
    assert d2 - d1 == 31 * 86400
    assert parse_datetime("2018-01-01 10:00") == d1 + 36000
    assert parse_datetime("2018-01-01T10:00:30") == d1 + 36030
    assert parse_datetime_op("2018-01-01..2018-02-01") == (False, "range", (d1, d2))
    assert parse_datetime_op(" 2018-01-01 .. 2018-02-01 ") == (False, "range", (d1, d2))
    assert parse_datetime_op("~2018-01-01..2018-02-01") == (True, "range", (d1, d2))
    assert parse_datetime_op(">=2018-01-01") == (False, ">=", d1)
    assert parse_datetime_op("~ <= 2018-02-01") == (True, "<=", d2)
    assert parse_datetime_op("2018-01-01") == (False, "=", d1)
    for bad in ("foo|bar", "~", "..", "..2018-01-01", "2018-01-01..", "asd..asd..asd", "2018-13-01"):
        with pytest.raises(QueryError):
            parse_datetime_op(bad)


def test_builder_sql_and_params():
    q = ExperimentQuery()
    clauses, params = q.where("metric.loss:<0.1, status:running|building, declarations.opt:~adam")
    assert clauses[0] == "json_extract(e.last_metric, ?) < ?" and params[:2] == ['$."loss"', 0.1]
    assert clauses[1] == "e.status IN (?, ?)" and params[2:4] == ["running", "building"]
    assert clauses[2] == "json_extract(e.declarations, ?) != ?" and params[4:] == ['$."opt"', "adam"]
    # negation flips comparison operators instead of wrapping them
    for expr, sql_op in (("~<1", ">="), ("~>1", "<="), ("~>=1", "<"), ("~<=1", ">")):
        c, _ = q.where(f"metric.loss:{expr}")
        assert c == [f"json_extract(e.last_metric, ?) {sql_op} ?"]
    c, _ = q.where("status:~running|failed")
    assert c == ["e.status NOT IN (?, ?)"]
    c, p = q.where("created_at:~2018-01-01..2018-02-01")
    assert c == ["NOT (e.created_at BETWEEN ? AND ?)"] and p == [parse_datetime("2018-01-01"),
                                                               parse_datetime("2018-02-01")]
    c, p = q.where("created_at:2018-01-01")  # a bare date means the whole day
    d = parse_datetime("2018-01-01")
    assert c == ["(e.created_at >= ? AND e.created_at < ?)"] and p == [d, d + 86400]
    c, p = q.where("tags:a|b")
    assert c[0].startswith("EXISTS (SELECT 1 FROM json_each(e.tags)") and p == ["a", "b"]
    c, _ = q.where("independent:false")
    assert c == ["NOT (e.group_id IS NULL)"]


def test_builder_proxies_and_errors():
    q = ExperimentQuery()
    assert q.where("metrics.loss:1")[0] == q.where("metric.loss:1")[0]  # metric proxies
    assert q.where("experiment_group:3") == q.where("group:3")
    for bad in ("bogus:1", "metric:1", "declarations:1", "metric.loss:abc"):
        with pytest.raises(QueryError):
            q.where(bad)


def test_sort_expressions():
    q = ExperimentQuery()
    # a missing or non-finite metric (stored as a string) sorts last either way
    assert q.order_by("-metric.loss").startswith("typeof(json_extract(e.last_metric, '$.\"loss\"')) NOT IN "
                                                 "('integer', 'real'), json_extract(e.last_metric, '$.\"loss\"') DESC")
    assert q.order_by("created_at").startswith("e.created_at IS NULL, e.created_at ASC")
    assert q.order_by("created_at, -id").endswith("e.id ASC")
    for bad in ("bogus", "tags", "metric", "metric.a'b", "independent"):
        with pytest.raises(QueryError):
            q.order_by(bad)


def test_group_and_job_queries():
    g, j = GroupQuery(), JobQuery()
    assert g.where("status:running")[0] and g.order_by("-created_at")
    assert j.where("status:~failed")[0] and j.order_by("created_at")
    with pytest.raises(QueryError):
        g.where("metric.loss:1")


def test_reference_operator_aliases_and_rejections():
    """query/parser.py:25-41 accepts ``=<`` / ``=>`` as ``<=`` / ``>=``; :104-109 rejects ``|`` and ``..`` in
    scalar conditions; datetime conditions reject ``|`` and ranges with more than two bounds."""
    from polyaxon_amd.store.query import ExperimentQuery, QueryError, parse_datetime_op, parse_scalar

    assert parse_scalar("=<0.5") == (False, "<=", 0.5)
    assert parse_scalar("=>3") == (False, ">=", 3)
    assert parse_scalar("~=<2") == (True, "<=", 2)
    assert parse_scalar("<-0.12") == (False, "<", -0.12)
    for bad in ("1|2", "1..2", "~0.1|0.2", "", "abc"):
        with pytest.raises(QueryError):
            parse_scalar(bad)
    assert parse_datetime_op("=>2018-01-01")[1] == ">="
    with pytest.raises(QueryError):
        parse_datetime_op("2018-01-01|2018-02-01")
    with pytest.raises(QueryError):
        parse_datetime_op("2018-01-01 .. 2018-02-01 .. 2018-03-01")
    q = ExperimentQuery()
    w, p = q.where("metric.loss:=<0.5, created_at:=>2018-01-01")
    assert len(w) == 2
    with pytest.raises(QueryError):
        q.where("metric.loss:0.1|0.2")
