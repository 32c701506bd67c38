"""REST API (FastAPI TestClient, real scheduler underneath) and the plx CLI in local mode."""
import json
import os
import sys

import pytest

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow

TOKEN = "t0ken"


@pytest.fixture
def api(tmp_path):
    from fastapi.testclient import TestClient

    from polyaxon_amd.api.server import create_app

    flow = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0), Device(1)])).start()
    client = TestClient(create_app(flow, admin_token=TOKEN))
    client.headers["Authorization"] = f"token {TOKEN}"
    yield client, flow
    flow.shutdown()


def test_auth_required(api):
    client, _ = api
    r = client.get("/api/v1/projects", headers={"Authorization": "token wrong"})
    assert r.status_code == 401
    assert client.get("/_health").json() == {"status": "ok"}


def test_experiment_lifecycle_over_rest(api):
    client, flow = api
    assert client.post("/api/v1/projects", json={"name": "mnist"}).status_code == 201
    content = {"version": 1, "kind": "experiment", "declarations": {"lr": 0.1},
               "run": {"cmd": "echo lr={{ lr }}"}}
    r = client.post("/api/v1/root/mnist/experiments", json={"content": content})
    assert r.status_code == 201, r.text
    xid = r.json()["id"]
    assert flow.wait("experiment", xid, timeout=30) == "succeeded"
    x = client.get(f"/api/v1/root/mnist/experiments/{xid}").json()
    assert x["status"] == "succeeded" and x["declarations"] == {"lr": 0.1}
    assert "master.0 -- lr=0.1" in client.get(f"/api/v1/root/mnist/experiments/{xid}/logs").text
    sts = client.get(f"/api/v1/root/mnist/experiments/{xid}/statuses").json()
    assert [s["status"] for s in sts["results"]][-1] == "succeeded"
    # metrics: single + batch, then query/sort through the list endpoint
    assert client.post(f"/api/v1/root/mnist/experiments/{xid}/metrics", json={"values": {"loss": 0.5}}).status_code == 201
    client.post(f"/api/v1/root/mnist/experiments/{xid}/metrics",
                json=[{"values": {"loss": 0.3}, "step": 2}, {"values": {"acc": 0.9}, "step": 2}])
    assert client.get(f"/api/v1/root/mnist/experiments/{xid}").json()["last_metric"] == {"loss": 0.3, "acc": 0.9}
    lst = client.get("/api/v1/root/mnist/experiments", params={"query": "metric.loss:<0.4", "sort": "-created_at"})
    assert [e["id"] for e in lst.json()["results"]] == [xid]
    assert client.get("/api/v1/root/mnist/experiments", params={"query": "bogus:1"}).status_code == 400
    # clone
    r = client.post(f"/api/v1/root/mnist/experiments/{xid}/restart", json={"declarations": {"lr": 0.2}})
    assert r.status_code == 201 and r.json()["original_experiment_id"] == xid
    assert flow.wait("experiment", r.json()["id"], timeout=30) == "succeeded"
    # update / bookmark / outputs / jobs
    assert client.patch(f"/api/v1/root/mnist/experiments/{xid}", json={"tags": ["best"]}).json()["tags"] == ["best"]
    assert client.post(f"/api/v1/root/mnist/experiments/{xid}/bookmark").json()["bookmarked"]
    assert client.get(f"/api/v1/root/mnist/experiments/{xid}/outputs").status_code == 200
    assert client.get(f"/api/v1/root/mnist/experiments/{xid}/jobs").json()["count"] == 1
    assert client.get(f"/api/v1/root/mnist/experiments/999").status_code == 404
    acts = client.get("/api/v1/activitylogs").json()
    assert any(a["event_type"] == "experiment.created" for a in acts["results"])


def test_ephemeral_token_exchange(api):
    client, flow = api
    r = client.post("/api/v1/root/p/experiments", json={"content": {"version": 1, "kind": "experiment",
                                                                     "run": {"cmd": "true"}}})
    xid = r.json()["id"]
    eph = client.post(f"/api/v1/root/p/experiments/{xid}/ephemeraltoken").json()["token"]
    r2 = client.post(f"/api/v1/root/p/experiments/{xid}/token", headers={"Authorization": f"token {eph}"})
    assert r2.status_code == 200 and r2.json()["token"] == TOKEN
    r3 = client.post(f"/api/v1/root/p/experiments/{xid + 1}/token", headers={"Authorization": f"token {eph}"})
    assert r3.status_code in (403, 404)


def test_group_over_rest_and_status(api):
    client, flow = api
    content = {"version": 1, "kind": "group",
               "hptuning": {"concurrency": 2, "matrix": {"x": {"values": [1, 2, 3]}}},
               "run": {"cmd": "echo {{ x }}"}}
    r = client.post("/api/v1/root/g/groups", json={"content": content})
    assert r.status_code == 201
    gid = r.json()["id"]
    assert flow.wait("group", gid, timeout=30) == "succeeded"
    g = client.get(f"/api/v1/root/g/groups/{gid}").json()
    assert g["num_experiments"] == 3 and g["status_counts"] == {"succeeded": 3}
    assert client.get(f"/api/v1/root/g/groups/{gid}/experiments", params={"sort": "-id"}).json()["count"] == 3
    st = client.get("/_status").json()
    assert st["checks"]["store"]["status"] == "ok" and st["checks"]["scheduler"]["status"] == "ok"
    assert client.post("/api/v1/root/g/groups", json={"content": {"version": 1, "kind": "group"}}).status_code == 400


def test_sse_log_stream(api):
    client, flow = api
    r = client.post("/api/v1/root/s/experiments",
                    json={"content": {"version": 1, "kind": "experiment", "run": {"cmd": "echo a; echo b"}}})
    xid = r.json()["id"]
    flow.wait("experiment", xid, timeout=30)
    with client.stream("GET", f"/streams/v1/root/s/experiments/{xid}/logs") as s:
        body = "".join(s.iter_text())
    assert "data: master.0 -- a" in body and "event: done" in body


def test_cli_local_mode(tmp_path, monkeypatch):
    from click.testing import CliRunner

    from polyaxon_amd.cli.main import cli

    monkeypatch.setenv("PLX_ROOT", str(tmp_path / "root"))
    monkeypatch.setenv("PLX_CONFIG", str(tmp_path / "cfg.yaml"))
    monkeypatch.delenv("PLX_HOST", raising=False)
    f = tmp_path / "xp.yml"
    f.write_text("version: 1\nkind: experiment\ndeclarations: {lr: 0.3}\nrun: {cmd: 'echo lr={{ lr }}'}\n")
    runner = CliRunner()
    r = runner.invoke(cli, ["check", "-f", str(f)])
    assert r.exit_code == 0 and "valid experiment" in r.output
    r = runner.invoke(cli, ["-p", "demo", "run", "-f", str(f), "--gpus", "1"])
    assert r.exit_code == 0, r.output
    assert "succeeded" in r.output and "lr=0.3" in r.output
    r = runner.invoke(cli, ["-p", "demo", "--json", "project", "experiments"])
    assert json.loads(r.output)[0]["status"] == "succeeded"
    r = runner.invoke(cli, ["-p", "demo", "experiment", "-xp", "1", "logs"])
    assert "master.0 -- lr=0.3" in r.output
    r = runner.invoke(cli, ["-p", "demo", "experiment", "-xp", "1", "statuses"])
    assert "succeeded" in r.output


def test_repo_upload_and_code_reference(api, tmp_path):
    import io
    import tarfile

    client, flow = api
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tar:
        data = b"print('hello from uploaded code')\n"
        info = tarfile.TarInfo("train.py")
        info.size = len(data)
        tar.addfile(info, io.BytesIO(data))
    r = client.post("/api/v1/root/up/repo/upload", content=buf.getvalue())
    assert r.status_code == 200, r.text
    sha, path = r.json()["commit"], r.json()["path"]
    assert len(sha) == 40
    content = {"version": 1, "kind": "experiment", "run": {"cmd": f"{sys.executable} train.py"}}
    xid = client.post("/api/v1/root/up/experiments", json={"content": content, "cwd": path}).json()["id"]
    assert flow.wait("experiment", xid, timeout=30) == "succeeded"
    assert "hello from uploaded code" in client.get(f"/api/v1/root/up/experiments/{xid}/logs").text
    ref = client.get(f"/api/v1/root/up/experiments/{xid}/coderef").json()
    assert ref["commit_sha"] == sha and ref["is_dirty"] == 0
    assert client.get("/api/v1/root/up/repo/download").status_code == 200


def test_cli_upload_and_run_snapshot(tmp_path, monkeypatch):
    from click.testing import CliRunner

    from polyaxon_amd.cli.main import cli

    monkeypatch.setenv("PLX_ROOT", str(tmp_path / "root"))
    monkeypatch.setenv("PLX_CONFIG", str(tmp_path / "cfg.yaml"))
    monkeypatch.delenv("PLX_HOST", raising=False)
    code = tmp_path / "code"
    code.mkdir()
    (code / "train.py").write_text("print('snapshot v1')\n")
    (code / "big.bin").write_text("x")
    (code / ".polyaxonignore").write_text("*.bin\n")
    (code / "xp.yml").write_text(f"version: 1\nkind: experiment\nrun: {{cmd: '{sys.executable} train.py'}}\n")
    monkeypatch.chdir(code)
    runner = CliRunner()
    r = runner.invoke(cli, ["-p", "up", "upload"])
    assert r.exit_code == 0 and "uploaded" in r.output, r.output
    repo = tmp_path / "root" / "repos" / "root" / "up"
    assert (repo / "train.py").exists() and not (repo / "big.bin").exists()
    (code / "train.py").write_text("print('snapshot v2')\n")
    r = runner.invoke(cli, ["-p", "up", "run", "-u", "-f", "xp.yml", "--gpus", "0"])
    assert r.exit_code == 0 and "snapshot v2" in r.output, r.output


def test_dashboard_page_and_query_token(api):
    client, flow = api
    r = client.get("/", headers={"Authorization": ""})
    assert r.status_code == 200 and "polyaxon-mi355x" in r.text and "EventSource" in r.text
    # streams accept ?token= (EventSource cannot send headers)
    xid = client.post("/api/v1/root/d/experiments",
                      json={"content": {"version": 1, "kind": "experiment", "run": {"cmd": "echo hi"}}}).json()["id"]
    flow.wait("experiment", xid, timeout=30)
    del client.headers["Authorization"]
    assert client.get("/api/v1/projects").status_code == 401
    with client.stream("GET", f"/streams/v1/root/d/experiments/{xid}/logs", params={"token": TOKEN}) as s:
        body = "".join(s.iter_text())
    assert "hi" in body


def test_users_and_project_permissions(api):
    client, flow = api
    assert client.post("/api/v1/projects", json={"name": "priv", "is_public": False}).status_code == 201
    assert client.post("/api/v1/projects", json={"name": "pub"}).status_code == 201
    r = client.post("/api/v1/users", json={"username": "alice"})
    assert r.status_code == 201
    alice = {"Authorization": f"token {r.json()['token']}"}
    assert client.get("/api/v1/users", headers=alice).json()["username"] == "alice"
    # alice: read public, not private; no writes into root's projects; not a superuser
    assert client.get("/api/v1/root/pub/experiments", headers=alice).status_code == 200
    assert client.get("/api/v1/root/priv/experiments", headers=alice).status_code == 403
    content = {"version": 1, "kind": "experiment", "run": {"cmd": "true"}}
    assert client.post("/api/v1/root/pub/experiments", json={"content": content}, headers=alice).status_code == 403
    assert client.post("/api/v1/users", json={"username": "eve"}, headers=alice).status_code == 403
    # her own project is fully hers
    assert client.post("/api/v1/projects", json={"name": "mine"}, headers=alice).status_code == 201
    r = client.post("/api/v1/alice/mine/experiments", json={"content": content}, headers=alice)
    assert r.status_code == 201
    assert flow.wait("experiment", r.json()["id"], timeout=30) == "succeeded"
    assert [u["username"] for u in client.get("/api/v1/users/list").json()["results"]] == ["root", "alice"]


def test_admin_table_browser(api):
    """Superuser admin (reference db/admin/*.py): tables with counts, paged rows with secrets redacted,
    edit and delete a row; non-superusers are refused."""
    client = api[0] if isinstance(api, tuple) else api
    r = client.post("/api/v1/projects", json={"name": "adm"})
    assert r.status_code == 201
    tables = {t["table"]: t for t in client.get("/api/v1/admin/tables").json()["results"]}
    assert {"projects", "experiments", "users", "kv"} <= set(tables)
    rows = client.get("/api/v1/admin/tables/users").json()
    assert rows["count"] >= 1 and all(u.get("token") in (None, "***") for u in rows["results"])
    proj = [p for p in client.get("/api/v1/admin/tables/projects").json()["results"] if p["name"] == "adm"][0]
    r = client.patch(f"/api/v1/admin/tables/projects/{proj['id']}", json={"description": "edited by admin"})
    assert r.status_code == 200 and r.json()["description"] == "edited by admin"
    assert client.patch(f"/api/v1/admin/tables/projects/{proj['id']}", json={"nope": 1}).status_code == 400
    assert client.get("/api/v1/admin/tables/not_a_table").status_code == 404
    assert client.delete(f"/api/v1/admin/tables/projects/{proj['id']}").status_code == 204
    assert client.delete(f"/api/v1/admin/tables/projects/{proj['id']}").status_code == 404
    tok = client.post("/api/v1/users", json={"username": "bob"}).json()["token"]
    assert client.get("/api/v1/admin/tables", headers={"Authorization": f"token {tok}"}).status_code == 403


def test_project_listing_privacy_and_ephemeral_scope(api):
    """Advisor round 1: private projects are not listed to other users, ephemeral per-trial tokens cannot use
    non-experiment routes, and the admin browser redacts password hashes."""
    client, flow = api
    assert client.post("/api/v1/projects", json={"name": "secret", "is_public": False}).status_code == 201
    assert client.post("/api/v1/projects", json={"name": "open"}).status_code == 201
    tok = client.post("/api/v1/users", json={"username": "carol"}).json()["token"]
    carol = {"Authorization": f"token {tok}"}
    names = [p["name"] for p in client.get("/api/v1/projects", headers=carol).json()["results"]]
    assert "open" in names and "secret" not in names
    assert {"open", "secret"} <= {p["name"] for p in client.get("/api/v1/projects").json()["results"]}
    # an ephemeral token for one experiment
    content = {"version": 1, "kind": "experiment", "run": {"cmd": "true"}}
    xid = client.post("/api/v1/root/open/experiments", json={"content": content}).json()["id"]
    eph = client.post(f"/api/v1/root/open/experiments/{xid}/ephemeraltoken").json()["token"]
    e = {"Authorization": f"token {eph}"}
    assert client.get(f"/api/v1/root/open/experiments/{xid}", headers=e).status_code == 200
    assert client.get("/api/v1/projects", headers=e).status_code == 403
    assert client.get("/api/v1/root/open/experiments", headers=e).status_code == 403
    # password hashes never leave through the admin browser

    flow.store.execute("INSERT OR REPLACE INTO user_credentials (username, password_hash) VALUES ('carol', 'pbkdf2$x')")
    rows = client.get("/api/v1/admin/tables/user_credentials").json()["results"]
    assert rows and all(r["password_hash"] == "***" for r in rows)


def test_dashboard_views_and_their_api_contract(api):
    """The dashboard's hash views (project tabs, experiment / group / compare / job / pipeline detail) and the
    fields each reads: one column per declaration and metric, status history, metric points, group hptuning and
    iterations, replica rows, the pipelines list."""
    client, flow = api
    page = client.get("/ui").text
    for marker in ("#/p/", "/compare/", "Status history", "Hyperparameter vs metric", "Learning curves",
                   "Side by side", "Iterations", "Replicas", "/pipelines", "esc("):
        assert marker in page, marker
    import shutil
    import subprocess

    node = shutil.which("node")
    if node:  # the page's script must at least parse
        js = page.split("<script>", 1)[1].split("</script>", 1)[0]
        r = subprocess.run([node, "--check", "-"], input=js, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
    content = {"version": 1, "kind": "group",
               "hptuning": {"concurrency": 2, "matrix": {"lr": {"values": [0.1, 0.2, 0.3]}},
                            "grid_search": {"n_experiments": 3}},
               "run": {"cmd": "echo {{ lr }}"}}
    gid = client.post("/api/v1/root/dash/groups", json={"content": content}).json()["id"]
    assert flow.wait("group", gid, timeout=30) == "succeeded"
    xs = client.get(f"/api/v1/root/dash/groups/{gid}/experiments").json()["results"]
    assert len(xs) == 3 and all(set(x["declarations"]) == {"lr"} for x in xs)
    for k, x in enumerate(xs):
        client.post(f"/api/v1/root/dash/experiments/{x['id']}/metrics",
                    json=[{"values": {"loss": 1.0 / (k + 1 + s)}, "step": s} for s in range(3)])
    x0 = xs[0]["id"]
    x = client.get(f"/api/v1/root/dash/experiments/{x0}").json()
    assert {"status", "declarations", "last_metric", "started_at", "finished_at", "group_id"} <= set(x)
    pts = client.get(f"/api/v1/root/dash/experiments/{x0}/metrics", params={"limit": 20000}).json()["results"]
    assert [p["step"] for p in pts] == [0, 1, 2] and all("loss" in p["values"] for p in pts)
    sts = client.get(f"/api/v1/root/dash/experiments/{x0}/statuses").json()["results"]
    assert {"status", "message", "created_at"} <= set(sts[0]) and sts[-1]["status"] == "succeeded"
    jobs = client.get(f"/api/v1/root/dash/experiments/{x0}/jobs").json()["results"]
    assert jobs and {"role", "idx", "status"} <= set(jobs[0])
    g = client.get(f"/api/v1/root/dash/groups/{gid}").json()
    assert g["search_algorithm"] and g["num_experiments"] == 3 and "hptuning" in g
    assert client.get(f"/api/v1/root/dash/groups/{gid}/statuses").json()["results"][-1]["status"] == "succeeded"
    assert "results" in client.get(f"/api/v1/root/dash/groups/{gid}/iterations").json()
    for tab in ("experiments", "groups", "jobs", "builds", "pipelines"):
        r = client.get(f"/api/v1/root/dash/{tab}")
        assert r.status_code == 200 and "results" in r.json(), tab
    pid = client.post("/api/v1/root/dash/pipelines", json={"content": {
        "version": 1, "kind": "pipeline", "ops": [{"name": "a", "template": {"version": 1, "kind": "job",
                                                                            "run": {"cmd": "true"}}}]}}).json()["id"]
    import time as _t
    end = _t.time() + 30
    while _t.time() < end:
        pl = client.get("/api/v1/root/dash/pipelines").json()["results"]
        if pl and pl[0]["last_run_status"] in ("finished", "succeeded"):
            break
        _t.sleep(0.1)
    assert pl[0]["id"] == pid and pl[0]["num_runs"] == 1 and pl[0]["last_run_status"] in ("finished", "succeeded")
    d = client.get(f"/api/v1/root/dash/pipelines/{pid}").json()
    run = client.get(f"/api/v1/root/dash/pipelines/{pid}/runs/{d['runs'][0]['id']}").json()
    assert run["operations"][0]["name"] == "a"
    assert "results" in client.get("/api/v1/activitylogs", params={"limit": 30}).json()


def test_dashboard_tables_filters_charts_contract(api):
    """The reference client's tables / filters / autocomplete / chart builder (client/src/components/{tables,filters,
    autocomplete,charts,metrics}): the page carries the query autocomplete, saved searches, server-side sort and
    pagination, the column chooser, bookmarks, the chart builder with saved chart views and parallel coordinates,
    and the API answers every call those make with the fields they read."""
    client, flow = api
    page = client.get("/ui").text
    for marker in ("function autocomplete(", "QFIELDS", "savesearch", "pager", "colpick", "function parallel(",
                   "chartviews", "smoothing", "log y", "#/bookmarks", "unbookmark", "offset="):
        assert marker in page, marker
    content = {"version": 1, "kind": "group",
               "hptuning": {"concurrency": 3, "matrix": {"lr": {"values": [0.1, 0.2, 0.3]}},
                            "grid_search": {"n_experiments": 3}}, "run": {"cmd": "echo {{ lr }}"}}
    gid = client.post("/api/v1/root/tf/groups", json={"content": content}).json()["id"]
    assert flow.wait("group", gid, timeout=30) == "succeeded"
    xs = client.get("/api/v1/root/tf/experiments", params={"sort": "declarations.lr"}).json()["results"]
    for k, x in enumerate(xs):
        client.post(f"/api/v1/root/tf/experiments/{x['id']}/metrics", json=[{"values": {"loss": 3.0 - k}, "step": 1}])
    # server-side sort on a metric + pagination (what the sort select and pager send)
    r = client.get("/api/v1/root/tf/experiments", params={"sort": "-metric.loss", "limit": 2, "offset": 0}).json()
    assert r["count"] == 3 and len(r["results"]) == 2
    assert [x["last_metric"]["loss"] for x in r["results"]] == [3.0, 2.0]
    r2 = client.get("/api/v1/root/tf/experiments", params={"sort": "-metric.loss", "limit": 2, "offset": 2}).json()
    assert [x["last_metric"]["loss"] for x in r2["results"]] == [1.0]
    # the autocomplete's field forms parse
    for q in ("status:succeeded", "metric.loss:<2.5", "declarations.lr:0.2|0.3", "status:~failed, metric.loss:>=1", "created_at:2020-01-01..2100-01-01"):
        assert client.get("/api/v1/root/tf/experiments", params={"query": q}).status_code == 200, q
    # saved searches
    assert client.post("/api/v1/searches/root/tf/experiments",
                       json={"name": "good", "query": "metric.loss:<2.5", "sort": "metric.loss"}).status_code == 201
    ss = client.get("/api/v1/searches/root/tf/experiments").json()["results"]
    assert ss[0]["name"] == "good" and ss[0]["query"]["query"] == "metric.loss:<2.5"
    # bookmarks, enriched with what the bookmarks view links to
    x0 = xs[0]["id"]
    assert client.post(f"/api/v1/root/tf/experiments/{x0}/bookmark").json()["bookmarked"]
    me = client.get("/api/v1/users").json()["username"]
    bm = client.get(f"/api/v1/bookmarks/{me}/experiments").json()["results"]
    assert bm and bm[0]["object_id"] == x0 and bm[0]["experiment"]["project"] == "tf"
    assert client.delete(f"/api/v1/root/tf/experiments/{x0}/unbookmark").json()["bookmarked"] is False
    assert client.get(f"/api/v1/bookmarks/{me}/experiments").json()["results"] == []
    # chart views (the chart builder's saved state)
    view = {"name": "v", "charts": [{"metrics": ["loss"], "x": "time", "smoothing": 0.6, "logy": True}]}
    assert client.post(f"/api/v1/root/tf/experiments/{x0}/chartviews", json=view).status_code == 201
    cv = client.get(f"/api/v1/root/tf/experiments/{x0}/chartviews").json()["results"]
    assert cv[0]["charts"][0]["smoothing"] == 0.6 and cv[0]["charts"][0]["logy"] is True
    pts = client.get(f"/api/v1/root/tf/experiments/{x0}/metrics", params={"limit": 20000}).json()["results"]
    assert "created_at" in pts[0]  # the wall-time x axis
