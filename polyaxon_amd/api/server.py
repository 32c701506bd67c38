"""REST API (+ SSE streams) over the tracking store and the polyflow scheduler.

Surface: SURVEY.md §8.3 — reference polyaxon/api/patterns.py:14-68 (``/api/v1/``), experiments
(api/experiments/urls.py:15-81), groups (api/experiment_groups/urls.py:9-32), jobs, builds, plugins
(notebook/tensorboard start/stop), cluster/nodes, versions, searches, bookmarks, activity logs,
``/_health`` and ``/_status``.  Auth: ``Authorization: token <token>`` (reference TokenAuthentication),
``X-POLYAXON-INTERNAL`` + internal token for in-trial services, and per-experiment ephemeral tokens that
are exchanged at ``/experiments/<id>/token`` (api/experiments/views.py:615-643).

Live logs and resources (reference Sanic websockets, streams/api.py:647-677) are served as
Server-Sent Events under ``/streams/v1/...`` (the WebSocket libraries are not part of this image; SSE is
plain HTTP and works with ``curl -N`` / EventSource).
"""
from __future__ import annotations

import asyncio
import json
import os
import time
from typing import Any, Dict, List, Optional

from fastapi import Depends, FastAPI, Header, HTTPException, Query, Request
from fastapi.responses import (FileResponse, JSONResponse, PlainTextResponse, RedirectResponse, Response,
                               StreamingResponse)

from polyaxon_amd import __version__
from polyaxon_amd.auth import Accounts, AuthError, validate_name
from polyaxon_amd.conf import Settings
from polyaxon_amd.spec import PolyaxonfileError, specification_for
from polyaxon_amd.store import QueryError

INTERNAL_HEADER = "x-polyaxon-internal"


def create_app(flow, admin_token: Optional[str] = None, internal_token: Optional[str] = None,
               require_auth: bool = True, settings: Optional[Settings] = None, sso_transport=None) -> FastAPI:
    store = flow.store
    settings = settings or Settings.load(env={})
    accounts = Accounts(store, settings, transport=sso_transport)
    _metric_buckets: Dict[int, Any] = {}  # xid -> (tokens, last refill) for api.throttle_metrics_per_s
    app = FastAPI(title="polyaxon-mi355x", version=__version__)
    if admin_token and not store.user_for_token(admin_token):
        if store.get_user("root"):
            store.execute("UPDATE users SET token = ? WHERE username = 'root'", (admin_token,))
        else:
            store.create_user("root", is_superuser=True, token=admin_token)
    internal = internal_token or os.environ.get("POLYAXON_SECRET_INTERNAL_TOKEN")

    # ------------------------------------------------------------------ auth
    def identify(authorization: Optional[str], x_polyaxon_internal: Optional[str], token: Optional[str]):
        if not require_auth:
            return {"username": "root", "is_superuser": 1}
        if authorization is None and token:  # EventSource (dashboard streams) cannot set headers
            authorization = f"token {token}"
        if x_polyaxon_internal and internal and authorization == f"token {internal}":
            return {"username": "internal", "is_superuser": 1}
        if authorization and authorization.lower().startswith("token "):
            tok = authorization.split(" ", 1)[1].strip()
            user = store.user_for_token(tok)
            if user:
                if not accounts.token_valid(user):
                    raise HTTPException(401, "Token expired or account inactive.")
                return user
            eph = store.kv_get(f"ephemeral:{tok}")
            if eph:
                return {"username": eph["user"], "is_superuser": 0, "scope": eph}
        raise HTTPException(401, "Authentication credentials were not provided or are invalid.")

    def auth(request: Request, authorization: Optional[str] = Header(None),
             x_polyaxon_internal: Optional[str] = Header(None),
             token: Optional[str] = Query(None)) -> Dict[str, Any]:
        """Authenticate, then authorise project-scoped routes (reference libs/permissions/projects.py):
        superusers and the owner may do anything; other users may only read public projects; an ephemeral
        token may only touch its own experiment."""
        user = identify(authorization, x_polyaxon_internal, token)
        pp = request.path_params
        scope = user.get("scope")
        if scope is not None and ("xid" not in pp or "username" not in pp or "project" not in pp):
            # an ephemeral (per-trial) token only reaches its own experiment's routes
            raise HTTPException(403, "ephemeral token is scoped to one experiment")
        if user.get("is_superuser") or "username" not in pp or "project" not in pp:
            return user
        if scope is not None:
            xid = pp.get("xid")
            if xid is None or int(xid) != int(scope.get("experiment", -1)):
                raise HTTPException(403, "ephemeral token is scoped to another experiment")
            return user
        owner = pp["username"]
        if user.get("username") == owner:
            return user
        proj = store.get_project(pp["project"], owner)
        if request.method in ("GET", "HEAD") and (proj is None or proj.get("is_public")):
            return user
        raise HTTPException(403, "You do not have permission to perform this action.")

    def project_or_404(user: str, project: str) -> Dict[str, Any]:
        p = store.get_project(project, user)
        if p is None:
            raise HTTPException(404, f"project {user}/{project} not found")
        return p

    def xp_or_404(user: str, project: str, xid: int) -> Dict[str, Any]:
        p = project_or_404(user, project)
        x = store.get_experiment(xid)
        if x is None or x["project_id"] != p["id"]:
            raise HTTPException(404, f"experiment {xid} not found")
        return x

    def group_or_404(user: str, project: str, gid: int) -> Dict[str, Any]:
        p = project_or_404(user, project)
        g = store.get_group(gid)
        if g is None or g["project_id"] != p["id"]:
            raise HTTPException(404, f"group {gid} not found")
        return g

    def job_or_404(user: str, project: str, jid: int, kind: Optional[str] = None) -> Dict[str, Any]:
        p = project_or_404(user, project)
        j = store.get_job(jid)
        if j is None or j["project_id"] != p["id"] or (kind and j["kind"] != kind):
            raise HTTPException(404, f"{kind or 'job'} {jid} not found")
        return j

    def page(rows: List[Dict], request: Request) -> Dict[str, Any]:
        limit = int(request.query_params.get("limit", 0) or 0)
        offset = int(request.query_params.get("offset", 0) or 0)
        total = len(rows)
        if limit:
            rows = rows[offset: offset + limit]
        return {"count": total, "results": rows}

    # ------------------------------------------------------------------ dashboard (static page over this API)
    static = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static", "index.html")

    @app.get("/", include_in_schema=False)
    @app.get("/ui", include_in_schema=False)
    def dashboard():
        return FileResponse(static, media_type="text/html")

    # ------------------------------------------------------------------ health / status / versions
    @app.get("/_health")
    def health():
        store.execute("SELECT 1").fetchone()
        return {"status": "ok"}

    @app.get("/_status")
    def status():
        from polyaxon_amd.obs.checks import run_checks

        return run_checks(flow)

    @app.get("/api/v1/versions/platform")
    def versions():
        return {"platform_version": __version__, "api_version": "v1", "arch": "gfx950"}

    @app.get("/api/v1/versions/cli")
    def versions_cli():
        return {"latest_version": __version__, "min_version": "0.2.0"}

    # ------------------------------------------------------------------ users / projects
    @app.get("/api/v1/users")
    def me(user=Depends(auth)):
        return {k: v for k, v in user.items() if k != "token"}

    # registered before the /api/v1/{username}/{project}/... routes: 'bookmarks/<user>/experiments' would match them
    @app.get("/api/v1/bookmarks/{username}/experiments")
    def user_bookmarks(username: str, user=Depends(auth)):
        out = []
        for b in store.bookmarks(username, "experiment"):
            x = store.get_experiment(b["object_id"])
            if x is not None:  # enough of the experiment to list and link it (the dashboard's bookmarks view)
                proj = store.get("projects", x["project_id"]) or {}
                b = dict(b, experiment={"id": x["id"], "status": x["status"], "project": proj.get("name"),
                                        "user": proj.get("user") or x.get("user"), "declarations": x["declarations"],
                                        "last_metric": x["last_metric"], "group_id": x["group_id"]})
            out.append(b)
        return {"results": out}

    def superuser(user=Depends(auth)):
        if not user.get("is_superuser"):
            raise HTTPException(403, "superuser only")
        return user

    @app.post("/api/v1/users", status_code=201)
    async def create_user(request: Request, user=Depends(superuser)):
        """Create a user and return its API token (reference `createuser` management command)."""
        body = await request.json()
        if not body.get("username") or store.get_user(body["username"]):
            raise HTTPException(400, "missing or existing username")
        try:
            validate_name(body["username"], settings.get("blacklist.extra"))
        except ValueError as e:
            raise HTTPException(400, str(e))
        u = store.create_user(body["username"], body.get("email", ""), bool(body.get("is_superuser")))
        if body.get("password"):
            _auth_call(accounts.set_password, u["username"], body["password"])
        flow.auditor.record("user.registered", "user", u["id"], user.get("username"))
        return u

    def _auth_call(fn, *args):
        try:
            return fn(*args)
        except AuthError as e:
            raise HTTPException(e.status, str(e))

    @app.post("/api/v1/users/token")
    async def login(request: Request):
        """Exchange username + password (local or LDAP) for an API token (reference users/token + login)."""
        body = await request.json()
        u = _auth_call(accounts.login, body.get("username", ""), body.get("password", ""))
        flow.auditor.record("user.logged_in", "user", u["id"], u["username"])
        return {"token": u["token"], "username": u["username"]}

    @app.post("/api/v1/users/logout")
    def logout(user=Depends(auth)):
        if user.get("scope") is None and user.get("username") != "internal":
            accounts.logout(user["username"])
            flow.auditor.record("user.logged_out", "user", user.get("id"), user["username"])
        return {"ok": True}

    @app.post("/api/v1/users/password")
    async def change_password(request: Request, user=Depends(auth)):
        body = await request.json()
        _auth_call(accounts.change_password, user["username"], body.get("old_password"), body.get("new_password"))
        flow.auditor.record("user.password_changed", "user", user.get("id"), user["username"])
        return {"ok": True}

    @app.post("/api/v1/users/register", status_code=201)
    async def register(request: Request):
        """Self-registration (reference SimpleRegistrationView): ``auth.registration`` = ``open`` returns a
        token at once; ``superuser_validation`` parks the account until ``/users/<name>/activate``."""
        body = await request.json()
        out = _auth_call(accounts.register, body.get("username", ""), body.get("email", ""),
                         body.get("password", ""))
        flow.auditor.record("user.registered", "user", None, body.get("username"))
        return out

    @app.get("/api/v1/users/pending")
    def pending_users(user=Depends(superuser)):
        return {"results": accounts.pending()}

    @app.post("/api/v1/users/{username}/activate")
    def activate_user(username: str, user=Depends(superuser)):
        _auth_call(accounts.activate, username)
        flow.auditor.record("user.activated", "user", None, user.get("username"))
        return {"ok": True}

    @app.post("/api/v1/users/{username}/deactivate")
    def deactivate_user(username: str, user=Depends(superuser)):
        _auth_call(accounts.deactivate, username)
        flow.auditor.record("user.deactivated", "user", None, user.get("username"))
        return {"ok": True}

    @app.post("/api/v1/users/{username}/password")
    async def set_password(username: str, request: Request, user=Depends(superuser)):
        body = await request.json()
        _auth_call(accounts.set_password, username, body.get("password", ""))
        return {"ok": True}

    @app.get("/api/v1/sso/providers")
    def sso_providers():
        return {"providers": accounts.sso_providers(), "ldap": bool(settings.get("auth.ldap.enabled"))}

    def _redirect_uri(request: Request, provider: str) -> str:
        return str(request.url_for("sso_complete", provider=provider))

    @app.get("/oauth/{provider}/login")
    def sso_login(provider: str, request: Request):
        url = _auth_call(accounts.sso_login_url, provider, _redirect_uri(request, provider))
        return RedirectResponse(url, status_code=302)

    @app.get("/oauth/{provider}/complete", name="sso_complete")
    def sso_complete(provider: str, request: Request, code: str = "", state: str = ""):
        out = _auth_call(accounts.sso_complete, provider, code, state, _redirect_uri(request, provider))
        flow.auditor.record("user.sso_logged_in", "user", None, out["username"])
        return out

    @app.get("/api/v1/users/list")
    def list_users(user=Depends(superuser)):
        rows = store.execute("SELECT id, username, email, is_superuser, created_at FROM users ORDER BY id").fetchall()
        return {"results": [dict(r) for r in rows]}

    # ------------------------------------------------------------------ admin (reference db/admin/*.py)
    # The reference registers every model with the Django admin; here a superuser gets a generic table
    # browser over the store: list tables with counts, page through rows, edit or delete a row.  Secrets
    # (API tokens, kv values holding ephemeral tokens) are never returned.
    _SECRET_COLS = {"token", "password_hash", "salt", "secret", "client_secret", "activation_key"}

    def _admin_tables() -> List[str]:
        rows = store.execute("SELECT name FROM sqlite_master WHERE type='table' AND name NOT LIKE 'sqlite_%' "
                             "ORDER BY name").fetchall()
        return [r[0] for r in rows]

    def _admin_table(name: str) -> List[str]:
        if name not in _admin_tables():
            raise HTTPException(404, f"table {name} not found")
        return [r[1] for r in store.execute(f"PRAGMA table_info({name})").fetchall()]

    def _redact(table: str, row: Dict[str, Any]) -> Dict[str, Any]:
        out = {k: ("***" if k in _SECRET_COLS else v) for k, v in row.items()}
        if table == "kv" and "v" in out:
            out["v"] = "***"
        return out

    @app.get("/api/v1/admin/tables")
    def admin_tables(user=Depends(superuser)):
        out = []
        for t in _admin_tables():
            n = store.execute(f"SELECT COUNT(*) FROM {t}").fetchone()[0]
            out.append({"table": t, "rows": n, "columns": _admin_table(t)})
        return {"results": out}

    @app.get("/api/v1/admin/tables/{table}")
    def admin_rows(table: str, request: Request, user=Depends(superuser)):
        cols = _admin_table(table)
        limit = min(int(request.query_params.get("limit", 50) or 50), 1000)
        offset = int(request.query_params.get("offset", 0) or 0)
        order = "id DESC" if "id" in cols else "rowid DESC"
        rows = store.execute(f"SELECT * FROM {table} ORDER BY {order} LIMIT ? OFFSET ?", (limit, offset)).fetchall()
        total = store.execute(f"SELECT COUNT(*) FROM {table}").fetchone()[0]
        return {"count": total, "columns": cols, "results": [_redact(table, dict(r)) for r in rows]}

    @app.patch("/api/v1/admin/tables/{table}/{rid}")
    async def admin_update(table: str, rid: int, request: Request, user=Depends(superuser)):
        cols = _admin_table(table)
        body = await request.json()
        bad = [k for k in body if k not in cols or k in ("id",) or k in _SECRET_COLS]
        if bad or not body or "id" not in cols:
            raise HTTPException(400, f"columns not editable: {bad or 'none given'}")
        sets = ", ".join(f"{k} = ?" for k in body)
        vals = [json.dumps(v) if isinstance(v, (dict, list)) else v for v in body.values()]
        cur = store.execute(f"UPDATE {table} SET {sets} WHERE id = ?", (*vals, rid))
        if cur.rowcount == 0:
            raise HTTPException(404, f"{table} row {rid} not found")
        flow.auditor.record("admin.updated", table, rid, user.get("username"))
        row = store.execute(f"SELECT * FROM {table} WHERE id = ?", (rid,)).fetchone()
        return _redact(table, dict(row))

    @app.delete("/api/v1/admin/tables/{table}/{rid}", status_code=204)
    def admin_delete(table: str, rid: int, user=Depends(superuser)):
        cols = _admin_table(table)
        if "id" not in cols:
            raise HTTPException(400, "table has no id column")
        if table == "users" and store.execute("SELECT username FROM users WHERE id = ?", (rid,)).fetchone() is not None \
                and store.execute("SELECT username FROM users WHERE id = ?", (rid,)).fetchone()[0] == user.get("username"):
            raise HTTPException(400, "cannot delete yourself")
        cur = store.execute(f"DELETE FROM {table} WHERE id = ?", (rid,))
        if cur.rowcount == 0:
            raise HTTPException(404, f"{table} row {rid} not found")
        flow.auditor.record("admin.deleted", table, rid, user.get("username"))
        return Response(status_code=204)

    @app.get("/api/v1/projects")
    def list_projects(request: Request, user=Depends(auth)):
        """All projects for superusers; otherwise the caller's own projects plus public ones."""
        rows = store.list_projects()
        if not user.get("is_superuser"):
            rows = [p for p in rows if p["user"] == user.get("username") or p.get("is_public")]
        return page(rows, request)

    @app.post("/api/v1/projects", status_code=201)
    async def create_project(request: Request, user=Depends(auth)):
        body = await request.json()
        try:
            validate_name(body.get("name", ""), settings.get("blacklist.extra"))
            p = store.create_project(body["name"], user.get("username", "root"), body.get("description", ""),
                                     body.get("is_public", True), body.get("tags"))
        except Exception as e:
            raise HTTPException(400, str(e))
        flow.auditor.record("project.created", "project", p["id"], p["user"])
        return p

    @app.get("/api/v1/{username}/{project}")
    def get_project(username: str, project: str, user=Depends(auth)):
        return project_or_404(username, project)

    @app.patch("/api/v1/{username}/{project}")
    async def update_project(username: str, project: str, request: Request, user=Depends(auth)):
        p = project_or_404(username, project)
        body = await request.json()
        store.update_project(p["id"], **{k: v for k, v in body.items() if k in ("description", "is_public", "tags")})
        return store.get("projects", p["id"])

    @app.delete("/api/v1/{username}/{project}", status_code=204)
    def delete_project(username: str, project: str, user=Depends(auth)):
        p = project_or_404(username, project)
        store.delete_project(p["id"])
        flow.auditor.record("project.deleted", "project", p["id"])
        return PlainTextResponse("", status_code=204)

    # ------------------------------------------------------------------ submission (run -f polyaxonfile)
    async def _submit(username: str, project: str, request: Request, expect: Optional[str]):
        body = await request.json()
        content = body.get("content", body.get("config", body))
        try:
            spec = specification_for(content)
        except PolyaxonfileError as e:
            raise HTTPException(400, f"invalid polyaxonfile: {e}")
        if expect and spec.kind != expect:
            raise HTTPException(400, f"expected kind `{expect}`, got `{spec.kind}`")
        store.get_or_create_project(project, username)
        res = flow.submit(spec, project=project, user=username, cwd=body.get("cwd") or os.getcwd(),
                          name=body.get("name"), description=body.get("description"))
        return res

    @app.post("/api/v1/{username}/{project}/experiments", status_code=201)
    async def create_experiment(username: str, project: str, request: Request, user=Depends(auth)):
        res = await _submit(username, project, request, "experiment")
        return store.get_experiment(res["id"])

    @app.post("/api/v1/{username}/{project}/groups", status_code=201)
    async def create_group(username: str, project: str, request: Request, user=Depends(auth)):
        res = await _submit(username, project, request, "group")
        return store.get_group(res["id"])

    @app.post("/api/v1/{username}/{project}/jobs", status_code=201)
    async def create_job(username: str, project: str, request: Request, user=Depends(auth)):
        res = await _submit(username, project, request, "job")
        return store.get_job(res["id"])

    @app.post("/api/v1/{username}/{project}/builds", status_code=201)
    async def create_build(username: str, project: str, request: Request, user=Depends(auth)):
        res = await _submit(username, project, request, "build")
        return store.get_job(res["id"])

    @app.post("/api/v1/{username}/{project}/pipelines", status_code=201)
    async def create_pipeline(username: str, project: str, request: Request, user=Depends(auth)):
        return await _submit(username, project, request, "pipeline")

    # ------------------------------------------------------------------ experiments
    @app.get("/api/v1/{username}/{project}/experiments")
    def list_experiments(username: str, project: str, request: Request, user=Depends(auth)):
        p = project_or_404(username, project)
        q = request.query_params
        try:
            rows = store.list_experiments(project_id=p["id"], group_id=int(q["group"]) if q.get("group") else None,
                                          independent=q.get("independent", "").lower() in ("1", "true"),
                                          query=q.get("query"), sort=q.get("sort"))
        except QueryError as e:
            raise HTTPException(400, str(e))
        if q.get("metrics", "").lower() in ("1", "true"):
            pass  # last_metric is always included
        if q.get("declarations", "").lower() in ("0", "false"):
            for r in rows:
                r.pop("declarations", None)
        return page(rows, request)

    @app.get("/api/v1/{username}/{project}/experiments/{xid}")
    def get_experiment(username: str, project: str, xid: int, user=Depends(auth)):
        return xp_or_404(username, project, xid)

    @app.patch("/api/v1/{username}/{project}/experiments/{xid}")
    async def update_experiment(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        body = await request.json()
        allowed = {k: v for k, v in body.items() if k in ("name", "description", "tags", "declarations", "run_env")}
        if "declarations" in allowed:
            allowed["declarations"] = dict(store.get_experiment(xid)["declarations"] or {}, **allowed["declarations"])
        store.update_experiment(xid, **allowed)
        flow.auditor.record("experiment.updated", "experiment", xid)
        return store.get_experiment(xid)

    @app.delete("/api/v1/{username}/{project}/experiments/{xid}", status_code=204)
    def delete_experiment(username: str, project: str, xid: int, user=Depends(auth)):
        xp_or_404(username, project, xid)
        flow.stop_experiment(xid, "Deleted")
        store.delete_experiment(xid)
        flow.auditor.record("experiment.deleted", "experiment", xid)
        return PlainTextResponse("", status_code=204)

    for strategy in ("restart", "resume", "copy"):
        def make(strategy=strategy):
            async def clone(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
                xp_or_404(username, project, xid)
                try:
                    body = await request.json()
                except Exception:
                    body = {}
                new = flow.clone_experiment(xid, strategy, declarations=(body or {}).get("declarations"),
                                            content=(body or {}).get("content"))
                return JSONResponse(store.get_experiment(new), status_code=201)
            return clone
        app.post(f"/api/v1/{{username}}/{{project}}/experiments/{{xid}}/{strategy}")(make())

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/stop")
    def stop_experiment(username: str, project: str, xid: int, user=Depends(auth)):
        xp_or_404(username, project, xid)
        flow.stop_experiment(xid)
        return {"stopped": True}

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/statuses")
    def experiment_statuses(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        return page(store.experiment_statuses(xid), request)

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/statuses", status_code=201)
    async def create_experiment_status(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        body = await request.json()
        ok = store.set_experiment_status(xid, body["status"], body.get("message"), body.get("traceback"))
        return {"accepted": ok, "status": store.get_experiment(xid)["status"]}

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/heartbeat")
    def experiment_heartbeat(username: str, project: str, xid: int, user=Depends(auth)):
        """Liveness from the tracking client (deadline: environment.heartbeat_timeout)."""
        xp_or_404(username, project, xid)
        now = time.time()
        store.kv_set(f"heartbeat:experiment:{xid}", now)
        return {"heartbeat": now}

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/metrics")
    def experiment_metrics(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        return page(store.get_metrics(xid), request)

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/metrics", status_code=201)
    async def create_metrics(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        """Single ``{"values": {...}}`` or a list of them (batched ingestion).  ``api.throttle_metrics_per_s``
        > 0 caps requests per experiment (reference throttle scope 'high', config_settings/rest.py:20); a batch
        counts as one request, so batching clients are never slowed down."""
        xp_or_404(username, project, xid)
        rate = settings.get("api.throttle_metrics_per_s")
        if rate:
            now = time.monotonic()
            tokens, last = _metric_buckets.get(xid, (rate, now))
            tokens = min(rate, tokens + (now - last) * rate)
            if tokens < 1.0:
                raise HTTPException(429, "Request was throttled.", headers={"Retry-After": f"{(1 - tokens) / rate:.2f}"})
            _metric_buckets[xid] = (tokens - 1.0, now)
        body = await request.json()
        rows = body if isinstance(body, list) else [body]
        store.add_metrics_batch([(xid, r.get("values", {}), r.get("step"), r.get("created_at")) for r in rows])
        flow.auditor.record("experiment.new_metric", "experiment", xid, n=len(rows))
        return {"created": len(rows)}

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/jobs")
    def experiment_jobs(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        return page(store.experiment_jobs(xid), request)

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/jobs/{jid}")
    def experiment_job(username: str, project: str, xid: int, jid: int, user=Depends(auth)):
        xp_or_404(username, project, xid)
        j = store.get("experiment_jobs", jid)
        if j is None or j["experiment_id"] != xid:
            raise HTTPException(404, "job not found")
        return j

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/jobs/{jid}/statuses")
    def experiment_job_statuses(username: str, project: str, xid: int, jid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        return page(store.experiment_job_statuses(jid), request)

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/logs")
    def experiment_logs(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        tail = request.query_params.get("tail")
        return PlainTextResponse(flow.logs("experiment", xid, int(tail) if tail else None))

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/outputs")
    def experiment_outputs(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        x = xp_or_404(username, project, xid)
        root = x["outputs_path"]
        path = request.query_params.get("path")
        if path:
            full = os.path.realpath(os.path.join(root, path))
            if not full.startswith(os.path.realpath(root)) or not os.path.isfile(full):
                raise HTTPException(404, "file not found")
            flow.auditor.record("experiment.outputs_downloaded", "experiment", xid)
            return FileResponse(full)
        files = []
        for dirpath, _, names in os.walk(root):
            for n in names:
                fp = os.path.join(dirpath, n)
                files.append({"path": os.path.relpath(fp, root), "size": os.path.getsize(fp)})
        return {"outputs_path": root, "files": sorted(files, key=lambda f: f["path"])}

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/coderef")
    def experiment_coderef(username: str, project: str, xid: int, user=Depends(auth)):
        x = xp_or_404(username, project, xid)
        if not x.get("code_reference_id"):
            raise HTTPException(404, "no code reference")
        return store.get("code_references", x["code_reference_id"])

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/bookmark")
    def bookmark(username: str, project: str, xid: int, user=Depends(auth)):
        xp_or_404(username, project, xid)
        store.set_bookmark(user["username"], "experiment", xid, True)
        flow.auditor.record("experiment.bookmarked", "experiment", xid, user["username"])
        return {"bookmarked": True}

    @app.delete("/api/v1/{username}/{project}/experiments/{xid}/unbookmark")
    def unbookmark(username: str, project: str, xid: int, user=Depends(auth)):
        store.set_bookmark(user["username"], "experiment", xid, False)
        return {"bookmarked": False}

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/ephemeraltoken", status_code=201)
    def make_ephemeral(username: str, project: str, xid: int, user=Depends(auth)):
        import uuid as _uuid

        xp_or_404(username, project, xid)
        tok = _uuid.uuid4().hex
        store.kv_set(f"ephemeral:{tok}", {"user": username, "experiment": xid}, ttl=3 * 3600)
        return {"token": tok}

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/token")
    def exchange_token(username: str, project: str, xid: int, user=Depends(auth)):
        """Ephemeral (scoped, 3 h) token -> user token (reference EphemeralAuthentication flow)."""
        scope = user.get("scope")
        if scope is None or scope.get("experiment") != xid:
            raise HTTPException(403, "token is not scoped to this experiment")
        u = store.get_user(username) or store.create_user(username)
        return {"token": u["token"]}

    @app.get("/api/v1/{username}/{project}/experiments/{xid}/chartviews")
    def chartviews(username: str, project: str, xid: int, user=Depends(auth)):
        xp_or_404(username, project, xid)
        return {"results": store.chart_views("experiment", xid)}

    @app.post("/api/v1/{username}/{project}/experiments/{xid}/chartviews", status_code=201)
    async def create_chartview(username: str, project: str, xid: int, request: Request, user=Depends(auth)):
        xp_or_404(username, project, xid)
        body = await request.json()
        cid = store.create_chart_view("experiment", xid, body.get("name", "chart"), body.get("charts", []),
                                      body.get("meta"))
        flow.auditor.record("chart_view.created", "chart_view", cid)
        return {"id": cid}

    # ------------------------------------------------------------------ groups
    @app.get("/api/v1/{username}/{project}/groups")
    def list_groups(username: str, project: str, request: Request, user=Depends(auth)):
        p = project_or_404(username, project)
        return page(store.list_groups(p["id"]), request)

    @app.get("/api/v1/{username}/{project}/groups/{gid}")
    def get_group(username: str, project: str, gid: int, user=Depends(auth)):
        g = group_or_404(username, project, gid)
        g["num_experiments"] = len(store.list_experiments(group_id=gid))
        g["status_counts"] = store.group_status_counts(gid)
        return g

    @app.get("/api/v1/{username}/{project}/groups/{gid}/statuses")
    def group_statuses(username: str, project: str, gid: int, request: Request, user=Depends(auth)):
        group_or_404(username, project, gid)
        return page(store.group_statuses(gid), request)

    @app.get("/api/v1/{username}/{project}/groups/{gid}/experiments")
    def group_experiments(username: str, project: str, gid: int, request: Request, user=Depends(auth)):
        group_or_404(username, project, gid)
        q = request.query_params
        try:
            rows = store.list_experiments(group_id=gid, query=q.get("query"), sort=q.get("sort"))
        except QueryError as e:
            raise HTTPException(400, str(e))
        return page(rows, request)

    @app.get("/api/v1/{username}/{project}/groups/{gid}/metrics")
    def group_metrics(username: str, project: str, gid: int, user=Depends(auth)):
        group_or_404(username, project, gid)
        return {"results": [{"id": x["id"], "last_metric": x["last_metric"], "declarations": x["declarations"]}
                            for x in store.list_experiments(group_id=gid)]}

    @app.get("/api/v1/{username}/{project}/groups/{gid}/iterations")
    def group_iterations(username: str, project: str, gid: int, user=Depends(auth)):
        group_or_404(username, project, gid)
        return {"results": store.iterations(gid)}

    @app.post("/api/v1/{username}/{project}/groups/{gid}/stop")
    async def stop_group(username: str, project: str, gid: int, request: Request, user=Depends(auth)):
        group_or_404(username, project, gid)
        try:
            body = await request.json()
        except Exception:
            body = {}
        flow.stop_group(gid, pending=bool((body or {}).get("pending", False)))
        return {"stopped": True}

    # ------------------------------------------------------------------ jobs / builds / plugins
    for kind, plural in (("job", "jobs"), ("build", "builds")):
        def make_routes(kind=kind, plural=plural):
            @app.get(f"/api/v1/{{username}}/{{project}}/{plural}", name=f"list_{plural}")
            def list_jobs(username: str, project: str, request: Request, user=Depends(auth)):
                p = project_or_404(username, project)
                return page(store.list_jobs(kind=kind, project_id=p["id"]), request)

            @app.get(f"/api/v1/{{username}}/{{project}}/{plural}/{{jid}}", name=f"get_{kind}")
            def get_job(username: str, project: str, jid: int, user=Depends(auth)):
                return job_or_404(username, project, jid, kind)

            @app.get(f"/api/v1/{{username}}/{{project}}/{plural}/{{jid}}/statuses", name=f"{kind}_statuses")
            def job_statuses(username: str, project: str, jid: int, request: Request, user=Depends(auth)):
                job_or_404(username, project, jid, kind)
                return page(store.job_statuses(jid), request)

            @app.get(f"/api/v1/{{username}}/{{project}}/{plural}/{{jid}}/logs", name=f"{kind}_logs")
            def job_logs(username: str, project: str, jid: int, user=Depends(auth)):
                job_or_404(username, project, jid, kind)
                return PlainTextResponse(flow.logs("job", jid))

            @app.post(f"/api/v1/{{username}}/{{project}}/{plural}/{{jid}}/stop", name=f"{kind}_stop")
            def job_stop(username: str, project: str, jid: int, user=Depends(auth)):
                job_or_404(username, project, jid, kind)
                return {"stopped": flow.stop_job(jid)}
        make_routes()

    for plugin in ("notebook", "tensorboard"):
        def make_plugin(plugin=plugin):
            @app.post(f"/api/v1/{{username}}/{{project}}/{plugin}/start", status_code=201, name=f"{plugin}_start")
            async def start(username: str, project: str, request: Request, user=Depends(auth)):
                try:
                    body = await request.json()
                except Exception:
                    body = {}
                content = (body or {}).get("content") or {"version": 1, "kind": plugin}
                store.get_or_create_project(project, username)
                res = flow.submit(content, project=project, user=username)
                return store.get_job(res["id"])

            @app.post(f"/api/v1/{{username}}/{{project}}/{plugin}/stop", name=f"{plugin}_stop")
            def stop(username: str, project: str, user=Depends(auth)):
                p = project_or_404(username, project)
                stopped = [j["id"] for j in store.list_jobs(kind=plugin, project_id=p["id"])
                           if j["status"] not in ("succeeded", "failed", "stopped") and flow.stop_job(j["id"])]
                return {"stopped": stopped}
        make_plugin()

    # ------------------------------------------------------------------ repos (polyaxon upload)
    @app.post("/api/v1/{username}/{project}/repo/upload")
    async def repo_upload(username: str, project: str, request: Request, user=Depends(auth)):
        from polyaxon_amd.polyflow.repos import ProjectRepo

        store.get_or_create_project(project, username)
        data = await request.body()
        try:
            sha = ProjectRepo(flow.paths.repos_root, username, project).upload_tarball(data)
        except Exception as e:
            raise HTTPException(400, f"invalid archive: {e}")
        flow.auditor.record("repo.new_commit", "project", store.get_project(project, username)["id"], commit=sha)
        return {"commit": sha, "path": ProjectRepo(flow.paths.repos_root, username, project).path}

    @app.get("/api/v1/{username}/{project}/repo/download")
    def repo_download(username: str, project: str, user=Depends(auth)):
        from fastapi.responses import Response

        from polyaxon_amd.polyflow.repos import ProjectRepo

        repo = ProjectRepo(flow.paths.repos_root, username, project)
        if not repo.last_commit:
            raise HTTPException(404, "no repo uploaded")
        return Response(repo.archive(), media_type="application/gzip")

    # ------------------------------------------------------------------ pipelines
    @app.get("/api/v1/{username}/{project}/pipelines")
    def list_pipelines(username: str, project: str, request: Request, user=Depends(auth)):
        p = project_or_404(username, project)
        rows = store._rows(store.execute(
            "SELECT p.*, (SELECT COUNT(*) FROM pipeline_runs r WHERE r.pipeline_id = p.id) AS num_runs, "
            "(SELECT r.status FROM pipeline_runs r WHERE r.pipeline_id = p.id ORDER BY r.id DESC LIMIT 1) "
            "AS last_run_status FROM pipelines p WHERE p.project_id = ? ORDER BY p.id DESC", (p["id"],)))
        return page(rows, request)

    @app.get("/api/v1/{username}/{project}/pipelines/{pid}/runs/{rid}")
    def pipeline_run(username: str, project: str, pid: int, rid: int, user=Depends(auth)):
        r = store.get("pipeline_runs", rid)
        if r is None or r["pipeline_id"] != pid:
            raise HTTPException(404, "pipeline run not found")
        r["operations"] = store.operation_runs(rid)
        return r

    @app.get("/api/v1/{username}/{project}/pipelines/{pid}")
    def pipeline_detail(username: str, project: str, pid: int, user=Depends(auth)):
        p = store.get("pipelines", pid)
        if p is None:
            raise HTTPException(404, "pipeline not found")
        p["runs"] = store._rows(store.execute("SELECT * FROM pipeline_runs WHERE pipeline_id = ? ORDER BY id", (pid,)))
        p["schedule_state"] = store.kv_get(f"pipeline_schedule:{pid}")
        return p

    @app.post("/api/v1/{username}/{project}/pipelines/{pid}/stop")
    def pipeline_stop(username: str, project: str, pid: int, user=Depends(auth)):
        if not flow.stop_pipeline(pid):
            raise HTTPException(404, "pipeline not running in this scheduler")
        return {"stopped": pid}

    # ------------------------------------------------------------------ cluster / nodes / activity / searches
    @app.get("/api/v1/cluster")
    def cluster(user=Depends(auth)):
        return {"nodes": store.nodes(), "devices": flow.call(flow.alloc.snapshot)}

    @app.get("/api/v1/nodes")
    def nodes(user=Depends(auth)):
        return {"results": store.nodes()}

    @app.get("/api/v1/nodes/{nid}/gpus")
    def node_gpus(nid: int, user=Depends(auth)):
        return {"results": store.node_gpus(nid)}

    @app.get("/api/v1/activitylogs")
    def activity(request: Request, user=Depends(auth)):
        return page(store.activities(limit=int(request.query_params.get("limit", 100))), request)

    @app.get("/api/v1/notifications")
    def notifications(user=Depends(auth)):
        return {"results": store.notifications()}

    @app.get("/api/v1/searches/{username}/{project}/experiments")
    def searches(username: str, project: str, user=Depends(auth)):
        p = project_or_404(username, project)
        return {"results": store.searches(p["id"], "experiment")}

    @app.post("/api/v1/searches/{username}/{project}/experiments", status_code=201)
    async def create_search(username: str, project: str, request: Request, user=Depends(auth)):
        p = project_or_404(username, project)
        body = await request.json()
        sid = store.create_search(user["username"], p["id"], "experiment", body.get("name", "search"),
                                  {"query": body.get("query"), "sort": body.get("sort")})
        flow.auditor.record("search.created", "search", sid)
        return {"id": sid}

    # ------------------------------------------------------------------ SSE streams (logs / resources / events)
    async def _tail_file_lines(path_fn, is_done_fn, prefix=""):
        pos = 0
        idle = 0
        while True:
            path = path_fn()
            if path and os.path.exists(path):
                with open(path, "r", errors="replace") as f:
                    f.seek(pos)
                    chunk = f.read()
                    pos = f.tell()
                for line in chunk.splitlines():
                    yield f"data: {prefix}{line}\n\n"
                idle = 0 if chunk else idle + 1
            if is_done_fn() and idle > 1:
                yield "event: done\ndata: {}\n\n"
                return
            await asyncio.sleep(0.2)

    @app.get("/streams/v1/{username}/{project}/experiments/{xid}/logs")
    async def stream_logs(username: str, project: str, xid: int, user=Depends(auth)):
        x = xp_or_404(username, project, xid)
        from polyaxon_amd.fsm import ExperimentLifeCycle

        path = lambda: os.path.join(x["logs_path"], "master.0.log")  # noqa: E731
        done = lambda: ExperimentLifeCycle.is_done(store.get_experiment(xid)["status"])  # noqa: E731
        return StreamingResponse(_tail_file_lines(path, done, "master.0 -- "), media_type="text/event-stream")

    @app.get("/streams/v1/{username}/{project}/experiments/{xid}/resources")
    async def stream_resources(username: str, project: str, xid: int, user=Depends(auth)):
        xp_or_404(username, project, xid)
        from polyaxon_amd.obs.telemetry import experiment_resources

        async def gen():
            for _ in range(int(os.environ.get("PLX_STREAM_MAX_TICKS", "1000000"))):
                yield f"data: {json.dumps(experiment_resources(flow, xid))}\n\n"
                await asyncio.sleep(settings.get("telemetry.interval_s"))
        return StreamingResponse(gen(), media_type="text/event-stream")

    return app
