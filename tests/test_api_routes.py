"""Every REST route refuses anonymous and wrong-token callers.

The reference enforces this by inheriting ``BaseViewTest.test_requires_auth`` into every view test
(tests/utils.py:284-316).  Here the sweep walks the app's route table instead, so a route added without an
auth dependency fails this test by construction.  Public routes (health, login / registration / SSO
entry points, the dashboard shell) are listed explicitly."""
import re

import pytest

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow

TOKEN = "t0ken"

# routes reachable without a token (by design)
PUBLIC = {
    "/_health", "/_status", "/ui", "/", "/favicon.ico",
    "/api/v1/users/token", "/api/v1/users/register", "/api/v1/users/activate/{key}",
}
PUBLIC_PREFIXES = ("/oauth/", "/docs", "/redoc", "/openapi", "/static", "/api/v1/users/token",
                   "/api/v1/users/register", "/api/v1/sso", "/api/v1/versions/")


def _fill(path: str) -> str:
    return re.sub(r"\{([^}]+)\}", lambda m: "1" if ("id" in m.group(1) or m.group(1) in ("index", "rid"))
                  else "root", path)


@pytest.fixture(scope="module")
def app_and_client(tmp_path_factory):
    from fastapi.testclient import TestClient

    from polyaxon_amd.api.server import create_app

    flow = Polyflow(str(tmp_path_factory.mktemp("plx")), allocator=DeviceAllocator([Device(0)])).start()
    app = create_app(flow, admin_token=TOKEN)
    yield app, TestClient(app)
    flow.shutdown()


def _protected_routes(app):
    out = []
    for r in app.routes:
        path = getattr(r, "path", "")
        if path in PUBLIC or path.startswith(PUBLIC_PREFIXES):
            continue
        for m in sorted(getattr(r, "methods", None) or ()):
            if m not in ("HEAD", "OPTIONS"):
                out.append((m, path))
    return out


def test_route_table_is_large(app_and_client):
    app, _ = app_and_client
    assert len(_protected_routes(app)) >= 60


@pytest.mark.parametrize("header", [None, "token wrong", "Bearer nope"])
def test_every_route_requires_auth(app_and_client, header):
    app, client = app_and_client
    open_routes = []
    for m, path in _protected_routes(app):
        headers = {"Authorization": header} if header else {}
        r = client.request(m, _fill(path), headers=headers, json={})
        if r.status_code not in (401, 403):
            open_routes.append((m, path, r.status_code))
    assert not open_routes, open_routes


def test_authenticated_sweep_has_no_server_errors(app_and_client):
    """With a valid token no route may crash on an unknown entity: 2xx/4xx only (the reference's views
    answer 404 for missing objects and 400 for bad payloads)."""
    app, client = app_and_client
    crashed = []
    for m, path in _protected_routes(app):
        if m == "DELETE" or path.startswith("/streams/"):
            continue  # deletions of the sweep's own fixtures / endless SSE streams
        r = client.request(m, _fill(path), headers={"Authorization": f"token {TOKEN}"}, json={})
        if r.status_code >= 500:
            crashed.append((m, path, r.status_code))
    assert not crashed, crashed
