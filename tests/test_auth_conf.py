"""Settings layering, passwords/reserved names, LDAP (against an in-process BER server), OAuth2 SSO (mock
provider), registration workflows over REST."""
import json
import socket
import threading
from urllib.parse import parse_qs, urlparse

import httpx
import pytest

from polyaxon_amd.auth import ldap as L
from polyaxon_amd.auth.passwords import check_password, hash_password, validate_name
from polyaxon_amd.conf import ConfigError, Settings
from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow

TOKEN = "adm1n"


# ---------------------------------------------------------------------------------------------- settings
def test_settings_layering(tmp_path):
    s = Settings.load(env={})
    assert s["api.port"] == 8000 and s["auth.registration"] == "disabled" and s["service"] == "monolith"
    f = tmp_path / "s.yaml"
    f.write_text("api:\n  port: 9001\nauth:\n  ldap:\n    attr_map: {email: mail, name: cn}\n")
    s = Settings.load(env={"PLX_API_PORT": "9100", "POLYAXON_DEBUG": "yes"}, files=[str(f)])
    assert s["api.port"] == 9100 and s.origins["api.port"] == "env"  # env beats file
    assert s["auth.ldap.attr_map"] == {"email": "mail", "name": "cn"} and s["debug"] is True
    s = Settings.load(env={"PLX_API_PORT": "9100"}, overrides={"api.port": 1234})
    assert s["api.port"] == 1234
    # POLYAXON_ spelling is accepted; PLX_ wins when both are set
    assert Settings.load(env={"POLYAXON_API_PORT": "1", "PLX_API_PORT": "2"})["api.port"] == 2
    assert Settings.load(env={}, profile="trial")["logs.level"] == "WARNING"
    assert Settings.load(env={"PLX_BLACKLIST_EXTRA": "foo, bar"})["blacklist.extra"] == ["foo", "bar"]


@pytest.mark.parametrize("env,frag", [
    ({"PLX_API_PORT": "http"}, "api.port"),
    ({"PLX_AUTH_REGISTRATION": "maybe"}, "not in"),
    ({"PLX_API_PORT": "0"}, "minimum"),
    ({"PLX_AUTH_LDAP_ENABLED": "1"}, "server_uri"),
    ({"PLX_AUTH_GITHUB_CLIENT_ID": "x"}, "together"),
    ({"PLX_SERVICE": "nope"}, "nope"),
])
def test_settings_reject_bad_values(env, frag):
    with pytest.raises(ConfigError, match=frag):
        Settings.load(env=env)


def test_settings_secrets_redacted_and_unknown_keys():
    s = Settings.load(env={"PLX_AUTH_GITHUB_CLIENT_ID": "cid", "PLX_AUTH_GITHUB_CLIENT_SECRET": "s3cret"})
    assert s.as_dict()["auth.github.client_secret"] == "***"
    assert s.as_dict(redact=False)["auth.github.client_secret"] == "s3cret"
    assert s.sso_providers() == ["github"]
    with pytest.raises(ConfigError, match="unknown setting"):
        Settings.load(env={}, overrides={"api.nope": 1})


# ---------------------------------------------------------------------------------------------- passwords
def test_password_hash_and_names():
    h = hash_password("correct horse", iterations=1000)
    assert check_password("correct horse", h) and not check_password("wrong", h)
    assert not check_password("x", "garbage")
    assert validate_name("alice") == "alice"
    for bad in ("admin", "API", "", "a/b", "-x", "x" * 200):
        with pytest.raises(ValueError):
            validate_name(bad)
    with pytest.raises(ValueError):
        validate_name("acme", extra_reserved=["ACME"])


# ---------------------------------------------------------------------------------------------- LDAP
class FakeLDAP:
    """Speaks just enough RFC 4511 to answer bind/search/unbind: users = {dn: (password, attrs)}."""

    def __init__(self, users, service=("cn=svc,dc=ex", "svcpw")):
        self.users = users
        self.service = service
        self.filters = []
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(8)
        self.port = self.sock.getsockname()[1]
        threading.Thread(target=self._serve, daemon=True).start()

    def _serve(self):
        while True:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._conn, args=(c,), daemon=True).start()

    def _match(self, tag, content, attrs, dn):
        if tag == 0xA3:
            (_, a), (_, v) = L.children(content)
            if a.decode().lower() == "dn":
                return v.decode() == dn
            return v.decode() in attrs.get(a.decode(), [])
        if tag == 0x87:
            return True
        if tag in (0xA0, 0xA1):
            rs = [self._match(t, c, attrs, dn) for t, c in L.children(content)]
            return all(rs) if tag == 0xA0 else any(rs)
        if tag == 0xA2:
            (t, c), = L.children(content)
            return not self._match(t, c, attrs, dn)
        return False

    def _conn(self, c):
        buf = b""
        while True:
            try:
                _, content, end = L.read_tlv(buf)
            except EOFError:
                chunk = c.recv(65536)
                if not chunk:
                    c.close()
                    return
                buf += chunk
                continue
            buf = buf[end:]
            (_, mid), (tag, op) = L.children(content)[:2]
            mid = L.as_int(mid)
            if tag == 0x42:
                c.close()
                return
            if tag == 0x60:
                parts = L.children(op)
                dn, pw = parts[1][1].decode(), parts[2][1].decode()
                ok = (dn, pw) == self.service or (dn in self.users and self.users[dn][0] == pw)
                code = 0 if ok else 49
                c.sendall(L.seq(L.ber_int(mid), L.seq(L.ber_int(code, 0x0A), L.ber_str(""), L.ber_str(""),
                                                        tag=0x61)))
            elif tag == 0x63:
                parts = L.children(op)
                base = parts[0][1].decode()
                ftag, fcontent = parts[6]
                self.filters.append((ftag, fcontent))
                for dn, (_, attrs) in self.users.items():
                    if dn.endswith(base) and self._match(ftag, fcontent, attrs, dn):
                        pa = b"".join(L.seq(L.ber_str(k), L.seq(*[L.ber_str(v) for v in vs], tag=0x31))
                                      for k, vs in attrs.items())
                        c.sendall(L.seq(L.ber_int(mid), L.seq(L.ber_str(dn), L.seq(pa), tag=0x64)))
                c.sendall(L.seq(L.ber_int(mid), L.seq(L.ber_int(0, 0x0A), L.ber_str(""), L.ber_str(""), tag=0x65)))

    def close(self):
        self.sock.close()


USERS = {"uid=alice,ou=people,dc=ex": ("wonderland", {"uid": ["alice"], "mail": ["alice@ex.org"]}),
         "uid=bob,ou=people,dc=ex": ("builder", {"uid": ["bob"], "mail": ["bob@ex.org"]})}


@pytest.fixture
def ldap_server():
    srv = FakeLDAP(USERS)
    yield srv
    srv.close()


def test_ldap_filter_encoding():
    assert L.encode_filter("(uid=a)") == L.tlv(0xA3, L.ber_str("uid") + L.ber_str("a"))
    f = L.encode_filter("(&(objectClass=*)(|(uid=a)(!(uid=b))))")
    assert f[0] == 0xA0
    esc = L.escape_filter_value("a*)(uid=*")
    assert "*" not in esc and "(" not in esc
    # escaped value decodes back to the literal string, as a single equality assertion
    assert L.encode_filter(f"(uid={esc})") == L.tlv(0xA3, L.ber_str("uid") + L.ber_str("a*)(uid=*"))
    with pytest.raises(ValueError):
        L.encode_filter("(uid=a")
    big = L.ber_str("x" * 300)
    assert L.read_tlv(big)[1] == b"x" * 300


def test_ldap_dn_template_and_search(ldap_server):
    uri = f"ldap://127.0.0.1:{ldap_server.port}"
    tmpl = L.LDAPAuthenticator(uri, user_dn_template="uid={username},ou=people,dc=ex")
    info = tmpl.authenticate("alice", "wonderland")
    assert info["dn"] == "uid=alice,ou=people,dc=ex" and info["email"] == "alice@ex.org"
    assert tmpl.authenticate("alice", "nope") is None
    assert tmpl.authenticate("alice", "") is None  # never an anonymous bind
    search = L.LDAPAuthenticator(uri, bind_dn="cn=svc,dc=ex", bind_password="svcpw", search_base_dn="dc=ex")
    assert search.authenticate("bob", "builder")["email"] == "bob@ex.org"
    assert search.authenticate("bob", "wonderland") is None
    assert search.authenticate("carol", "x") is None
    # injection: the wildcard is escaped, so it matches nobody instead of everybody
    assert search.authenticate("*", "builder") is None


# ---------------------------------------------------------------------------------------------- REST
def _github_transport(calls):
    def handler(req: httpx.Request):
        calls.append(str(req.url))
        if req.url.path == "/login/oauth/access_token":
            form = parse_qs(req.content.decode())
            if form.get("code") != ["good"]:
                return httpx.Response(200, json={"error": "bad_verification_code"})
            return httpx.Response(200, json={"access_token": "gho_1", "token_type": "bearer"})
        assert req.headers["authorization"] == "Bearer gho_1"
        if req.url.path == "/user":
            return httpx.Response(200, json={"id": 42, "login": "octo", "name": "Octo Cat", "email": None})
        if req.url.path == "/user/emails":
            return httpx.Response(200, json=[{"email": "x@y", "primary": False, "verified": True},
                                             {"email": "octo@gh.io", "primary": True, "verified": True}])
        return httpx.Response(404)
    return httpx.MockTransport(handler)


@pytest.fixture
def make_api(tmp_path):
    from fastapi.testclient import TestClient

    from polyaxon_amd.api.server import create_app

    flows = []

    def build(env, transport=None):
        flow = Polyflow(str(tmp_path / f"plx{len(flows)}"), allocator=DeviceAllocator([Device(0)])).start()
        flows.append(flow)
        st = Settings.load(env=env)
        client = TestClient(create_app(flow, admin_token=TOKEN, settings=st, sso_transport=transport))
        return client
    yield build
    for f in flows:
        f.shutdown()


def _h(tok):
    return {"Authorization": f"token {tok}"}


def test_password_login_logout_and_registration(make_api):
    client = make_api({"PLX_AUTH_REGISTRATION": "superuser_validation", "PLX_AUTH_TOKEN_TTL_S": "3600"})
    r = client.post("/api/v1/users", json={"username": "ann", "password": "hunter2hunter2"}, headers=_h(TOKEN))
    assert r.status_code == 201
    assert client.post("/api/v1/users/token", json={"username": "ann", "password": "bad"}).status_code == 401
    tok = client.post("/api/v1/users/token", json={"username": "ann", "password": "hunter2hunter2"}).json()["token"]
    assert client.get("/api/v1/users", headers=_h(tok)).json()["username"] == "ann"
    r = client.post("/api/v1/users/password", json={"old_password": "hunter2hunter2", "new_password": "123"},
                    headers=_h(tok))
    assert r.status_code == 400  # too short
    assert client.post("/api/v1/users/password", json={"old_password": "hunter2hunter2",
                                                       "new_password": "n3w-passw0rd"}, headers=_h(tok)).is_success
    assert client.post("/api/v1/users/logout", headers=_h(tok)).is_success
    assert client.get("/api/v1/users", headers=_h(tok)).status_code == 401  # token rotated away
    assert client.post("/api/v1/users/token", json={"username": "ann", "password": "n3w-passw0rd"}).is_success
    # reserved / malformed names
    assert client.post("/api/v1/users", json={"username": "admin"}, headers=_h(TOKEN)).status_code == 400
    assert client.post("/api/v1/projects", json={"name": "streams"}, headers=_h(TOKEN)).status_code == 400
    # registration awaiting superuser validation
    r = client.post("/api/v1/users/register", json={"username": "zed", "email": "z@x", "password": "zzzzzzzz9"})
    assert r.status_code == 201 and r.json()["is_active"] is False and "token" not in r.json()
    assert client.post("/api/v1/users/token", json={"username": "zed", "password": "zzzzzzzz9"}).status_code == 403
    assert [u["username"] for u in client.get("/api/v1/users/pending", headers=_h(TOKEN)).json()["results"]] == ["zed"]
    assert client.post("/api/v1/users/zed/activate", headers=_h(tok)).status_code in (401, 403)
    assert client.post("/api/v1/users/zed/activate", headers=_h(TOKEN)).is_success
    ztok = client.post("/api/v1/users/token", json={"username": "zed", "password": "zzzzzzzz9"}).json()["token"]
    assert client.get("/api/v1/users", headers=_h(ztok)).is_success
    assert client.post("/api/v1/users/zed/deactivate", headers=_h(TOKEN)).is_success
    assert client.get("/api/v1/users", headers=_h(ztok)).status_code == 401


def test_registration_disabled_and_open(make_api):
    c = make_api({})
    assert c.post("/api/v1/users/register", json={"username": "a1", "password": "aaaaaaaa1"}).status_code == 403
    c = make_api({"PLX_AUTH_REGISTRATION": "open"})
    r = c.post("/api/v1/users/register", json={"username": "a1", "password": "aaaaaaaa1"})
    assert r.status_code == 201 and c.get("/api/v1/users", headers=_h(r.json()["token"])).is_success
    assert c.post("/api/v1/users/register", json={"username": "a1", "password": "aaaaaaaa1"}).status_code == 400


def test_ldap_login_over_rest(make_api, ldap_server):
    c = make_api({"PLX_AUTH_LDAP_ENABLED": "true", "PLX_AUTH_LDAP_SERVER_URI": f"ldap://127.0.0.1:{ldap_server.port}",
                  "PLX_AUTH_LDAP_BIND_DN": "cn=svc,dc=ex", "PLX_AUTH_LDAP_BIND_PASSWORD": "svcpw",
                  "PLX_AUTH_LDAP_SEARCH_BASE_DN": "dc=ex"})
    assert c.get("/api/v1/sso/providers").json() == {"providers": [], "ldap": True}
    assert c.post("/api/v1/users/token", json={"username": "alice", "password": "x"}).status_code == 401
    r = c.post("/api/v1/users/token", json={"username": "alice", "password": "wonderland"})
    assert r.status_code == 200, r.text
    me = c.get("/api/v1/users", headers=_h(r.json()["token"])).json()
    assert me["username"] == "alice" and me["email"] == "alice@ex.org"
    # second login reuses the user
    assert c.post("/api/v1/users/token", json={"username": "alice", "password": "wonderland"}).is_success


def test_github_sso_flow(make_api):
    calls = []
    c = make_api({"PLX_AUTH_GITHUB_CLIENT_ID": "cid", "PLX_AUTH_GITHUB_CLIENT_SECRET": "csec",
                  "PLX_AUTH_GITHUB_URL": "https://gh.test", "PLX_AUTH_GITHUB_API_URL": "https://api.gh.test"},
                 transport=_github_transport(calls))
    assert c.get("/api/v1/sso/providers").json()["providers"] == ["github"]
    assert c.get("/oauth/gitlab/login", follow_redirects=False).status_code == 404
    r = c.get("/oauth/github/login", follow_redirects=False)
    assert r.status_code == 302
    loc = urlparse(r.headers["location"])
    q = parse_qs(loc.query)
    assert loc.netloc == "gh.test" and q["client_id"] == ["cid"] and q["scope"] == ["user:email"]
    state = q["state"][0]
    tampered = state[:-1] + ("1" if state[-1] == "0" else "0")  # always a different last character
    bad = c.get("/oauth/github/complete", params={"code": "good", "state": tampered})
    assert bad.status_code == 400
    r = c.get("/oauth/github/complete", params={"code": "good", "state": state})
    assert r.status_code == 200, r.text
    out = r.json()
    assert out["username"] == "octo" and out["email"] == "octo@gh.io"
    assert c.get("/api/v1/users", headers=_h(out["token"])).json()["username"] == "octo"
    # a state is single-use
    assert c.get("/oauth/github/complete", params={"code": "good", "state": state}).status_code == 400
    # a second sign-in links to the same user; a bad code fails cleanly
    st2 = parse_qs(urlparse(c.get("/oauth/github/login", follow_redirects=False).headers["location"]).query)["state"][0]
    assert c.get("/oauth/github/complete", params={"code": "good", "state": st2}).json()["username"] == "octo"
    st3 = parse_qs(urlparse(c.get("/oauth/github/login", follow_redirects=False).headers["location"]).query)["state"][0]
    assert c.get("/oauth/github/complete", params={"code": "bad", "state": st3}).status_code == 400
    assert any(u.endswith("/user/emails") for u in calls)


def test_settings_cli(tmp_path, monkeypatch, capsys):
    from polyaxon_amd.cli.main import main

    monkeypatch.setenv("PLX_CONFIG", str(tmp_path / "c.yaml"))
    monkeypatch.setenv("PLX_API_PORT", "8123")
    assert main(["--json", "settings"]) == 0
    rows = {r["key"]: r for r in json.loads(capsys.readouterr().out)}
    assert rows["api.port"]["value"] == 8123 and rows["api.port"]["origin"] == "env"
    assert main(["settings", "--set", "api.port=abc"]) == 1


def test_settings_drive_scheduler_and_observability(tmp_path):
    import socket as _s

    from polyaxon_amd.obs.events import Stats

    recv = _s.socket(_s.AF_INET, _s.SOCK_DGRAM)
    recv.bind(("127.0.0.1", 0))
    recv.settimeout(5)
    st = Settings.load(env={"PLX_STATS_BACKEND": "datadog", "PLX_STATS_PORT": str(recv.getsockname()[1]),
                            "PLX_TRACKER_BACKEND": "jsonl", "PLX_SCHEDULER_RECONCILE_INTERVAL_S": "0.5",
                            "PLX_SCHEDULER_BUILD_REUSE_S": "60"})
    flow = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0)]), settings=st)
    try:
        assert flow.reconcile_s == 0.5 and flow.build_reuse_s == 60.0
        flow.auditor.record("project.created", "project", 1, "ann")
        line = recv.recv(4096).decode()
        assert line.startswith("polyaxon.project.created:1|c|#") and "service:monolith" in line
        ev = json.loads((tmp_path / "plx" / "tracker" / "events.jsonl").read_text().splitlines()[0])
        assert ev["event"] == "project.created" and ev["actor"] == "ann"
    finally:
        recv.close()
    assert Stats(None)._line("a", "1", "c") == "polyaxon.a:1|c"


def test_metric_throttle(make_api):
    c = make_api({"PLX_API_THROTTLE_METRICS_PER_S": "2"})
    assert c.post("/api/v1/projects", json={"name": "p1"}, headers=_h(TOKEN)).status_code == 201
    x = c.post("/api/v1/root/p1/experiments", json={"content": {"version": 1, "kind": "experiment",
                                                               "run": {"cmd": "true"}}}, headers=_h(TOKEN)).json()
    url = f"/api/v1/root/p1/experiments/{x['id']}/metrics"
    codes = [c.post(url, json={"values": {"loss": 1.0}}, headers=_h(TOKEN)).status_code for _ in range(4)]
    assert codes[:2] == [201, 201] and 429 in codes[2:]
    # a batch is one request: 50 points go through in one call once the bucket refills
    import time as _t
    _t.sleep(0.6)
    r = c.post(url, json=[{"values": {"loss": float(i)}, "step": i} for i in range(50)], headers=_h(TOKEN))
    assert r.status_code == 201 and r.json()["created"] == 50
