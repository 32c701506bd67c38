"""User accounts over the tracking store: passwords, login/logout, registration, LDAP and SSO sign-in.

Reference: api/users/views.py (``LoginView``/``LogoutView``/``TokenView``, ``SimpleRegistrationView`` +
superuser activation, password change), config_settings/registration.py (``REGISTRATION_WORKFLOW``:
superuser validation vs. open), sso/wizard.py (create-or-link the user behind an identity).

API tokens stay in ``users.token`` (what every request authenticates with).  Credentials live in their own
table: a PBKDF2 hash for local users, ``provider``/``external_id`` for LDAP and SSO identities, an
``is_active`` flag for registrations awaiting validation, and an optional token expiry.
"""
from __future__ import annotations

import time
import uuid
from typing import Any, Dict, Optional

from polyaxon_amd.auth.ldap import LDAPAuthenticator
from polyaxon_amd.auth.oauth import OAuthError, OAuthFlow, provider_from_settings
from polyaxon_amd.auth.passwords import check_password, check_strength, hash_password, validate_name

CREDENTIALS_SCHEMA = """
CREATE TABLE IF NOT EXISTS user_credentials (username TEXT PRIMARY KEY, password_hash TEXT, provider TEXT,
    external_id TEXT, is_active INTEGER DEFAULT 1, token_expires_at REAL, updated_at REAL,
    UNIQUE(provider, external_id));
"""


class AuthError(RuntimeError):
    def __init__(self, message: str, status: int = 401):
        super().__init__(message)
        self.status = status


class Accounts:
    def __init__(self, store, settings, transport=None):
        self.store = store
        self.s = settings
        self.transport = transport
        store.conn().executescript(CREDENTIALS_SCHEMA)
        key = settings.get("secret.key") or store.kv_get("secret:key")
        if not key:
            key = uuid.uuid4().hex + uuid.uuid4().hex
            store.kv_set("secret:key", key)
        self.flow = OAuthFlow(key, lambda n, ttl: store.kv_set(f"oauth_nonce:{n}", 1, ttl), self._pop_nonce,
                              transport)

    # ------------------------------------------------------------------ helpers
    def _pop_nonce(self, nonce: str) -> bool:
        k = f"oauth_nonce:{nonce}"
        if self.store.kv_get(k) is None:
            return False
        self.store.kv_delete(k)
        return True

    def _cred(self, username: str) -> Optional[Dict[str, Any]]:
        r = self.store.execute("SELECT * FROM user_credentials WHERE username = ?", (username,)).fetchone()
        return dict(r) if r else None

    def _upsert_cred(self, username: str, **values) -> None:
        cur = self._cred(username)
        values["updated_at"] = time.time()
        if cur is None:
            cols = ["username"] + list(values)
            self.store.execute(f"INSERT INTO user_credentials ({', '.join(cols)}) VALUES "
                               f"({', '.join('?' * len(cols))})", [username] + list(values.values()))
        else:
            sets = ", ".join(f"{k} = ?" for k in values)
            self.store.execute(f"UPDATE user_credentials SET {sets} WHERE username = ?",
                               list(values.values()) + [username])

    def _issue_token(self, username: str) -> Dict[str, Any]:
        tok = uuid.uuid4().hex
        self.store.execute("UPDATE users SET token = ? WHERE username = ?", (tok, username))
        ttl = self.s.get("auth.token_ttl_s")
        self._upsert_cred(username, token_expires_at=(time.time() + ttl) if ttl else None)
        return self.store.get_user(username)

    def _new_user(self, username: str, email: str = "", superuser: bool = False) -> Dict[str, Any]:
        try:
            validate_name(username, self.s.get("blacklist.extra"))
        except ValueError as e:
            raise AuthError(str(e), 400)
        if self.store.get_user(username):
            raise AuthError(f"user {username} exists", 400)
        return self.store.create_user(username, email or "", superuser)

    # ------------------------------------------------------------------ request-time checks
    def token_valid(self, user: Dict[str, Any]) -> bool:
        c = self._cred(user["username"])
        if c is None:
            return True
        if not c.get("is_active"):
            return False
        exp = c.get("token_expires_at")
        return exp is None or time.time() < exp

    # ------------------------------------------------------------------ local passwords
    def set_password(self, username: str, password: str) -> None:
        if not self.store.get_user(username):
            raise AuthError(f"user {username} not found", 404)
        try:
            check_strength(password, self.s.get("auth.password_min_length"))
        except ValueError as e:
            raise AuthError(str(e), 400)
        self._upsert_cred(username, password_hash=hash_password(password))

    def change_password(self, username: str, old: str, new: str) -> None:
        c = self._cred(username)
        if not c or not c.get("password_hash") or not check_password(old or "", c["password_hash"]):
            raise AuthError("old password is incorrect", 400)
        self.set_password(username, new)

    def login(self, username: str, password: str) -> Dict[str, Any]:
        """Local password first, then LDAP (which creates the user on first sign-in)."""
        c = self._cred(username) if username else None
        if c and c.get("password_hash"):
            if not check_password(password or "", c["password_hash"]):
                raise AuthError("invalid credentials")
            if not c.get("is_active"):
                raise AuthError("account awaiting activation", 403)
            return self._issue_token(username)
        ldap = LDAPAuthenticator.from_settings(self.s)
        if ldap is not None and (c is None or c.get("provider") == "ldap"):
            try:
                info = ldap.authenticate(username, password)
            except (OSError, ConnectionError) as e:
                raise AuthError(f"LDAP server unavailable: {e}", 503)
            if info is None:
                raise AuthError("invalid credentials")
            if not self.store.get_user(username):
                self._new_user(username, info.get("email", ""))
            self._upsert_cred(username, provider="ldap", external_id=info["dn"], is_active=1)
            if info.get("email"):
                self.store.execute("UPDATE users SET email = ? WHERE username = ?", (info["email"], username))
            return self._issue_token(username)
        raise AuthError("invalid credentials")

    def logout(self, username: str) -> None:
        """Invalidate the current token by rotating it; the new one is not returned."""
        self.store.execute("UPDATE users SET token = ? WHERE username = ?", (uuid.uuid4().hex, username))

    # ------------------------------------------------------------------ registration
    def register(self, username: str, email: str, password: str) -> Dict[str, Any]:
        wf = self.s.get("auth.registration")
        if wf == "disabled":
            raise AuthError("registration is disabled", 403)
        try:
            check_strength(password, self.s.get("auth.password_min_length"))
        except ValueError as e:
            raise AuthError(str(e), 400)
        self._new_user(username, email)
        active = wf == "open"
        self._upsert_cred(username, password_hash=hash_password(password), is_active=int(active))
        if not active:  # no usable token until a superuser validates the account
            self.store.execute("UPDATE users SET token = NULL WHERE username = ?", (username,))
            return {"username": username, "email": email, "is_active": False}
        u = self._issue_token(username)
        return {"username": username, "email": email, "is_active": True, "token": u["token"]}

    def activate(self, username: str) -> None:
        if not self.store.get_user(username):
            raise AuthError(f"user {username} not found", 404)
        self._upsert_cred(username, is_active=1)
        if not self.store.get_user(username).get("token"):
            self.store.execute("UPDATE users SET token = ? WHERE username = ?", (uuid.uuid4().hex, username))

    def deactivate(self, username: str) -> None:
        self._upsert_cred(username, is_active=0)

    def pending(self):
        rows = self.store.execute("SELECT u.username, u.email, u.created_at FROM users u JOIN user_credentials c "
                                  "ON c.username = u.username WHERE c.is_active = 0 ORDER BY u.id").fetchall()
        return [dict(r) for r in rows]

    # ------------------------------------------------------------------ SSO
    def sso_providers(self):
        return self.s.sso_providers()

    def _provider(self, name: str):
        p = provider_from_settings(name, self.s) if name in ("github", "gitlab", "bitbucket", "azure") else None
        if p is None:
            raise AuthError(f"SSO provider {name!r} is not configured", 404)
        return p

    def sso_login_url(self, name: str, redirect_uri: str) -> str:
        return self.flow.login_url(self._provider(name), redirect_uri)

    def sso_complete(self, name: str, code: str, state: str, redirect_uri: str) -> Dict[str, Any]:
        p = self._provider(name)
        try:
            ident = self.flow.complete(p, code, state, redirect_uri)
        except OAuthError as e:
            raise AuthError(f"SSO failed: {e}", 400)
        row = self.store.execute("SELECT username FROM user_credentials WHERE provider = ? AND external_id = ?",
                                 (name, ident["external_id"])).fetchone()
        if row:
            username = row[0]
        else:  # first sign-in: create the user, de-duplicating the name
            base = ident["username"]
            username, k = base, 1
            while self.store.get_user(username):
                k += 1
                username = f"{base}{k}"
            try:
                self._new_user(username, ident.get("email") or "")
            except AuthError:
                username = f"{name}-{ident['external_id']}"
                self._new_user(username, ident.get("email") or "")
            self._upsert_cred(username, provider=name, external_id=ident["external_id"], is_active=1)
        c = self._cred(username)
        if c and not c.get("is_active"):
            raise AuthError("account deactivated", 403)
        u = self._issue_token(username)
        return {"username": username, "email": u.get("email"), "token": u["token"], "provider": name}
