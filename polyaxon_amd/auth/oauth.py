"""OAuth 2.0 single sign-on: GitHub, GitLab, Bitbucket, Azure AD.

Reference: sso/providers/oauth2/provider.py (authorize URL, code -> access token exchange, ``get_oauth_data``),
sso/providers/{github,gitlab,bitbucket,azure}_provider.py (user/e-mail lookups), sso/wizard.py:26-121 (state
kept across the redirect).  Flow here:

1. ``login_url(provider)`` returns the provider's authorize URL with a signed, single-use ``state``;
2. the provider redirects to ``/oauth/<provider>/complete?code=...&state=...``;
3. ``complete()`` checks the state (HMAC + one-time nonce + 10 min age), exchanges the code for an access
   token, fetches the identity and returns ``{external_id, username, email, name}``.

HTTP goes through ``httpx``; tests inject an ``httpx.MockTransport`` in place of the real provider.
"""
from __future__ import annotations

import hashlib
import hmac
import secrets
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, Optional
from urllib.parse import urlencode

import httpx

STATE_MAX_AGE_S = 600.0


class OAuthError(RuntimeError):
    pass


@dataclass
class Provider:
    name: str
    client_id: str
    client_secret: str
    authorize_url: str
    token_url: str
    user_url: str
    scopes: str
    email_url: Optional[str] = None

    def identity(self, user: Dict[str, Any], emails: Any) -> Dict[str, Any]:
        if self.name == "github":
            email = user.get("email")
            if not email and isinstance(emails, list):  # private e-mail: pick the primary verified one
                prim = [e for e in emails if e.get("primary") and e.get("verified")] or \
                       [e for e in emails if e.get("verified")]
                email = prim[0]["email"] if prim else None
            return {"external_id": str(user["id"]), "username": user.get("login"), "email": email,
                    "name": user.get("name")}
        if self.name == "gitlab":
            return {"external_id": str(user["id"]), "username": user.get("username"), "email": user.get("email"),
                    "name": user.get("name")}
        if self.name == "bitbucket":
            email = None
            if isinstance(emails, dict):
                vals = [e for e in emails.get("values", []) if e.get("is_primary")]
                email = vals[0]["email"] if vals else None
            return {"external_id": str(user.get("uuid") or user.get("account_id")),
                    "username": user.get("username") or user.get("nickname"), "email": email,
                    "name": user.get("display_name")}
        if self.name == "azure":
            email = user.get("mail") or user.get("userPrincipalName")
            return {"external_id": str(user["id"]), "username": (email or "").split("@")[0] or None, "email": email,
                    "name": user.get("displayName")}
        raise OAuthError(f"unknown provider {self.name}")


def provider_from_settings(name: str, s) -> Optional[Provider]:
    cid, sec = s.get(f"auth.{name}.client_id"), s.get(f"auth.{name}.client_secret")
    if not cid:
        return None
    if name == "github":
        url, api = s.get("auth.github.url").rstrip("/"), s.get("auth.github.api_url").rstrip("/")
        return Provider(name, cid, sec, f"{url}/login/oauth/authorize", f"{url}/login/oauth/access_token",
                        f"{api}/user", "user:email", f"{api}/user/emails")
    if name == "gitlab":
        url = s.get("auth.gitlab.url").rstrip("/")
        return Provider(name, cid, sec, f"{url}/oauth/authorize", f"{url}/oauth/token", f"{url}/api/v4/user",
                        "read_user")
    if name == "bitbucket":
        url, api = s.get("auth.bitbucket.url").rstrip("/"), s.get("auth.bitbucket.api_url").rstrip("/")
        return Provider(name, cid, sec, f"{url}/site/oauth2/authorize", f"{url}/site/oauth2/access_token",
                        f"{api}/2.0/user", "account email", f"{api}/2.0/user/emails")
    if name == "azure":
        url, tenant = s.get("auth.azure.url").rstrip("/"), s.get("auth.azure.tenant_id")
        api = s.get("auth.azure.api_url").rstrip("/")
        return Provider(name, cid, sec, f"{url}/{tenant}/oauth2/v2.0/authorize", f"{url}/{tenant}/oauth2/v2.0/token",
                        f"{api}/v1.0/me", "openid email profile User.Read")
    raise OAuthError(f"unknown provider {name}")


class OAuthFlow:
    """State signing + code exchange.  ``nonce_store`` is a (set, pop) pair over the platform kv store so
    a state can be redeemed once."""

    def __init__(self, secret_key: str, nonce_put: Callable[[str, float], None],
                 nonce_pop: Callable[[str], bool], transport: Optional[httpx.BaseTransport] = None):
        self.key = secret_key.encode()
        self.nonce_put = nonce_put
        self.nonce_pop = nonce_pop
        self.transport = transport

    def _sign(self, msg: str) -> str:
        return hmac.new(self.key, msg.encode(), hashlib.sha256).hexdigest()[:32]

    def make_state(self, provider: str, now: Optional[float] = None) -> str:
        nonce = secrets.token_urlsafe(12)
        ts = int(now if now is not None else time.time())
        self.nonce_put(nonce, STATE_MAX_AGE_S)
        body = f"{provider}.{nonce}.{ts}"
        return f"{body}.{self._sign(body)}"

    def check_state(self, provider: str, state: str, now: Optional[float] = None) -> None:
        try:
            prov, nonce, ts, sig = state.split(".")
        except (AttributeError, ValueError):
            raise OAuthError("malformed state")
        if not hmac.compare_digest(sig, self._sign(f"{prov}.{nonce}.{ts}")) or prov != provider:
            raise OAuthError("bad state signature")
        if (now if now is not None else time.time()) - int(ts) > STATE_MAX_AGE_S:
            raise OAuthError("state expired")
        if not self.nonce_pop(nonce):
            raise OAuthError("state already used")

    def login_url(self, p: Provider, redirect_uri: str) -> str:
        q = {"client_id": p.client_id, "redirect_uri": redirect_uri, "response_type": "code", "scope": p.scopes,
             "state": self.make_state(p.name)}
        return f"{p.authorize_url}?{urlencode(q)}"

    def complete(self, p: Provider, code: str, state: str, redirect_uri: str) -> Dict[str, Any]:
        self.check_state(p.name, state)
        if not code:
            raise OAuthError("missing code")
        with httpx.Client(transport=self.transport, timeout=10.0) as http:
            r = http.post(p.token_url, data={"grant_type": "authorization_code", "code": code,
                                             "redirect_uri": redirect_uri, "client_id": p.client_id,
                                             "client_secret": p.client_secret},
                          headers={"Accept": "application/json"})
            if r.status_code != 200:
                raise OAuthError(f"token exchange failed: HTTP {r.status_code}")
            tok = r.json()
            if "access_token" not in tok:
                raise OAuthError(f"token exchange failed: {tok.get('error_description') or tok.get('error')}")
            hdr = {"Authorization": f"Bearer {tok['access_token']}", "Accept": "application/json"}
            u = http.get(p.user_url, headers=hdr)
            if u.status_code != 200:
                raise OAuthError(f"user lookup failed: HTTP {u.status_code}")
            emails = None
            if p.email_url:
                e = http.get(p.email_url, headers=hdr)
                emails = e.json() if e.status_code == 200 else None
        ident = p.identity(u.json(), emails)
        if not ident.get("username"):
            raise OAuthError("provider returned no username")
        ident["provider"] = p.name
        return ident
