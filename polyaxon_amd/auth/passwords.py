"""Password hashing and reserved names.

Reference: Django's PBKDF2 password hasher behind ``auth_views.LoginView`` (api/users/urls.py) and
``libs/blacklist.py`` (names that would collide with API/dashboard routes).  Hashes are stored as
``pbkdf2_sha256$<iterations>$<salt>$<b64 digest>`` so the iteration count can be raised later without
invalidating stored hashes.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import re
from typing import Iterable

ITERATIONS = 200_000

RESERVED_NAMES = frozenset({
    "user", "users", "admin", "experiment", "experiments", "experiment_group", "experimentgroup", "group",
    "groups", "project", "projects", "api", "polyaxon", "plx", "dashboard", "index", "log", "logs", "metric",
    "metrics", "public", "version", "versions", "support", "repo", "cluster", "event", "events", "manage",
    "login", "logout", "account", "register", "oauth", "sso", "token", "static", "_static", "status",
    "statuses", "streams", "searches", "bookmarks", "activitylogs", "notifications", "nodes", "jobs", "builds",
    "notebook", "tensorboard", "pipelines", "help", "doc", "docs", "404", "500", "ui", "_health", "_status",
    "internal", "root_",
})

_NAME = re.compile(r"^[A-Za-z0-9][A-Za-z0-9_.-]{0,127}$")


def validate_name(name: str, extra_reserved: Iterable[str] = ()) -> str:
    """Reject empty, malformed or reserved user/project names (reference libs/blacklist.py:1-60)."""
    if not name or not _NAME.match(name):
        raise ValueError(f"invalid name {name!r}: use letters, digits, '_', '-', '.'")
    low = name.lower()
    if low in RESERVED_NAMES or low in {e.lower() for e in extra_reserved}:
        raise ValueError(f"name {name!r} is reserved")
    return name


def hash_password(password: str, iterations: int = ITERATIONS, salt: str = "") -> str:
    salt = salt or base64.b64encode(os.urandom(12)).decode().rstrip("=")
    dk = hashlib.pbkdf2_hmac("sha256", password.encode(), salt.encode(), iterations)
    return f"pbkdf2_sha256${iterations}${salt}${base64.b64encode(dk).decode()}"


def check_password(password: str, encoded: str) -> bool:
    try:
        algo, it, salt, _ = encoded.split("$", 3)
    except (AttributeError, ValueError):
        return False
    if algo != "pbkdf2_sha256":
        return False
    return hmac.compare_digest(hash_password(password, int(it), salt), encoded)


def check_strength(password: str, min_length: int) -> None:
    if len(password or "") < min_length:
        raise ValueError(f"password must have at least {min_length} characters")
    if password.isdigit():
        raise ValueError("password must not be entirely numeric")
