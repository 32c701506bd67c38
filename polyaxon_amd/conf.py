"""Layered, typed platform settings (reference polyaxon/polyaxon/config_manager.py:22-233 + env_vars/*.json).

The reference reads ``defaults.json`` < ``os.environ`` < ``test.json``/``local.json`` through ``rhea`` with typed
getters (``get_string/get_int/get_boolean/get_list/get_dict``, ``is_optional``, ``is_secret``, ``options``) and
picks a service profile from ``POLYAXON_SERVICE`` (config_settings/__init__.py:18-44).  Here one node-local
process owns the control plane, so the settings are a single declared table of :class:`Option` rows resolved
once in this order (later wins):

1. the declared defaults below;
2. the service profile's overrides (``monolith`` = API + scheduler in one process, ``api``, ``scheduler``,
   ``trial`` = in-trial client);
3. JSON or YAML files (``PLX_SETTINGS_FILE``, or ``<root>/settings.yaml`` when present);
4. environment variables ``PLX_<KEY>`` with dots as underscores (``auth.ldap.server_uri`` ->
   ``PLX_AUTH_LDAP_SERVER_URI``), plus the reference's ``POLYAXON_<KEY>`` spelling;
5. explicit ``overrides=`` (tests, ``plx server --set k=v``).

Every value is parsed and validated against its declared type and choices when the settings are built, so a
bad value fails at start-up with the key and the layer it came from, not later inside a request.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterable, List, Mapping, Optional, Sequence, Tuple


class ConfigError(ValueError):
    pass


_TRUE = {"1", "true", "yes", "on", "y", "t"}
_FALSE = {"0", "false", "no", "off", "n", "f", ""}


def _to_bool(v: Any) -> bool:
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return bool(v)
    s = str(v).strip().lower()
    if s in _TRUE:
        return True
    if s in _FALSE:
        return False
    raise ValueError(f"not a boolean: {v!r}")


def _to_list(v: Any) -> List[Any]:
    if isinstance(v, (list, tuple)):
        return list(v)
    s = str(v).strip()
    if s.startswith("["):
        out = json.loads(s)
        if not isinstance(out, list):
            raise ValueError("not a list")
        return out
    return [p.strip() for p in s.split(",") if p.strip()]


def _to_dict(v: Any) -> Dict[str, Any]:
    if isinstance(v, Mapping):
        return dict(v)
    out = json.loads(str(v))
    if not isinstance(out, dict):
        raise ValueError("not a JSON object")
    return out


_PARSERS: Dict[str, Callable[[Any], Any]] = {
    "str": lambda v: str(v),
    "int": lambda v: v if isinstance(v, int) and not isinstance(v, bool) else int(str(v).strip()),
    "float": lambda v: float(v),
    "bool": _to_bool,
    "list": _to_list,
    "dict": _to_dict,
    "path": lambda v: os.path.expanduser(str(v)),
}


@dataclass(frozen=True)
class Option:
    key: str
    type: str = "str"
    default: Any = None
    help: str = ""
    choices: Optional[Sequence[Any]] = None
    secret: bool = False
    minimum: Optional[float] = None

    @property
    def env_names(self) -> Tuple[str, str]:
        k = self.key.upper().replace(".", "_")
        return f"PLX_{k}", f"POLYAXON_{k}"

    def parse(self, raw: Any, origin: str) -> Any:
        if raw is None:
            return None
        try:
            v = _PARSERS[self.type](raw)
        except (ValueError, TypeError) as e:
            raise ConfigError(f"{self.key}: cannot parse {self._show(raw)} as {self.type} (from {origin}): {e}")
        if self.choices is not None and v not in self.choices:
            raise ConfigError(f"{self.key}: {self._show(v)} not in {list(self.choices)} (from {origin})")
        if self.minimum is not None and v < self.minimum:
            raise ConfigError(f"{self.key}: {v} < minimum {self.minimum} (from {origin})")
        return v

    def _show(self, v: Any) -> str:
        return "'***'" if self.secret else repr(v)


# Declared settings.  Reference sources: config_settings/{core,auth,celery_settings,rest,registration,
# notifications,stats,k8s,spawner}.py and env_vars/defaults.json.
OPTIONS: List[Option] = [
    Option("service", "str", "monolith", "process role (reference POLYAXON_SERVICE)",
           choices=("monolith", "api", "scheduler", "trial")),
    Option("environment", "str", "production", "deployment environment tag", choices=("production", "staging",
                                                                                      "local", "testing")),
    Option("debug", "bool", False, "verbose logging and tracebacks in API errors"),
    Option("root", "path", "~/.polyflow", "node root: store, outputs, logs, repos"),
    # api
    Option("api.host", "str", "127.0.0.1", "REST bind address"),
    Option("api.port", "int", 8000, "REST port", minimum=1),
    Option("api.require_auth", "bool", True, "reject unauthenticated requests"),
    Option("api.throttle_metrics_per_s", "float", 0.0, "per-experiment metric POST rate cap; 0 = unlimited "
           "(reference scope 'high' = 20/s, config_settings/rest.py:20)", minimum=0),
    Option("api.page_size", "int", 100, "default page size", minimum=1),
    Option("api.admin_token", "str", None, "root user's API token", secret=True),
    Option("secret.internal_token", "str", None, "token in-trial services present with X-POLYAXON-INTERNAL",
           secret=True),
    Option("secret.key", "str", None, "HMAC key for ephemeral tokens and OAuth state", secret=True),
    # scheduler
    Option("scheduler.reconcile_interval_s", "float", 5.0, "status reconciliation cron period "
           "(reference 30 s, celery_settings.py:68-71)", minimum=0.05),
    Option("scheduler.heartbeat_timeout_s", "float", 0.0, "fail a trial whose heartbeat is older; 0 = off",
           minimum=0),
    Option("scheduler.max_restarts", "int", 0, "default per-experiment retries (spec max_restarts wins)",
           minimum=0),
    Option("scheduler.build_reuse_s", "float", 6 * 3600.0, "built-environment reuse window "
           "(reference dockerizer_scheduler.py:48-50)", minimum=0),
    Option("build.backend", "str", "native", "build jobs: native environment dir, container image (docker/podman), "
           "or auto (container when an engine is installed)", choices=("native", "container", "auto")),
    Option("build.registry", "str", "localhost:5000", "image registry prefix for container builds "
           "(reference REGISTRY_HOST, docker_images/image_info.py:68-80)"),
    Option("build.push", "bool", False, "push container builds to build.registry"),
    Option("scheduler.gpus", "int", None, "number of devices to schedule on (default: all visible)", minimum=0),
    Option("scheduler.stop_grace_s", "float", 10.0, "SIGTERM -> SIGKILL grace when stopping runs", minimum=0),
    Option("scheduler.numa_bind", "bool", True, "pin each replica to the CPUs local to its GPUs"),
    Option("scheduler.clean_after_s", "float", 0.0, "delete outputs of finished runs older than this; 0 = keep",
           minimum=0),
    Option("scheduler.gang_reserve_s", "float", 30.0, "after a multi-GPU run has waited this long, smaller runs "
           "may not take the devices it needs (no starvation of DP gangs)", minimum=0),
    Option("scheduler.resident_idle_s", "float", 300.0, "shut an idle resident executor down after this long",
           minimum=0),
    Option("scheduler.health_probe", "bool", True, "probe GPU health (amd-smi RAS/ECC, KFD) on every reconcile and "
           "stop placing work on unhealthy devices"),
    # auth (reference config_settings/auth.py, registration.py, sso)
    Option("auth.registration", "str", "disabled", "self-registration workflow",
           choices=("disabled", "superuser_validation", "open")),
    Option("auth.password_min_length", "int", 8, minimum=1),
    Option("auth.token_ttl_s", "float", 0.0, "API token lifetime after login; 0 = no expiry", minimum=0),
    Option("auth.ephemeral_ttl_s", "float", 3 * 3600.0, "ephemeral token TTL (reference 3 h)", minimum=1),
    Option("auth.ldap.enabled", "bool", False),
    Option("auth.ldap.server_uri", "str", None, "ldap://host:port"),
    Option("auth.ldap.bind_dn", "str", None, "service account DN for user search"),
    Option("auth.ldap.bind_password", "str", None, secret=True),
    Option("auth.ldap.user_dn_template", "str", None, "e.g. uid={username},ou=people,dc=example,dc=org"),
    Option("auth.ldap.search_base_dn", "str", None),
    Option("auth.ldap.search_filter", "str", "(uid={username})"),
    Option("auth.ldap.attr_map", "dict", {"email": "mail"}, "user field -> LDAP attribute"),
    Option("auth.ldap.timeout_s", "float", 5.0, minimum=0.01),
    Option("auth.github.client_id", "str", None),
    Option("auth.github.client_secret", "str", None, secret=True),
    Option("auth.github.url", "str", "https://github.com"),
    Option("auth.github.api_url", "str", "https://api.github.com"),
    Option("auth.gitlab.client_id", "str", None),
    Option("auth.gitlab.client_secret", "str", None, secret=True),
    Option("auth.gitlab.url", "str", "https://gitlab.com"),
    Option("auth.bitbucket.client_id", "str", None),
    Option("auth.bitbucket.client_secret", "str", None, secret=True),
    Option("auth.bitbucket.url", "str", "https://bitbucket.org"),
    Option("auth.bitbucket.api_url", "str", "https://api.bitbucket.org"),
    Option("auth.azure.client_id", "str", None),
    Option("auth.azure.client_secret", "str", None, secret=True),
    Option("auth.azure.tenant_id", "str", "common"),
    Option("auth.azure.url", "str", "https://login.microsoftonline.com"),
    Option("auth.azure.api_url", "str", "https://graph.microsoft.com"),
    # observability (reference stats/, tracker/, notifier)
    Option("stats.backend", "str", "noop", choices=("noop", "memory", "statsd", "datadog")),
    Option("stats.host", "str", "127.0.0.1"),
    Option("stats.port", "int", 8125, minimum=1),
    Option("stats.prefix", "str", "polyaxon"),
    Option("tracker.backend", "str", "noop", choices=("noop", "memory", "jsonl")),
    Option("notifications", "str", None, "inline JSON or path to the notifier config"),
    Option("logs.level", "str", "INFO", choices=("DEBUG", "INFO", "WARNING", "ERROR")),
    Option("logs.batch_lines", "int", 50, "log batch size (reference publisher/__init__.py:4-6)", minimum=1),
    Option("logs.batch_s", "float", 2.0, minimum=0.0),
    Option("telemetry.interval_s", "float", 1.0, "resource sampling period", minimum=0.05),
    # names reserved by the API routes (reference libs/blacklist.py)
    Option("blacklist.extra", "list", [], "extra reserved user/project names"),
]

PROFILES: Dict[str, Dict[str, Any]] = {
    "monolith": {},
    "api": {"scheduler.reconcile_interval_s": 30.0},
    "scheduler": {"api.require_auth": True},
    "trial": {"telemetry.interval_s": 5.0, "logs.level": "WARNING"},
}


def _load_file(path: str) -> Dict[str, Any]:
    with open(path) as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml
        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text or "{}")
    if not isinstance(data, dict):
        raise ConfigError(f"{path}: settings file must hold a mapping")
    return _flatten(data)


def _flatten(d: Mapping[str, Any], prefix: str = "") -> Dict[str, Any]:
    """``{"auth": {"ldap": {"enabled": true}}}`` -> ``{"auth.ldap.enabled": true}``; dict-typed options keep
    their value whole."""
    out: Dict[str, Any] = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, Mapping) and key not in _BY_KEY:
            out.update(_flatten(v, key + "."))
        else:
            out[key] = v
    return out


_BY_KEY: Dict[str, Option] = {o.key: o for o in OPTIONS}


@dataclass
class Settings:
    values: Dict[str, Any]
    origins: Dict[str, str] = field(default_factory=dict)

    # ------------------------------------------------------------------ construction
    @classmethod
    def load(cls, env: Optional[Mapping[str, str]] = None, files: Iterable[str] = (),
             overrides: Optional[Mapping[str, Any]] = None, profile: Optional[str] = None,
             strict: bool = True) -> "Settings":
        env = os.environ if env is None else env
        values = {o.key: o.default for o in OPTIONS}
        origins = {o.key: "default" for o in OPTIONS}

        def apply(layer: Mapping[str, Any], origin: str) -> None:
            for k, raw in layer.items():
                opt = _BY_KEY.get(k)
                if opt is None:
                    if strict:
                        raise ConfigError(f"unknown setting {k!r} (from {origin})")
                    continue
                values[k] = opt.parse(raw, origin)
                origins[k] = origin

        env_layer: Dict[str, Any] = {}
        for o in OPTIONS:
            for name in reversed(o.env_names):  # PLX_ wins over POLYAXON_
                if name in env:
                    env_layer[o.key] = env[name]
        svc = profile or env_layer.get("service") or (overrides or {}).get("service") or "monolith"
        if svc not in PROFILES:
            raise ConfigError(f"unknown service profile {svc!r}")
        apply({"service": svc}, "profile")
        apply(PROFILES[svc], f"profile:{svc}")
        file_list = list(files)
        if not file_list and env.get("PLX_SETTINGS_FILE"):
            file_list = [env["PLX_SETTINGS_FILE"]]
        for path in file_list:
            apply(_load_file(path), path)
        if not file_list:
            root = os.path.expanduser(str(env_layer.get("root") or values["root"]))
            default_file = os.path.join(root, "settings.yaml")
            if os.path.isfile(default_file):
                apply(_load_file(default_file), default_file)
        apply(env_layer, "env")
        if overrides:
            apply(dict(overrides), "overrides")
        s = cls(values, origins)
        s.validate()
        return s

    def validate(self) -> None:
        if self.get("auth.ldap.enabled"):
            if not self.get("auth.ldap.server_uri"):
                raise ConfigError("auth.ldap.enabled needs auth.ldap.server_uri")
            if not (self.get("auth.ldap.user_dn_template") or self.get("auth.ldap.search_base_dn")):
                raise ConfigError("auth.ldap needs user_dn_template or search_base_dn")
        for prov in ("github", "gitlab", "bitbucket", "azure"):
            cid, sec = self.get(f"auth.{prov}.client_id"), self.get(f"auth.{prov}.client_secret")
            if bool(cid) != bool(sec):
                raise ConfigError(f"auth.{prov}: client_id and client_secret must be set together")

    # ------------------------------------------------------------------ access
    def get(self, key: str, default: Any = None) -> Any:
        if key not in _BY_KEY:
            raise KeyError(key)
        v = self.values.get(key)
        return default if v is None else v

    def __getitem__(self, key: str) -> Any:
        return self.get(key)

    def section(self, prefix: str) -> Dict[str, Any]:
        p = prefix.rstrip(".") + "."
        return {k[len(p):]: v for k, v in self.values.items() if k.startswith(p)}

    def sso_providers(self) -> List[str]:
        return [p for p in ("github", "gitlab", "bitbucket", "azure") if self.get(f"auth.{p}.client_id")]

    def as_dict(self, redact: bool = True) -> Dict[str, Any]:
        out = {}
        for o in OPTIONS:
            v = self.values.get(o.key)
            out[o.key] = "***" if (redact and o.secret and v) else v
        return out

    def describe(self) -> List[Dict[str, Any]]:
        return [{"key": o.key, "type": o.type, "value": self.as_dict()[o.key], "origin": self.origins.get(o.key),
                 "env": o.env_names[0], "help": o.help} for o in OPTIONS]


_current: Optional[Settings] = None


def settings() -> Settings:
    """Process-wide settings, resolved on first use."""
    global _current
    if _current is None:
        _current = Settings.load()
    return _current


def set_settings(s: Optional[Settings]) -> None:
    global _current
    _current = s
