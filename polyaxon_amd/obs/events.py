"""Event bus = the reference's event_manager + auditor + activitylogs + notifier + tracker + stats.

Reference: polyaxon/event_manager/ (typed event catalogue, 116 types, event.py:13-148), auditor/service.py
(one ``record`` fanned out to notifier, tracker and activity logs), notifier/service.py, activitylogs/,
tracker/publish_tracker.py (Segment analytics), stats/ (statsd/datadog counters), action_manager/ (email,
Slack, Discord, Mattermost, HipChat, PagerDuty, generic webhooks).

Here: event types are ``<subject>.<action>`` strings validated against :data:`EVENT_TYPES`;
:class:`Auditor.record` synchronously writes the activity log row and the notification row (for
notifying events) and hands webhook deliveries to a background thread so the scheduler loop never blocks
on the network.  Subscribers (``subscribe(pattern, fn)``) get every matching event in-process (the
websocket/SSE streams and tests use this).
"""
from __future__ import annotations

import fnmatch
import json
import os
import logging
import queue
import threading
import time
import urllib.request
from collections import Counter
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

log = logging.getLogger("polyaxon_amd.events")

SUBJECTS = {
    "experiment": ["created", "updated", "deleted", "viewed", "stopped", "resumed", "restarted", "copied",
                   "bookmarked", "unbookmarked", "new_status", "new_metric", "succeeded", "failed", "done",
                   "resources_viewed", "logs_viewed", "outputs_downloaded", "statuses_viewed", "jobs_viewed",
                   "metrics_viewed", "deleted_triggered", "stopped_triggered", "resumed_triggered",
                   "restarted_triggered", "copied_triggered"],
    "experiment_group": ["created", "updated", "deleted", "viewed", "stopped", "resumed", "bookmarked",
                         "unbookmarked", "new_status", "experiments_viewed", "statuses_viewed", "metrics_viewed",
                         "iteration", "random", "grid", "hyperband", "bo", "asha", "done", "succeeded", "failed",
                         "deleted_triggered", "stopped_triggered", "unit_redispatched"],
    "experiment_job": ["viewed", "resources_viewed", "logs_viewed", "statuses_viewed", "new_status", "failed",
                       "succeeded", "done"],
    "job": ["created", "updated", "started", "started_triggered", "deleted", "deleted_triggered", "viewed",
            "bookmarked", "unbookmarked", "stopped", "stopped_triggered", "restarted", "restarted_triggered",
            "statuses_viewed", "logs_viewed", "new_status", "failed", "succeeded", "done", "outputs_downloaded"],
    "build_job": ["created", "updated", "started", "started_triggered", "deleted", "deleted_triggered", "viewed",
                  "bookmarked", "unbookmarked", "stopped", "stopped_triggered", "statuses_viewed", "logs_viewed",
                  "new_status", "failed", "succeeded", "done"],
    "notebook": ["started", "started_triggered", "stopped", "stopped_triggered", "viewed", "new_status", "failed",
                 "succeeded"],
    "tensorboard": ["started", "started_triggered", "stopped", "stopped_triggered", "viewed", "new_status",
                    "failed", "succeeded"],
    "project": ["created", "updated", "deleted", "viewed", "bookmarked", "unbookmarked", "set_public",
                "set_private", "experiments_viewed", "jobs_viewed", "builds_viewed", "experiment_groups_viewed",
                "tensorboards_viewed", "deleted_triggered"],
    "pipeline": ["created", "started", "succeeded", "failed", "stopped", "done"],
    "operation": ["created", "started", "succeeded", "failed", "upstream_failed", "retrying", "skipped", "stopped"],
    "repo": ["created", "new_commit", "downloaded"],
    "cluster": ["created", "updated", "resources_updated", "node_created", "node_updated", "node_deleted",
                "node_gpu", "node_gpu_unhealthy", "event"],
    "resident_executor": ["started", "stopped", "lost", "yielded"],
    "user": ["registered", "updated", "activated", "deactivated", "deleted", "viewed", "password_changed",
             "logged_in", "logged_out", "sso_logged_in"],
    "superuser": ["role_granted", "role_revoked"],
    "permission": ["project_denied", "repo_denied", "experiment_group_denied", "experiment_denied",
                   "tensorboard_denied", "notebook_denied", "build_job_denied", "experiment_job_denied",
                   "cluster_denied", "user_role_denied"],
    "search": ["created", "deleted"],
    "chart_view": ["created", "deleted"],
    "bookmark": ["created", "deleted"],
    "webhook_action": ["executed"],
    "email_action": ["executed"],
    "admin": ["updated", "deleted"],
}
EVENT_TYPES = frozenset(f"{s}.{a}" for s, acts in SUBJECTS.items() for a in acts)
# events that also create a user-visible notification (reference notifier/service.py event list)
NOTIFY = frozenset(e for e in EVENT_TYPES if e.endswith((".succeeded", ".failed", ".done", ".stopped",
                                                         ".upstream_failed")))


@dataclass
class Event:
    event_type: str
    object_kind: Optional[str] = None
    object_id: Optional[int] = None
    actor: Optional[str] = None
    context: Dict[str, Any] = field(default_factory=dict)
    created_at: float = field(default_factory=time.time)

    @property
    def subject(self) -> str:
        return self.event_type.split(".", 1)[0]

    @property
    def action(self) -> str:
        return self.event_type.split(".", 1)[1]

    def to_dict(self) -> Dict[str, Any]:
        return {"event_type": self.event_type, "object_kind": self.object_kind, "object_id": self.object_id,
                "actor": self.actor, "context": self.context, "created_at": self.created_at}

    def readable(self) -> str:
        who = f"{self.actor} " if self.actor else ""
        obj = f"{self.object_kind} {self.object_id}" if self.object_kind else self.subject
        return f"{who}{self.action.replace('_', ' ')}: {obj}"


class Stats:
    """Counters/timings (reference stats/: noop | statsd | datadog). Always kept in-process; ``statsd_addr``
    also sends them over UDP, as plain statsd lines or, with ``backend="datadog"``, DogStatsD lines carrying
    ``tags`` (reference stats/datadog.py:11-35)."""

    def __init__(self, statsd_addr: Optional[Tuple[str, int]] = None, prefix: str = "polyaxon",
                 backend: str = "statsd", tags: Optional[List[str]] = None):
        self.counters: Counter = Counter()
        self.timings: Dict[str, List[float]] = {}
        self.prefix = prefix
        self.backend = backend
        self.tags = list(tags or [])
        self._addr = statsd_addr
        self._sock = None
        if statsd_addr:
            import socket

            self._sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)

    def _line(self, key: str, value: str, kind: str) -> str:
        line = f"{self.prefix}.{key}:{value}|{kind}"
        if self.backend == "datadog" and self.tags:
            line += "|#" + ",".join(self.tags)
        return line

    def incr(self, key: str, value: int = 1) -> None:
        self.counters[key] += value
        self._send(self._line(key, str(value), "c"))

    def timing(self, key: str, ms: float) -> None:
        self.timings.setdefault(key, []).append(ms)
        self._send(self._line(key, f"{ms:.3f}", "ms"))

    def _send(self, payload: str) -> None:
        if self._sock is not None:
            try:
                self._sock.sendto(payload.encode(), self._addr)
            except OSError:
                pass


class WebhookAction:
    """Generic webhook + chat integrations (Slack/Mattermost/Discord payload shapes; PagerDuty events v2)."""

    KINDS = ("webhook", "slack", "mattermost", "discord", "hipchat", "pagerduty")

    def __init__(self, url: str, kind: str = "webhook", method: str = "POST", events: Optional[List[str]] = None,
                 timeout: float = 5.0):
        if kind not in self.KINDS:
            raise ValueError(f"unknown webhook kind {kind}")
        if not url.startswith(("http://", "https://")):
            raise ValueError(f"invalid webhook URL {url}")
        if method.upper() not in ("GET", "POST"):
            raise ValueError(f"unsupported webhook method {method}")
        self.url, self.kind, self.method = url, kind, method.upper()
        self.events = events or ["*"]
        self.timeout = timeout

    def matches(self, event_type: str) -> bool:
        return any(fnmatch.fnmatch(event_type, p) for p in self.events)

    def payload(self, ev: Event) -> Dict[str, Any]:
        text = ev.readable()
        if self.kind in ("slack", "mattermost"):
            return {"text": text, "attachments": [{"fields": [{"title": k, "value": str(v), "short": True}
                                                              for k, v in ev.context.items()]}]}
        if self.kind == "discord":
            return {"content": text}
        if self.kind == "hipchat":
            return {"message": text, "notify": True}
        if self.kind == "pagerduty":
            return {"event_action": "trigger", "payload": {"summary": text, "source": "polyaxon-mi355x",
                                                           "severity": "error" if "failed" in ev.event_type
                                                           else "info", "custom_details": ev.context}}
        return {"subject": ev.event_type, "body": text, "datetime": ev.created_at, "context": ev.context}

    def execute(self, ev: Event) -> bool:
        data = json.dumps(self.payload(ev)).encode()
        req = urllib.request.Request(self.url, data=data if self.method == "POST" else None, method=self.method,
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return 200 <= r.status < 300
        except Exception as e:  # delivery failures never break the platform (reference safe_request)
            log.warning("webhook %s failed: %s", self.url, e)
            return False


class EmailAction:
    """E-mail notification (reference action_manager/actions/email.py): one message per matching event over
    SMTP (optional STARTTLS + login).  Delivery failures are logged, never raised."""

    kind = "email"

    def __init__(self, host: str, to: List[str], port: int = 25, sender: str = "polyaxon@localhost",
                 events: Optional[List[str]] = None, use_tls: bool = False, username: Optional[str] = None,
                 password: Optional[str] = None, timeout: float = 5.0, subject_prefix: str = "[polyaxon]"):
        if not to:
            raise ValueError("email action needs at least one recipient")
        self.host, self.port, self.to, self.sender = host, int(port), list(to), sender
        self.events = events or ["*.succeeded", "*.failed", "*.stopped"]
        self.use_tls, self.username, self.password = use_tls, username, password
        self.timeout, self.subject_prefix = timeout, subject_prefix
        self.url = f"smtp://{host}:{port}"

    def matches(self, event_type: str) -> bool:
        return any(fnmatch.fnmatch(event_type, p) for p in self.events)

    def message(self, ev: Event):
        from email.message import EmailMessage

        msg = EmailMessage()
        msg["Subject"] = f"{self.subject_prefix} {ev.readable()}"
        msg["From"] = self.sender
        msg["To"] = ", ".join(self.to)
        body = [ev.readable(), "", f"event: {ev.event_type}", f"at: {time.ctime(ev.created_at)}"]
        body += [f"{k}: {v}" for k, v in ev.context.items()]
        msg.set_content("\n".join(body))
        return msg

    def execute(self, ev: Event) -> bool:
        import smtplib

        try:
            with smtplib.SMTP(self.host, self.port, timeout=self.timeout) as smtp:
                if self.use_tls:
                    smtp.starttls()
                if self.username:
                    smtp.login(self.username, self.password or "")
                smtp.send_message(self.message(ev))
            return True
        except Exception as e:
            log.warning("email to %s via %s failed: %s", self.to, self.url, e)
            return False


class JsonlTracker:
    """Product-analytics sink (reference tracker/publish_tracker.py sends every event to Segment).  The node
    has no egress, so events are appended as JSON lines to a local file an operator can ship elsewhere."""

    def __init__(self, path: str):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._lock = threading.Lock()

    def __call__(self, ev: Event) -> None:
        line = json.dumps({"event": ev.event_type, "actor": ev.actor, "object_kind": ev.object_kind,
                           "object_id": ev.object_id, "ts": ev.created_at}, default=str)
        with self._lock, open(self.path, "a") as f:
            f.write(line + "\n")


def actions_from_config(cfg: Dict[str, Any]) -> List[Any]:
    """``{"webhooks": [{"url", "kind", "method", "events"}...], "email": {"host", "port", "to", "sender",
    "events", "use_tls", "username", "password"}}`` -> action objects (reference INTEGRATIONS_* settings)."""
    out: List[Any] = []
    for w in cfg.get("webhooks", []) or []:
        out.append(WebhookAction(w["url"], kind=w.get("kind", "webhook"), method=w.get("method", "POST"),
                                 events=w.get("events")))
    em = cfg.get("email")
    if em:
        out.append(EmailAction(em["host"], em["to"] if isinstance(em["to"], list) else [em["to"]],
                               port=em.get("port", 25), sender=em.get("sender", "polyaxon@localhost"),
                               events=em.get("events"), use_tls=bool(em.get("use_tls")),
                               username=em.get("username"), password=em.get("password")))
    return out


def load_notification_config(value: Optional[str]) -> Dict[str, Any]:
    """PLX_NOTIFICATIONS: inline JSON, or a path to a JSON / YAML file."""
    if not value:
        return {}
    value = value.strip()
    if value.startswith("{"):
        return json.loads(value)
    with open(value) as f:
        text = f.read()
    if value.endswith((".yml", ".yaml")):
        import yaml

        return yaml.safe_load(text) or {}
    return json.loads(text)


class Auditor:
    def __init__(self, store=None, stats: Optional[Stats] = None, strict: bool = True):
        self.store = store
        self.stats = stats or Stats()
        self.strict = strict
        self.actions: List[Any] = []
        self._subs: List[Tuple[str, Callable[[Event], None]]] = []
        self._q: "queue.Queue[Tuple[WebhookAction, Event]]" = queue.Queue()
        self._worker: Optional[threading.Thread] = None
        self.delivered: List[Tuple[str, bool]] = []

    @classmethod
    def from_settings(cls, store, settings, root: Optional[str] = None) -> "Auditor":
        """Stats backend, tracker and notification actions from :mod:`polyaxon_amd.conf` settings."""
        backend = settings.get("stats.backend")
        addr = (settings.get("stats.host"), settings.get("stats.port")) if backend in ("statsd", "datadog") else None
        a = cls(store, Stats(addr, prefix=settings.get("stats.prefix"), backend=backend or "statsd",
                             tags=[f"service:{settings.get('service')}", f"env:{settings.get('environment')}"]))
        if settings.get("tracker.backend") == "memory":
            a.tracked = []
            a.subscribe("*", a.tracked.append)
        elif settings.get("tracker.backend") == "jsonl":
            a.subscribe("*", JsonlTracker(os.path.join(root or settings.get("root"), "tracker", "events.jsonl")))
        if settings.get("notifications"):
            a.configure(load_notification_config(settings.get("notifications")))
        return a

    def subscribe(self, pattern: str, fn: Callable[[Event], None]) -> None:
        self._subs.append((pattern, fn))

    def add_action(self, action) -> None:
        self.actions.append(action)

    def configure(self, cfg: Dict[str, Any]) -> None:
        for a in actions_from_config(cfg):
            self.add_action(a)

    def record(self, event_type: str, object_kind: Optional[str] = None, object_id: Optional[int] = None,
               actor: Optional[str] = None, **context) -> Event:
        if self.strict and event_type not in EVENT_TYPES:
            raise ValueError(f"unknown event type {event_type!r}")
        ev = Event(event_type, object_kind, object_id, actor, context)
        self.stats.incr(event_type)
        if self.store is not None:
            self.store.add_activity(event_type, actor, object_kind, object_id, context)
            if event_type in NOTIFY:
                self.store.add_notification(event_type, object_kind, object_id, context, user=actor)
        for pattern, fn in list(self._subs):
            if fnmatch.fnmatch(event_type, pattern):
                try:
                    fn(ev)
                except Exception:  # subscribers must not break the emitter
                    log.exception("event subscriber failed")
        for a in self.actions:
            if a.matches(event_type):
                self._ensure_worker()
                self._q.put((a, ev))
        return ev

    def _ensure_worker(self) -> None:
        if self._worker is None or not self._worker.is_alive():
            self._worker = threading.Thread(target=self._deliver, name="plx-webhooks", daemon=True)
            self._worker.start()

    def _deliver(self) -> None:
        while True:
            a, ev = self._q.get()
            ok = a.execute(ev)
            self.delivered.append((a.url, ok))
            self.stats.incr("email_action.executed" if getattr(a, "kind", "") == "email" else "webhook_action.executed")
            self._q.task_done()

    def flush(self, timeout: float = 10.0) -> None:
        end = time.time() + timeout
        while self._q.unfinished_tasks and time.time() < end:
            time.sleep(0.01)
