"""Notification actions (reference action_manager/ + notifier/): webhooks (generic / Slack / PagerDuty payloads)
and e-mail, delivered asynchronously by the auditor, configured from PLX_NOTIFICATIONS. Local HTTP and SMTP
servers stand in for the external services (reference tests patch safe_request / send_mass_template_mail)."""
import json
import time
import socketserver
import sys
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

from polyaxon_amd.obs.events import Auditor, EmailAction, WebhookAction, actions_from_config, load_notification_config
from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow


def _http_sink():
    got = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):
            n = int(self.headers.get("Content-Length", 0))
            got.append((self.path, json.loads(self.rfile.read(n) or b"{}")))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, got


def _smtp_sink():
    """Minimal SMTP server: records (mail from, rcpt to, data) per message."""
    got = []

    class S(socketserver.StreamRequestHandler):
        def handle(self):
            w = lambda line: self.wfile.write((line + "\r\n").encode())  # noqa: E731
            w("220 plx-test ESMTP")
            frm, rcpt = None, []
            while True:
                line = self.rfile.readline().decode(errors="replace").rstrip("\r\n")
                if not line:
                    return
                cmd = line.upper()
                if cmd.startswith(("EHLO", "HELO")):
                    w("250 plx-test")
                elif cmd.startswith("MAIL FROM"):
                    frm = line.split(":", 1)[1].strip()
                    w("250 OK")
                elif cmd.startswith("RCPT TO"):
                    rcpt.append(line.split(":", 1)[1].strip())
                    w("250 OK")
                elif cmd == "DATA":
                    w("354 go ahead")
                    data = []
                    while True:
                        d = self.rfile.readline().decode(errors="replace")
                        if d.rstrip("\r\n") == ".":
                            break
                        data.append(d)
                    got.append((frm, rcpt, "".join(data)))
                    w("250 queued")
                elif cmd == "QUIT":
                    w("221 bye")
                    return
                else:
                    w("250 OK")

    srv = socketserver.ThreadingTCPServer(("127.0.0.1", 0), S)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, got


def test_webhook_payload_shapes_and_delivery():
    srv, got = _http_sink()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}"
        aud = Auditor()
        aud.add_action(WebhookAction(url + "/generic", events=["experiment.*"]))
        aud.add_action(WebhookAction(url + "/slack", kind="slack", events=["*.failed"]))
        aud.add_action(WebhookAction(url + "/pd", kind="pagerduty", events=["experiment.failed"]))
        aud.record("experiment.succeeded", "experiment", 1, "root", loss=0.1)
        aud.record("experiment.failed", "experiment", 2, "root")
        aud.record("project.created", "project", 3, "root")  # matches nothing
        aud.flush()
        paths = sorted(p for p, _ in got)
        assert paths == ["/generic", "/generic", "/pd", "/slack"]
        slack = [b for p, b in got if p == "/slack"][0]
        assert "failed" in slack["text"]
        pd = [b for p, b in got if p == "/pd"][0]
        assert pd["event_action"] == "trigger" and pd["payload"]["severity"] == "error"
        assert all(ok for _, ok in aud.delivered)
    finally:
        srv.shutdown()


def test_email_action_delivers_over_smtp():
    srv, got = _smtp_sink()
    try:
        aud = Auditor()
        aud.add_action(EmailAction("127.0.0.1", ["ops@example.com"], port=srv.server_address[1],
                                   sender="plx@example.com"))
        aud.record("experiment_group.succeeded", "experiment_group", 7, "root", best="lr=0.1")
        aud.record("experiment.new_metric", "experiment", 1, "root")  # not in the default e-mail events
        aud.flush()
        assert len(got) == 1
        frm, rcpt, data = got[0]
        assert "plx@example.com" in frm and any("ops@example.com" in r for r in rcpt)
        assert "Subject: [polyaxon] root succeeded: experiment_group 7" in data and "best: lr=0.1" in data
        assert aud.stats.counters["email_action.executed"] == 1
    finally:
        srv.shutdown()


def test_failed_delivery_is_logged_not_raised():
    aud = Auditor()
    aud.add_action(EmailAction("127.0.0.1", ["x@y"], port=1))  # nothing listens on port 1
    aud.record("experiment.failed", "experiment", 1)
    aud.flush()
    assert aud.delivered == [("smtp://127.0.0.1:1", False)]


def test_notifications_from_env_config(tmp_path, monkeypatch):
    srv, got = _http_sink()
    try:
        cfg = {"webhooks": [{"url": f"http://127.0.0.1:{srv.server_address[1]}/hook", "events": ["experiment.succeeded"]}],
               "email": {"host": "127.0.0.1", "port": 1, "to": "a@b"}}
        assert [type(a).__name__ for a in actions_from_config(cfg)] == ["WebhookAction", "EmailAction"]
        path = tmp_path / "notify.yaml"
        path.write_text("webhooks:\n  - url: http://127.0.0.1:9/x\n    kind: discord\n")
        assert load_notification_config(str(path))["webhooks"][0]["kind"] == "discord"
        monkeypatch.setenv("PLX_NOTIFICATIONS", json.dumps({"webhooks": cfg["webhooks"]}))
        flow = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0)])).start()
        try:
            x = flow.submit({"version": 1, "kind": "experiment", "run": {"cmd": f"{sys.executable} -c 'pass'"}})
            assert flow.wait("experiment", x["id"], timeout=30) == "succeeded"
            # the scheduler records the event right after the status it waits on: flush until it has arrived
            deadline = time.monotonic() + 10
            while not got and time.monotonic() < deadline:
                flow.auditor.flush()
                time.sleep(0.05)
            assert [p for p, _ in got] == ["/hook"] and got[0][1]["subject"] == "experiment.succeeded"
        finally:
            flow.shutdown()
    finally:
        srv.shutdown()
