"""Event catalogue and auditor fan-out, one case per event type.

Mirrors the reference's tests/test_auditor (every event type is recorded by the tracker, the notifier and
the activity logs: auditor/service.py:22-44) and tests/test_event_manager (attribute extraction and
serialisation, event_manager/event.py:13-148)."""
import json

import pytest

from polyaxon_amd.obs.events import EVENT_TYPES, NOTIFY, SUBJECTS, Auditor, Event, JsonlTracker, Stats
from polyaxon_amd.store import Store


@pytest.fixture(scope="module")
def store():
    return Store(":memory:")


def test_catalogue_shape():
    assert len(EVENT_TYPES) == sum(len(v) for v in SUBJECTS.values())  # no duplicate actions per subject
    assert len(EVENT_TYPES) >= 116  # the reference catalogue has 116 event types
    for e in EVENT_TYPES:
        subject, action = e.split(".", 1)
        assert subject in SUBJECTS and action
    # notifications exist exactly for terminal outcomes
    assert "experiment.succeeded" in NOTIFY and "experiment.failed" in NOTIFY
    assert "operation.upstream_failed" in NOTIFY
    assert "experiment.created" not in NOTIFY and "user.logged_in" not in NOTIFY


@pytest.mark.parametrize("event_type", sorted(EVENT_TYPES))
def test_every_event_fans_out(store, event_type):
    seen = []
    a = Auditor(store, Stats())
    a.subscribe("*", seen.append)
    subject_seen = []
    a.subscribe(event_type.split(".")[0] + ".*", subject_seen.append)
    ev = a.record(event_type, "experiment", 42, "alice", answer=42)
    # tracker (subscribers), stats, activity log, notifier
    assert seen == [ev] and subject_seen == [ev]
    assert a.stats.counters[event_type] == 1
    acts = [r for r in store.activities("experiment", 42) if r["event_type"] == event_type]
    assert acts and acts[0]["actor"] == "alice" and acts[0]["context"] == {"answer": 42}
    notes = [n for n in store.notifications() if n["event_type"] == event_type]
    assert bool(notes) == (event_type in NOTIFY)
    # serialisation round trip
    d = ev.to_dict()
    assert json.loads(json.dumps(d)) == d
    assert d["event_type"] == event_type and d["object_id"] == 42
    assert ev.subject + "." + ev.action == event_type


def test_unknown_event_rejected_unless_lenient():
    with pytest.raises(ValueError):
        Auditor(None).record("experiment.exploded")
    ev = Auditor(None, strict=False).record("experiment.exploded", "experiment", 1)
    assert ev.action == "exploded"


def test_readable_and_subscriber_isolation():
    ev = Event("experiment.new_status", "experiment", 7, "bob")
    assert ev.readable() == "bob new status: experiment 7"
    assert Event("cluster.node_gpu").readable() == "node gpu: cluster"
    a = Auditor(None)
    got = []
    a.subscribe("experiment.*", lambda e: 1 / 0)  # a failing subscriber must not break the emitter
    a.subscribe("experiment.*", got.append)
    a.subscribe("job.*", got.append)
    a.record("experiment.created", "experiment", 1)
    assert [e.event_type for e in got] == ["experiment.created"]


def test_jsonl_tracker_appends_every_event(tmp_path):
    path = tmp_path / "tracker" / "events.jsonl"
    a = Auditor(None)
    a.subscribe("*", JsonlTracker(str(path)))
    for e in ("experiment.created", "experiment_group.hyperband", "user.logged_in"):
        a.record(e, actor="root")
    rows = [json.loads(line) for line in path.read_text().splitlines()]
    assert [r["event"] for r in rows] == ["experiment.created", "experiment_group.hyperband", "user.logged_in"]
    assert all(r["actor"] == "root" for r in rows)
