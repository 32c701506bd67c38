"""Tracking store (SQLite/WAL) and query DSL."""
from polyaxon_amd.store.db import Store, StoreError  # noqa: F401
from polyaxon_amd.store.query import ExperimentQuery, GroupQuery, JobQuery, QueryError  # noqa: F401
