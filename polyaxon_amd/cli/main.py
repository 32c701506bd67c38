"""``plx`` command line (reference polyaxon-cli, docs/templates/polyaxon_cli/commands/*.md).

Two modes, chosen automatically:
* **server mode** — when ``PLX_HOST`` (or ``plx config set host``) points at a running ``plx server``, every
  command is a REST call (token from ``PLX_TOKEN`` / config);
* **local mode** — otherwise the CLI opens the node's store under ``PLX_ROOT`` (default ``~/.polyflow``)
  directly; ``plx run`` then starts an in-process polyflow scheduler and blocks until the submitted run
  finishes (``--detach`` is only meaningful in server mode).

Commands: init, check, run, server, config, version, project, experiment, group, job, build, notebook,
tensorboard, pipeline, cluster, bookmark, search.
"""
from __future__ import annotations

import json
import os
import sys
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Any, Dict, List, Optional

import click
import yaml

from polyaxon_amd import __version__

CONFIG_PATH = os.path.expanduser(os.environ.get("PLX_CONFIG", "~/.polyflow/config.yaml"))


# ------------------------------------------------------------------ config (layered: file < env < flags)
def load_config() -> Dict[str, Any]:
    cfg: Dict[str, Any] = {"root": os.path.expanduser("~/.polyflow"), "user": "root"}
    if os.path.exists(CONFIG_PATH):
        with open(CONFIG_PATH) as f:
            cfg.update(yaml.safe_load(f) or {})
    for key in ("root", "host", "token", "user", "project"):
        env = os.environ.get(f"PLX_{key.upper()}")
        if env:
            cfg[key] = env
    return cfg


def save_config(cfg: Dict[str, Any]) -> None:
    os.makedirs(os.path.dirname(CONFIG_PATH), exist_ok=True)
    with open(CONFIG_PATH, "w") as f:
        yaml.safe_dump(cfg, f)


class Ctx:
    def __init__(self, cfg: Dict[str, Any], project: Optional[str]):
        self.cfg = cfg
        self.user = cfg.get("user", "root")
        proj = project or cfg.get("project") or "default"
        if "/" in proj:
            self.user, proj = proj.split("/", 1)
        self.project = proj
        self.host = cfg.get("host")
        self._store = None

    # REST
    def api(self, method: str, path: str, payload=None, raw: bool = False, body: Optional[bytes] = None):
        url = self.host.rstrip("/") + path
        data = body if body is not None else (json.dumps(payload).encode() if payload is not None else None)
        headers = {"Content-Type": "application/octet-stream" if body is not None else "application/json"}
        if self.cfg.get("token"):
            headers["Authorization"] = f"token {self.cfg['token']}"
        req = urllib.request.Request(url, data=data, method=method, headers=headers)
        try:
            with urllib.request.urlopen(req, timeout=30) as r:
                body = r.read()
        except urllib.error.HTTPError as e:
            raise click.ClickException(f"{e.code}: {e.read().decode(errors='replace')}")
        if raw:
            return body.decode(errors="replace")
        return json.loads(body) if body else None

    # local
    @property
    def store(self):
        if self._store is None:
            from polyaxon_amd.store import Store

            root = os.path.expanduser(self.cfg["root"])
            os.makedirs(root, exist_ok=True)
            self._store = Store(os.path.join(root, "polyaxon.sqlite"))
        return self._store

    def project_id(self) -> int:
        p = self.store.get_project(self.project, self.user)
        if p is None:
            raise click.ClickException(f"project {self.user}/{self.project} not found")
        return p["id"]

    def base(self) -> str:
        return f"/api/v1/{self.user}/{self.project}"


def out(obj, fmt: str = "table", columns: Optional[List[str]] = None) -> None:
    if fmt == "json":
        click.echo(json.dumps(obj, indent=2, default=str))
        return
    rows = obj.get("results", obj) if isinstance(obj, dict) and "results" in obj else obj
    if isinstance(rows, list):
        if not rows:
            click.echo("(none)")
            return
        cols = columns or [c for c in rows[0].keys() if not isinstance(rows[0][c], (dict, list))][:8]
        widths = {c: max(len(c), *(len(_fmt(r.get(c))) for r in rows)) for c in cols}
        click.echo("  ".join(c.upper().ljust(widths[c]) for c in cols))
        for r in rows:
            click.echo("  ".join(_fmt(r.get(c)).ljust(widths[c]) for c in cols))
    elif isinstance(obj, dict):
        for k, v in obj.items():
            click.echo(f"{k}: {json.dumps(v, default=str) if isinstance(v, (dict, list)) else v}")
    else:
        click.echo(str(obj))


def _fmt(v) -> str:
    if isinstance(v, float) and v > 1e9:
        return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(v))
    if isinstance(v, (dict, list)):
        return json.dumps(v, default=str)
    return "" if v is None else str(v)


@click.group()
@click.option("-p", "--project", default=None, help="[user/]project")
@click.option("--json", "as_json", is_flag=True, help="JSON output")
@click.pass_context
def cli(ctx, project, as_json):
    """polyaxon-mi355x: experiments and hyper-parameter search on a MI355X node."""
    ctx.obj = Ctx(load_config(), project)
    ctx.obj.fmt = "json" if as_json else "table"


@cli.command()
def version():
    """Print versions."""
    click.echo(f"plx {__version__} (gfx950 / ROCm)")


@cli.group()
def config():
    """Show or set CLI configuration (~/.polyflow/config.yaml)."""


@config.command("show")
@click.pass_obj
def config_show(c):
    out(c.cfg, c.fmt)


@config.command("set")
@click.argument("key")
@click.argument("value")
def config_set(key, value):
    cfg = load_config()
    cfg[key] = value
    save_config(cfg)
    click.echo(f"{key} = {value}")


@cli.command()
@click.argument("project")
@click.option("--polyaxonfile", is_flag=True, help="also write a template polyaxonfile.yml")
def init(project, polyaxonfile):
    """Initialise the current directory for PROJECT (reference `polyaxon init`)."""
    cfg = load_config()
    cfg["project"] = project
    save_config(cfg)
    if polyaxonfile and not os.path.exists("polyaxonfile.yml"):
        with open("polyaxonfile.yml", "w") as f:
            f.write("version: 1\nkind: experiment\nenvironment:\n  resources:\n    gpu: {requests: 1, limits: 1}\n"
                    "run:\n  cmd: python train.py\n")
    click.echo(f"initialised project {project}")


@cli.command()
@click.option("-f", "--file", "files", multiple=True, required=True, help="Polyaxonfile(s), merged in order")
@click.option("--definition", is_flag=True, help="print the parsed definition")
@click.pass_obj
def check(c, files, definition):
    """Validate polyaxonfiles (reference `polyaxon check`)."""
    from polyaxon_amd.spec import PolyaxonfileError, specification_for

    try:
        spec = specification_for(list(files))
    except PolyaxonfileError as e:
        raise click.ClickException(f"invalid polyaxonfile: {e}")
    click.echo(f"valid {spec.kind}")
    if spec.kind == "group":
        click.echo(f"search algorithm: {spec.search_algorithm}, concurrency: {spec.concurrency}, "
                   f"matrix space: {spec.matrix_space}")
    if definition:
        out(spec.parsed_data, "json")


@cli.command()
@click.option("-f", "--file", "files", multiple=True, required=True)
@click.option("-n", "--name", default=None)
@click.option("--description", default=None)
@click.option("-d", "--detach", is_flag=True, help="server mode: return immediately")
@click.option("--gpus", type=int, default=None, help="local mode: number of HIP devices to manage")
@click.option("-u", "--upload", is_flag=True, help="upload the current directory first and run that snapshot")
@click.pass_obj
def run(c, files, name, description, detach, gpus, upload):
    """Run an experiment, group, job, build or pipeline from polyaxonfile(s)."""
    from polyaxon_amd.spec import PolyaxonfileError, read_raw_spec

    try:
        content = read_raw_spec(list(files))
    except PolyaxonfileError as e:
        raise click.ClickException(str(e))
    cwd = _upload(c)["path"] if upload else os.getcwd()
    if c.host:
        kind = content.get("kind")
        path = {"experiment": "experiments", "group": "groups", "job": "jobs", "build": "builds",
                "pipeline": "pipelines"}.get(kind)
        if path is None:
            raise click.ClickException(f"cannot run kind {kind} remotely")
        res = c.api("POST", f"{c.base()}/{path}", {"content": content, "name": name, "description": description,
                                                     "cwd": cwd})
        click.echo(f"created {kind} {res.get('id')}")
        return
    from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
    from polyaxon_amd.polyflow.scheduler import Polyflow

    alloc = DeviceAllocator([Device(i) for i in range(gpus)]) if gpus is not None else None
    flow = Polyflow(os.path.expanduser(c.cfg["root"]), allocator=alloc).start()
    try:
        res = flow.submit(content, project=c.project, user=c.user, cwd=cwd, name=name, description=description)
        kind, rid = res["kind"], res["id"]
        click.echo(f"created {kind} {rid}; waiting (Ctrl-C to stop)")
        wait_kind = {"pipeline": "pipeline_run"}.get(kind, "group" if kind == "group" else
                                                    ("experiment" if kind == "experiment" else "job"))
        wid = res.get("run_id", rid)
        try:
            st = flow.wait(wait_kind, wid)
        except KeyboardInterrupt:
            st = "stopped"
        click.echo(f"{kind} {rid} {st}")
        if kind == "experiment":
            click.echo(flow.logs("experiment", rid, tail=20))
    finally:
        flow.shutdown()


def _tar_dir(path: str) -> bytes:
    """Tarball of ``path`` minus .git/__pycache__ and the patterns in .polyaxonignore (reference CLI upload)."""
    import fnmatch
    import io
    import tarfile

    ignore = [".git", "__pycache__", "*.pyc", ".polyaxon"]
    pi = os.path.join(path, ".polyaxonignore")
    if os.path.exists(pi):
        with open(pi) as f:
            ignore += [ln.strip().rstrip("/") for ln in f if ln.strip() and not ln.startswith("#")]

    def skip(rel: str) -> bool:
        parts = rel.split(os.sep)
        return any(fnmatch.fnmatch(rel, pat) or any(fnmatch.fnmatch(p, pat) for p in parts) for pat in ignore)

    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tar:
        for root, dirs, files in os.walk(path):
            rel_root = os.path.relpath(root, path)
            dirs[:] = sorted(d for d in dirs if not skip(os.path.normpath(os.path.join(rel_root, d))))
            for fn in sorted(files):
                rel = os.path.normpath(os.path.join(rel_root, fn))
                if not skip(rel):
                    tar.add(os.path.join(root, fn), arcname=rel, recursive=False)
    return buf.getvalue()


def _upload(c) -> Dict[str, Any]:
    data = _tar_dir(os.getcwd())
    if c.host:
        return c.api("POST", f"{c.base()}/repo/upload", body=data)
    from polyaxon_amd.polyflow.paths import Paths
    from polyaxon_amd.polyflow.repos import ProjectRepo

    repo = ProjectRepo(Paths(os.path.expanduser(c.cfg["root"])).repos_root, c.user, c.project)
    return {"commit": repo.upload_tarball(data), "path": repo.path}


@cli.command()
@click.pass_obj
def upload(c):
    """Upload the current directory as the project's code (reference `polyaxon upload`)."""
    res = _upload(c)
    click.echo(f"uploaded {len(res['commit']) and res['commit'][:12]} -> {res['path']}")


@cli.command()
@click.option("--host", default="127.0.0.1")
@click.option("--port", default=8000, type=int)
@click.option("--token", default=None, help="admin token (default: generated and printed)")
@click.option("--gpus", type=int, default=None)
@click.option("--set", "sets", multiple=True, help="settings override key=value (see `plx settings`)")
@click.pass_obj
def server(c, host, port, token, gpus, sets):
    """Run the scheduler + REST API (reference api/ + scheduler services in one process)."""
    import uuid

    import uvicorn

    from polyaxon_amd.api.server import create_app
    from polyaxon_amd.conf import ConfigError, Settings, set_settings
    from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
    from polyaxon_amd.polyflow.scheduler import Polyflow

    try:
        st = Settings.load(overrides=dict(kv.split("=", 1) for kv in sets))
    except ConfigError as e:
        raise click.ClickException(str(e))
    set_settings(st)
    gpus = gpus if gpus is not None else st.get("scheduler.gpus")
    token = token or st.get("api.admin_token") or c.cfg.get("token") or uuid.uuid4().hex
    alloc = DeviceAllocator([Device(i) for i in range(gpus)]) if gpus is not None else None
    import logging

    logging.basicConfig(level=getattr(logging, st.get("logs.level")))
    root = st.get("root") if st.origins.get("root") != "default" else os.path.expanduser(c.cfg["root"])
    flow = Polyflow(root, allocator=alloc, api_host=f"http://{host}:{port}", settings=st).start()
    click.echo(f"plx server on http://{host}:{port}  token={token}")
    try:
        uvicorn.run(create_app(flow, admin_token=token, settings=st, internal_token=st.get("secret.internal_token"),
                               require_auth=st.get("api.require_auth")),
                    host=host, port=port, log_level="warning")
    finally:
        flow.shutdown()


# ------------------------------------------------------------------ project
@cli.group()
def project():
    """Projects."""


@project.command("create")
@click.option("--name", required=True)
@click.option("--description", default="")
@click.pass_obj
def project_create(c, name, description):
    if c.host:
        out(c.api("POST", "/api/v1/projects", {"name": name, "description": description}), c.fmt)
    else:
        out(c.store.create_project(name, c.user, description), c.fmt)


@project.command("list")
@click.pass_obj
def project_list(c):
    rows = c.api("GET", "/api/v1/projects") if c.host else c.store.list_projects()
    out(rows, c.fmt, ["id", "user", "name", "description", "created_at"])


@project.command("get")
@click.pass_obj
def project_get(c):
    out(c.api("GET", c.base()) if c.host else c.store.get_project(c.project, c.user), c.fmt)


@project.command("delete")
@click.pass_obj
def project_delete(c):
    if c.host:
        c.api("DELETE", c.base())
    else:
        c.store.delete_project(c.project_id())
    click.echo("deleted")


@project.command("experiments")
@click.option("-q", "--query", default=None)
@click.option("-s", "--sort", default=None)
@click.option("--independent", is_flag=True)
@click.pass_obj
def project_experiments(c, query, sort, independent):
    if c.host:
        qs = urllib.parse.urlencode({k: v for k, v in (("query", query), ("sort", sort),
                                                       ("independent", "true" if independent else None)) if v})
        rows = c.api("GET", f"{c.base()}/experiments?{qs}")
    else:
        rows = c.store.list_experiments(project_id=c.project_id(), query=query, sort=sort, independent=independent)
    out(rows, c.fmt, ["id", "name", "status", "group_id", "last_metric", "declarations", "created_at"])


@project.command("groups")
@click.pass_obj
def project_groups(c):
    rows = c.api("GET", f"{c.base()}/groups") if c.host else c.store.list_groups(c.project_id())
    out(rows, c.fmt, ["id", "name", "status", "search_algorithm", "concurrency", "created_at"])


# ------------------------------------------------------------------ experiment
@cli.group()
@click.option("-xp", "--experiment", "xid", type=int, required=True)
@click.pass_obj
def experiment(c, xid):
    """Experiment commands."""
    c.xid = xid


@experiment.command("get")
@click.option("-j", "--job", "jid", type=int, default=None)
@click.pass_obj
def xp_get(c, jid):
    if jid:
        res = c.api("GET", f"{c.base()}/experiments/{c.xid}/jobs/{jid}") if c.host else c.store.get(
            "experiment_jobs", jid)
    else:
        res = c.api("GET", f"{c.base()}/experiments/{c.xid}") if c.host else c.store.get_experiment(c.xid)
    out(res, c.fmt)


@experiment.command("statuses")
@click.option("-j", "--job", "jid", type=int, default=None)
@click.pass_obj
def xp_statuses(c, jid):
    if c.host:
        path = f"/jobs/{jid}/statuses" if jid else "/statuses"
        rows = c.api("GET", f"{c.base()}/experiments/{c.xid}{path}")
    else:
        rows = c.store.experiment_job_statuses(jid) if jid else c.store.experiment_statuses(c.xid)
    out(rows, c.fmt, ["id", "status", "message", "created_at"])


@experiment.command("metrics")
@click.pass_obj
def xp_metrics(c):
    rows = c.api("GET", f"{c.base()}/experiments/{c.xid}/metrics") if c.host else c.store.get_metrics(c.xid)
    out(rows, c.fmt, ["id", "step", "values", "created_at"])


@experiment.command("jobs")
@click.pass_obj
def xp_jobs(c):
    rows = c.api("GET", f"{c.base()}/experiments/{c.xid}/jobs") if c.host else c.store.experiment_jobs(c.xid)
    out(rows, c.fmt, ["id", "role", "idx", "status", "devices", "pid", "exit_code"])


@experiment.command("logs")
@click.option("--tail", type=int, default=None)
@click.pass_obj
def xp_logs(c, tail):
    if c.host:
        click.echo(c.api("GET", f"{c.base()}/experiments/{c.xid}/logs" + (f"?tail={tail}" if tail else ""), raw=True))
        return
    from polyaxon_amd.polyflow.paths import Paths

    x = c.store.get_experiment(c.xid)
    for j in c.store.experiment_jobs(c.xid):
        text = Paths.read_log(os.path.join(x["logs_path"], f"{j['role']}.{j['idx']}.log"), tail)
        for line in text.splitlines():
            click.echo(f"{j['role']}.{j['idx']} -- {line}")


@experiment.command("outputs")
@click.pass_obj
def xp_outputs(c):
    if c.host:
        out(c.api("GET", f"{c.base()}/experiments/{c.xid}/outputs"), c.fmt)
    else:
        click.echo(c.store.get_experiment(c.xid)["outputs_path"])


@experiment.command("update")
@click.option("--name", default=None)
@click.option("--description", default=None)
@click.option("--tags", default=None, help="comma separated")
@click.pass_obj
def xp_update(c, name, description, tags):
    vals = {k: v for k, v in (("name", name), ("description", description)) if v is not None}
    if tags is not None:
        vals["tags"] = [t.strip() for t in tags.split(",") if t.strip()]
    if c.host:
        out(c.api("PATCH", f"{c.base()}/experiments/{c.xid}", vals), c.fmt)
    else:
        c.store.update_experiment(c.xid, **vals)
        out(c.store.get_experiment(c.xid), c.fmt)


@experiment.command("delete")
@click.pass_obj
def xp_delete(c):
    if c.host:
        c.api("DELETE", f"{c.base()}/experiments/{c.xid}")
    else:
        c.store.delete_experiment(c.xid)
    click.echo("deleted")


for _action in ("stop", "restart", "resume", "copy"):
    def _mk(action=_action):
        @experiment.command(action)
        @click.pass_obj
        def cmd(c):
            if not c.host:
                raise click.ClickException(f"`experiment {action}` needs a running `plx server` (set PLX_HOST)")
            out(c.api("POST", f"{c.base()}/experiments/{c.xid}/{action}", {}), c.fmt)
        cmd.__doc__ = f"{action.capitalize()} the experiment."
    _mk()


@experiment.command("bookmark")
@click.pass_obj
def xp_bookmark(c):
    if c.host:
        c.api("POST", f"{c.base()}/experiments/{c.xid}/bookmark")
    else:
        c.store.set_bookmark(c.user, "experiment", c.xid, True)
    click.echo("bookmarked")


@experiment.command("resources")
@click.pass_obj
def xp_resources(c):
    if not c.host:
        raise click.ClickException("resources need a running `plx server`")
    click.echo(c.api("GET", f"/streams/v1/{c.user}/{c.project}/experiments/{c.xid}/resources", raw=True)[:4000])


# ------------------------------------------------------------------ group
@cli.group()
@click.option("-g", "--group", "gid", type=int, required=True)
@click.pass_obj
def group(c, gid):
    """Experiment group commands."""
    c.gid = gid


@group.command("get")
@click.pass_obj
def group_get(c):
    out(c.api("GET", f"{c.base()}/groups/{c.gid}") if c.host else c.store.get_group(c.gid), c.fmt)


@group.command("experiments")
@click.option("-q", "--query", default=None)
@click.option("-s", "--sort", default=None)
@click.pass_obj
def group_experiments(c, query, sort):
    if c.host:
        qs = urllib.parse.urlencode({k: v for k, v in (("query", query), ("sort", sort)) if v})
        rows = c.api("GET", f"{c.base()}/groups/{c.gid}/experiments?{qs}")
    else:
        rows = c.store.list_experiments(group_id=c.gid, query=query, sort=sort)
    out(rows, c.fmt, ["id", "status", "declarations", "last_metric", "cloning_strategy", "original_experiment_id"])


@group.command("statuses")
@click.pass_obj
def group_statuses(c):
    rows = c.api("GET", f"{c.base()}/groups/{c.gid}/statuses") if c.host else c.store.group_statuses(c.gid)
    out(rows, c.fmt, ["id", "status", "message", "created_at"])


@group.command("stop")
@click.option("--pending", is_flag=True, help="only stop pending experiments")
@click.pass_obj
def group_stop(c, pending):
    if not c.host:
        raise click.ClickException("`group stop` needs a running `plx server`")
    c.api("POST", f"{c.base()}/groups/{c.gid}/stop", {"pending": pending})
    click.echo("stopping")


# ------------------------------------------------------------------ jobs / builds / plugins
for _kind, _plural in (("job", "jobs"), ("build", "builds")):
    def _mk_kind(kind=_kind, plural=_plural):
        @cli.group(kind)
        @click.option("-j", f"--{kind}", "jid", type=int, required=True)
        @click.pass_obj
        def grp(c, jid):
            c.jid = jid
        grp.__doc__ = f"{kind.capitalize()} commands."

        @grp.command("get")
        @click.pass_obj
        def get(c):
            out(c.api("GET", f"{c.base()}/{plural}/{c.jid}") if c.host else c.store.get_job(c.jid), c.fmt)

        @grp.command("statuses")
        @click.pass_obj
        def statuses(c):
            rows = c.api("GET", f"{c.base()}/{plural}/{c.jid}/statuses") if c.host else c.store.job_statuses(c.jid)
            out(rows, c.fmt, ["id", "status", "message", "created_at"])

        @grp.command("logs")
        @click.pass_obj
        def logs(c):
            if c.host:
                click.echo(c.api("GET", f"{c.base()}/{plural}/{c.jid}/logs", raw=True))
            else:
                from polyaxon_amd.polyflow.paths import Paths

                click.echo(Paths.read_log(os.path.join(c.store.get_job(c.jid)["logs_path"], "master.0.log")))

        @grp.command("stop")
        @click.pass_obj
        def stop(c):
            if not c.host:
                raise click.ClickException("needs a running `plx server`")
            out(c.api("POST", f"{c.base()}/{plural}/{c.jid}/stop"), c.fmt)
    _mk_kind()


for _plugin in ("notebook", "tensorboard"):
    def _mk_plugin(plugin=_plugin):
        @cli.group(plugin)
        def grp():
            pass
        grp.__doc__ = f"{plugin.capitalize()} plugin (start/stop)."

        @grp.command("start")
        @click.option("-f", "--file", "files", multiple=True)
        @click.pass_obj
        def start(c, files):
            if not c.host:
                raise click.ClickException("needs a running `plx server`")
            content = None
            if files:
                from polyaxon_amd.spec import read_raw_spec

                content = read_raw_spec(list(files))
            out(c.api("POST", f"{c.base()}/{plugin}/start", {"content": content}), c.fmt)

        @grp.command("stop")
        @click.pass_obj
        def stop(c):
            if not c.host:
                raise click.ClickException("needs a running `plx server`")
            out(c.api("POST", f"{c.base()}/{plugin}/stop"), c.fmt)
    _mk_plugin()


@cli.command()
@click.pass_obj
def whoami(c):
    """Show the authenticated user (server mode) or the configured local user."""
    if c.host:
        out(c.api("GET", "/api/v1/users"), c.fmt)
    else:
        out({"username": c.user, "mode": "local", "root": c.cfg["root"]}, c.fmt)


@cli.group()
def user():
    """Users (reference `createuser` management command)."""


@user.command("create")
@click.argument("username")
@click.option("--email", default="")
@click.option("--superuser", is_flag=True)
@click.pass_obj
def user_create(c, username, email, superuser):
    if c.host:
        u = c.api("POST", "/api/v1/users", {"username": username, "email": email, "is_superuser": superuser})
    else:
        if c.store.get_user(username):
            raise click.ClickException(f"user {username} exists")
        u = c.store.create_user(username, email, superuser)
    click.echo(f"created user {u['username']} token={u['token']}")


@user.command("password")
@click.argument("username")
@click.option("--password", prompt=True, hide_input=True, confirmation_prompt=True)
@click.pass_obj
def user_password(c, username, password):
    """Set a user's password (superuser; server mode)."""
    _need_host(c, "user password")
    c.api("POST", f"/api/v1/users/{username}/password", {"password": password})
    click.echo("password set")


@user.command("activate")
@click.argument("username")
@click.pass_obj
def user_activate(c, username):
    """Validate a pending registration (reference superuser-validation workflow)."""
    _need_host(c, "user activate")
    c.api("POST", f"/api/v1/users/{username}/activate", {})
    click.echo(f"activated {username}")


@user.command("pending")
@click.pass_obj
def user_pending(c):
    _need_host(c, "user pending")
    out(c.api("GET", "/api/v1/users/pending")["results"], c.fmt)


def _need_host(c, what: str) -> None:
    if not c.host:
        raise click.ClickException(f"`{what}` needs a running `plx server` (set PLX_HOST)")


@cli.command()
@click.option("--username", "-u", prompt=True)
@click.option("--password", "-p", prompt=True, hide_input=True)
@click.pass_obj
def login(c, username, password):
    """Log in (local password or LDAP) and store the API token in the CLI config."""
    _need_host(c, "login")
    res = c.api("POST", "/api/v1/users/token", {"username": username, "password": password})
    cfg = load_config()
    cfg.update({"token": res["token"], "user": res["username"], "host": c.host})
    save_config(cfg)
    click.echo(f"logged in as {res['username']}")


@cli.command()
@click.pass_obj
def logout(c):
    """Invalidate the stored token."""
    if c.host and c.cfg.get("token"):
        c.api("POST", "/api/v1/users/logout", {})
    cfg = load_config()
    cfg.pop("token", None)
    save_config(cfg)
    click.echo("logged out")


@cli.command()
@click.option("--username", "-u", prompt=True)
@click.option("--email", "-e", default="")
@click.option("--password", "-p", prompt=True, hide_input=True, confirmation_prompt=True)
@click.pass_obj
def register(c, username, email, password):
    """Self-register (when the server allows it)."""
    _need_host(c, "register")
    res = c.api("POST", "/api/v1/users/register", {"username": username, "email": email, "password": password})
    click.echo("registered; " + ("token=" + res["token"] if res.get("token") else "awaiting activation"))


@cli.command("settings")
@click.option("--set", "sets", multiple=True, help="key=value override to validate")
@click.pass_obj
def settings_show(c, sets):
    """Show the resolved platform settings with each value's origin (secrets redacted)."""
    from polyaxon_amd.conf import ConfigError, Settings

    try:
        st = Settings.load(overrides=dict(kv.split("=", 1) for kv in sets))
    except ConfigError as e:
        raise click.ClickException(str(e))
    rows = st.describe()
    if c.fmt == "json":
        out(rows, "json")
    else:
        out(rows, "table", ["key", "value", "origin", "env"])


@cli.group()
def deploy():
    """Node deployment wizard (reference deploy/ web wizard -> Helm values)."""


def _deploy_cfg(root, host, port, gpus, registration, service_user):
    from polyaxon_amd.deploy import DeployConfig

    return DeployConfig(root=root, host=host, port=port, gpus=gpus, registration=registration,
                        service_user=service_user)


_deploy_opts = [
    click.option("--root", default="/var/lib/polyaxon-mi355x"),
    click.option("--host", default="0.0.0.0"),
    click.option("--port", default=8000, type=int),
    click.option("--gpus", default=None, type=int),
    click.option("--registration", default="disabled",
                 type=click.Choice(["disabled", "superuser_validation", "open"])),
    click.option("--service-user", default="polyaxon"),
]


def _with_deploy_opts(f):
    for o in reversed(_deploy_opts):
        f = o(f)
    return f


@deploy.command("check")
@_with_deploy_opts
@click.pass_obj
def deploy_check(c, root, host, port, gpus, registration, service_user):
    """Preflight: /dev/kfd, gfx950 agents, RCCL, port, disk, writable root."""
    from dataclasses import asdict

    from polyaxon_amd.deploy import preflight

    checks = preflight(_deploy_cfg(root, host, port, gpus, registration, service_user))
    out([asdict(ch) for ch in checks], c.fmt, ["name", "ok", "required", "detail"])
    if any(not ch.ok and ch.required for ch in checks):
        raise click.ClickException("preflight failed")


@deploy.command("generate")
@_with_deploy_opts
@click.option("--out", "out_dir", default="./plx-deploy")
@click.pass_obj
def deploy_generate(c, root, host, port, gpus, registration, service_user, out_dir):
    """Write settings.yaml, a systemd unit and the client env for this node."""
    from polyaxon_amd.deploy import generate

    out(generate(_deploy_cfg(root, host, port, gpus, registration, service_user), out_dir), "json")


@cli.group()
def admin():
    """Management commands (reference commands/management/commands/*.py)."""


@admin.command("clean")
@click.argument("what", type=click.Choice(["stale", "experiments", "groups", "jobs", "outputs"]))
@click.option("--older-than", default="7d", help="outputs: age cutoff, e.g. 3600s, 12h, 7d")
@click.option("--dry-run", is_flag=True)
@click.option("--force", is_flag=True, help="clean even though a scheduler looks alive")
@click.pass_obj
def admin_clean(c, what, older_than, dry_run, force):
    """Stop runs the store still calls running (after a crash), or delete old outputs."""
    from polyaxon_amd.polyflow.cleaning import clean_outputs, clean_stale, scheduler_alive

    if c.host:
        raise click.ClickException("`admin clean` runs against the node's store: unset PLX_HOST")
    if what != "outputs" and not force and scheduler_alive(os.path.expanduser(c.cfg["root"])):
        raise click.ClickException("a scheduler is running on this root; its runs are live (use --force)")
    if what == "outputs":
        mult = {"s": 1, "m": 60, "h": 3600, "d": 86400}
        unit = older_than[-1] if older_than[-1] in mult else "s"
        secs = float(older_than.rstrip("smhd")) * mult[unit]
        paths = clean_outputs(c.store, secs, dry_run=dry_run)
        out({"deleted": paths, "dry_run": dry_run}, "json")
        return
    kinds = ("experiments", "groups", "jobs") if what == "stale" else (what,)
    out(clean_stale(c.store, kinds=kinds), "json")


@cli.group()
def cluster():
    """Cluster (node + HIP devices)."""


@cluster.command("get")
@click.pass_obj
def cluster_get(c):
    if c.host:
        out(c.api("GET", "/api/v1/cluster"), "json")
    else:
        from polyaxon_amd.obs.telemetry import gpu_stats

        out({"nodes": c.store.nodes(), "gpus": gpu_stats()}, "json")


def main(argv=None) -> int:
    try:
        cli.main(args=argv, prog_name="plx", standalone_mode=False)
    except click.ClickException as e:
        e.show()
        return 1
    except click.exceptions.Abort:
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
