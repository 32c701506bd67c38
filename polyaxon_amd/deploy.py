"""Node deployment wizard: preflight checks + generated artifacts for one MI355X node.

Reference: deploy/src/components/{deploy,settings,preview,cli}.tsx and deploy/src/libs/artifacts.ts — a web
form that fills Helm ``values`` (namespace, ingress, initial admin user, NVIDIA lib/bin mounts, persistence
claims for logs/repos/outputs/data, node selectors) and prints the ``helm install`` / ``polyaxon config``
commands.  There is no Kubernetes layer here, so the same decisions become:

* ``settings.yaml`` — the platform settings (:mod:`polyaxon_amd.conf`): API bind/port, node root, GPUs to
  schedule, registration, LDAP/SSO blocks left commented for the operator;
* ``polyaxon-mi355x.service`` — a systemd unit running ``plx server`` with the ROCm environment it needs
  (``HSA_ENABLE_IPC_MODE_LEGACY=0`` for RCCL dmabuf IPC, no ``HIP_VISIBLE_DEVICES`` narrowing unless asked);
* ``plx.env`` — the client side (``PLX_HOST``, ``PLX_TOKEN``), the equivalent of ``polyaxon config set``;
* a preflight report: ``/dev/kfd`` + ``/dev/dri`` access, visible gfx950 agents, free port, free disk under
  the root, RCCL library present, writable root.
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import socket
import sys
import uuid
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional

import yaml


@dataclass
class DeployConfig:
    root: str = "/var/lib/polyaxon-mi355x"
    host: str = "0.0.0.0"
    port: int = 8000
    gpus: Optional[int] = None
    admin_user: str = "root"
    admin_email: str = "root@localhost"
    registration: str = "disabled"
    service_user: str = "polyaxon"
    python: str = sys.executable
    extra_env: Dict[str, str] = field(default_factory=dict)


@dataclass
class Check:
    name: str
    ok: bool
    detail: str
    required: bool = True


def _gfx_agents() -> List[str]:
    """gfx targets of the KFD topology nodes (no HIP call, so this is safe before any GPU init)."""
    out = []
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        try:
            props = dict(line.split(None, 1) for line in open(p).read().splitlines() if " " in line)
        except OSError:
            continue
        ver = int(props.get("gfx_target_version", "0").strip() or 0)
        if ver:
            major, minor, step = ver // 10000, (ver // 100) % 100, ver % 100
            out.append(f"gfx{major}{minor:x}{step:x}")
    return out


def preflight(cfg: DeployConfig) -> List[Check]:
    checks: List[Check] = []
    kfd = os.path.exists("/dev/kfd")
    checks.append(Check("dev_kfd", kfd and os.access("/dev/kfd", os.R_OK | os.W_OK),
                        "/dev/kfd present and accessible" if kfd else "/dev/kfd missing (amdgpu driver not loaded?)"))
    dri = sorted(glob.glob("/dev/dri/renderD*"))
    checks.append(Check("dev_dri", bool(dri), f"{len(dri)} render nodes"))
    agents = _gfx_agents()
    n950 = sum(a == "gfx950" for a in agents)
    checks.append(Check("gfx950_agents", n950 > 0, f"agents: {agents or 'none'}"))
    if cfg.gpus is not None:
        checks.append(Check("gpu_count", n950 >= cfg.gpus, f"requested {cfg.gpus}, visible gfx950 {n950}"))
    rccl = glob.glob("/opt/rocm/lib/librccl.so*")
    checks.append(Check("rccl", bool(rccl), rccl[0] if rccl else "librccl.so not under /opt/rocm/lib"))
    s = socket.socket()
    try:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((cfg.host, cfg.port))
        port_ok, port_detail = True, f"{cfg.host}:{cfg.port} free"
    except OSError as e:
        port_ok, port_detail = False, f"{cfg.host}:{cfg.port} unavailable: {e}"
    finally:
        s.close()
    checks.append(Check("port", port_ok, port_detail))
    probe = cfg.root
    while probe and not os.path.exists(probe):
        probe = os.path.dirname(probe)
    probe = probe or "/"
    free_gb = shutil.disk_usage(probe).free / 2 ** 30
    checks.append(Check("disk", free_gb >= 50, f"{free_gb:.0f} GiB free under {probe} (want >= 50 for outputs)",
                        required=False))
    checks.append(Check("root_writable", os.access(probe, os.W_OK), f"{probe} writable"))
    checks.append(Check("python", sys.version_info >= (3, 9), sys.version.split()[0]))
    return checks


def settings_yaml(cfg: DeployConfig, admin_token: str) -> str:
    data: Dict[str, Any] = {
        "service": "monolith",
        "root": cfg.root,
        "api": {"host": cfg.host, "port": cfg.port, "require_auth": True, "admin_token": admin_token},
        "scheduler": {"reconcile_interval_s": 5.0},
        "auth": {"registration": cfg.registration},
    }
    if cfg.gpus is not None:
        data["scheduler"]["gpus"] = cfg.gpus
    body = yaml.safe_dump(data, sort_keys=False)
    return ("# polyaxon-mi355x node settings (see `plx settings` for every key and its origin)\n" + body +
            "# LDAP (uncomment):\n"
            "# auth:\n#   ldap: {enabled: true, server_uri: ldap://ldap:389, "
            "user_dn_template: 'uid={username},ou=people,dc=example,dc=org'}\n"
            "# SSO (uncomment one):\n"
            "#   github: {client_id: ..., client_secret: ...}\n")


def systemd_unit(cfg: DeployConfig, settings_path: str) -> str:
    env = {"PLX_SETTINGS_FILE": settings_path, "HSA_ENABLE_IPC_MODE_LEGACY": "0", "PYTHONUNBUFFERED": "1"}
    env.update(cfg.extra_env)
    env_lines = "\n".join(f"Environment={k}={v}" for k, v in env.items())
    return f"""[Unit]
Description=polyaxon-mi355x scheduler + REST API
After=network-online.target

[Service]
Type=simple
User={cfg.service_user}
SupplementaryGroups=video render
{env_lines}
ExecStart={cfg.python} -m polyaxon_amd.cli server --host {cfg.host} --port {cfg.port}
Restart=on-failure
RestartSec=5
LimitNOFILE=1048576
LimitMEMLOCK=infinity

[Install]
WantedBy=multi-user.target
"""


def client_env(cfg: DeployConfig, admin_token: str) -> str:
    host = "127.0.0.1" if cfg.host in ("0.0.0.0", "::") else cfg.host
    return f"PLX_HOST=http://{host}:{cfg.port}\nPLX_TOKEN={admin_token}\n"


def generate(cfg: DeployConfig, out_dir: str, admin_token: Optional[str] = None) -> Dict[str, Any]:
    os.makedirs(out_dir, exist_ok=True)
    token = admin_token or uuid.uuid4().hex
    settings_path = os.path.join(out_dir, "settings.yaml")
    files = {
        "settings.yaml": settings_yaml(cfg, token),
        "polyaxon-mi355x.service": systemd_unit(cfg, os.path.abspath(settings_path)),
        "plx.env": client_env(cfg, token),
        "deploy.json": json.dumps(asdict(cfg), indent=2) + "\n",
    }
    for name, text in files.items():
        path = os.path.join(out_dir, name)
        with open(path, "w") as f:
            f.write(text)
        if name in ("settings.yaml", "plx.env"):
            os.chmod(path, 0o600)  # both hold the admin token
    return {"files": sorted(files), "out_dir": out_dir,
            "next": [f"sudo cp {out_dir}/polyaxon-mi355x.service /etc/systemd/system/",
                     "sudo systemctl daemon-reload && sudo systemctl enable --now polyaxon-mi355x",
                     f"set -a; . {out_dir}/plx.env; set +a; plx whoami"]}
