"""Build jobs (the reference's dockerizer): Dockerfile rendering, image naming and the build command.

Reference: ``dockerizer/dockerfile.py:1-40`` (``POLYAXON_DOCKER_TEMPLATE``), ``dockerizer/builder.py:32-294``
(``DockerBuilder``: render, build, push), ``docker_images/image_info.py:60-80`` (``<registry>/<project>_<id>``
tagged with the build uuid), ``scheduler/dockerizer_scheduler.py:29-128`` (create/start a build job, reuse a
build of the same spec from the last 6 h).

On one MI355X node there is no registry or kubelet that needs an image, so two backends exist:

* ``native`` (default): ``build_steps`` run as a process in a cached environment directory
  (``<root>/envs/<spec hash>``); packages go to ``<env>/site`` (``pip --target``) and trials of the same
  build hash get ``PLX_BUILD_DIR`` and that ``site`` on ``PYTHONPATH``.  The rendered Dockerfile is still
  written into the environment directory, so the same build can be reproduced as a container elsewhere.
* ``container``: the rendered Dockerfile is built with ``docker`` or ``podman`` (whichever is on ``PATH``) and
  tagged ``<registry>/<project>_<id>:<hash>``; pushed when ``build.push`` is set.  ``auto`` picks
  ``container`` when an engine is installed and ``native`` otherwise.

The Dockerfile targets a ROCm base: the run-time device contract (``HIP_VISIBLE_DEVICES``, ``/dev/kfd`` and
``/dev/dri`` access) is applied by the scheduler when the replica starts, not baked into the image.
"""
from __future__ import annotations

import os
import shlex
import shutil
from typing import List, Optional, Sequence, Tuple

DEFAULT_WORKDIR = "/code"
DEFAULT_REGISTRY = "localhost:5000"
BACKENDS = ("native", "container", "auto")
ENGINES = ("docker", "podman")


def _env_value(v) -> str:
    s = str(v)
    return json_quote(s) if (not s or any(c.isspace() or c in "\"'\\$" for c in s)) else s


def json_quote(s: str) -> str:
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


def render_dockerfile(image: str, build_steps: Sequence[str] = (), env_vars: Sequence[Sequence[str]] = (),
                      workdir: str = DEFAULT_WORKDIR, context: Optional[str] = None, copy_code: bool = True) -> str:
    """Dockerfile text for a ``build:`` section.  Layer order matches the reference template: base image,
    locale/shell env, user env vars, workdir, dependency manifests found in the build context (copied before
    the steps so an unchanged manifest keeps the step layers cached), the steps, then the code itself."""
    if not image:
        raise ValueError("a build needs a base image")
    lines = [f"FROM {image}", "",
             "ENV LC_ALL=C.UTF-8 LANG=C.UTF-8 LANGUAGE=C.UTF-8",
             "ENV SHELL=/bin/bash"]
    for kv in env_vars or ():
        k, v = kv
        lines.append(f"ENV {k}={_env_value(v)}")
    lines += ["", f"WORKDIR {workdir}"]
    if context:
        for manifest in ("requirements.txt", "setup.py", "pyproject.toml", "environment.yml"):
            if os.path.isfile(os.path.join(context, manifest)):
                lines.append(f"COPY {manifest} {workdir}/")
    for step in build_steps or ():
        lines.append(f"RUN {step}")
    if copy_code:
        lines.append(f"COPY . {workdir}")
    return "\n".join(lines) + "\n"


def image_name(project_name: str, project_id: int, registry: str = DEFAULT_REGISTRY) -> str:
    """``<registry>/<project>_<id>`` (reference ``get_image_name``), lower-cased as image names must be."""
    return f"{registry}/{project_name.lower()}_{project_id}"


def image_info(project_name: str, project_id: int, tag: str, registry: str = DEFAULT_REGISTRY) -> Tuple[str, str]:
    return image_name(project_name, project_id, registry), tag


def tagged_image(project_name: str, project_id: int, tag: str, registry: str = DEFAULT_REGISTRY) -> str:
    name, tag = image_info(project_name, project_id, tag, registry)
    return f"{name}:{tag}"


def container_engine() -> Optional[str]:
    for e in ENGINES:
        path = shutil.which(e)
        if path:
            return path
    return None


def resolve_backend(backend: str) -> str:
    if backend not in BACKENDS:
        raise ValueError(f"build backend {backend!r} not in {BACKENDS}")
    if backend == "auto":
        return "container" if container_engine() else "native"
    return backend


def container_build_command(dockerfile: str, context: str, tag: str, nocache: bool = False, push: bool = False,
                            engine: Optional[str] = None) -> str:
    """Shell command that builds (and optionally pushes) the image; fails loudly without an engine."""
    engine = engine or container_engine()
    if engine is None:
        raise RuntimeError("build backend 'container' needs docker or podman on PATH")
    args: List[str] = [engine, "build", "-t", tag, "-f", dockerfile]
    if nocache:
        args.append("--no-cache")
    args.append(context)
    cmd = " ".join(shlex.quote(a) for a in args)
    if push:
        cmd += " && " + " ".join(shlex.quote(a) for a in (engine, "push", tag))
    return cmd


def native_build_command(build_steps: Sequence[str]) -> str:
    return " && ".join(build_steps) if build_steps else "true"


def write_dockerfile(env_dir: str, image: str, build_steps: Sequence[str], env_vars, context: Optional[str]) -> str:
    os.makedirs(env_dir, exist_ok=True)
    path = os.path.join(env_dir, "Dockerfile")
    with open(path + ".tmp", "w") as f:
        f.write(render_dockerfile(image, build_steps, env_vars, context=context))
    os.replace(path + ".tmp", path)
    return path
