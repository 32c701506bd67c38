"""Build and load the in-tree native libraries (HIP kernels for gfx950 + C++ runtime pieces).

Every library is compiled with ``hipcc --offload-arch=gfx950`` (or ``g++`` for host-only C++) straight
into ``polyaxon_amd/_native/lib<name>.so`` and loaded with :mod:`ctypes`.  The kernels take raw device
pointers and a ``hipStream_t`` (torch's current stream), so they are captured by hipGraphs like any other
launch.  There is deliberately no pure-PyTorch fallback on a GPU box: if a library is missing there,
:func:`lib` raises, so a silent eager path can never pass for the native one.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import shutil
import subprocess
import threading
from pathlib import Path
from typing import Dict, Iterable, List, Optional

PKG_DIR = Path(__file__).resolve().parent.parent
CSRC = PKG_DIR / "csrc"
OUT = PKG_DIR / "_native"
ARCH = os.environ.get("PLX_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

# name -> (sources, kind, extra link flags)
LIBRARIES: Dict[str, dict] = {
    "plx_train": {"sources": ["train_kernels.hip"], "kind": "hip", "link": []},
    "plx_polytune": {"sources": ["polytune_kernels.hip"], "kind": "hip", "link": []},
    "plx_bn": {"sources": ["bn_kernels.hip"], "kind": "hip", "link": []},
    "plx_procmon": {"sources": ["procmon.cpp"], "kind": "cpp", "link": ["-lpthread"]},
    "plx_gp": {"sources": ["gp_kernels.hip", "gp_chol.hip"], "kind": "hip", "link": []},
    "plx_rms": {"sources": ["rmsnorm.hip"], "kind": "hip", "link": []},
    "plx_conv": {"sources": ["conv_gemm.hip"], "kind": "hip", "link": []},
    "plx_pool": {"sources": ["pool_kernels.hip"], "kind": "hip", "link": []},
    "plx_lm": {"sources": ["lm_kernels.hip"], "kind": "hip", "link": []},
    "plx_gemm": {"sources": ["gemm256.hip"], "kind": "hip", "link": []},
    "plx_attn": {"sources": ["attn_kernels.hip"], "kind": "hip", "link": []},
    "plx_rccl": {"sources": ["rccl_comm.cpp"], "kind": "hip_host", "link": ["-lrccl", "-pthread"]},
}

_lock = threading.Lock()
_loaded: Dict[str, ctypes.CDLL] = {}


def _register(name: str, sources: List[str], kind: str, link: Optional[List[str]] = None) -> None:
    LIBRARIES[name] = {"sources": sources, "kind": kind, "link": list(link or [])}


def lib_path(name: str) -> Path:
    return OUT / f"lib{name}.so"


def _digest(sources: Iterable[Path], flags: List[str]) -> str:
    h = hashlib.sha256()
    for s in sources:
        h.update(s.read_bytes())
    for hdr in sorted(CSRC.glob("*.h")):
        h.update(hdr.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _flags(kind: str) -> List[str]:
    common = ["-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-function", f"-I{CSRC}"]
    if kind == "hip":
        # PLX_HANDOFF_FENCES=1: the in-launch partial-row hand-offs use release / acquire fences (csrc/handoff.h)
        fences = ["-DPLX_HANDOFF_FENCES=1"] if os.environ.get("PLX_HANDOFF_FENCES") == "1" else []
        return common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + fences
    if kind == "hip_host":  # host C++ that links the HIP runtime (streams, events, pinned memory, RCCL)
        return common + [f"-I{ROCM / 'include'}", "-D__HIP_PLATFORM_AMD__"]
    return common  # plain host C++


def build(name: str, force: bool = False, verbose: bool = False) -> Path:
    """Compile one library if its sources changed. Returns the .so path."""
    spec = LIBRARIES[name]
    srcs = [CSRC / s for s in spec["sources"]]
    flags = _flags(spec["kind"])
    out = lib_path(name)
    stamp = out.with_suffix(".so.sha")
    digest = _digest(srcs, flags + spec["link"])
    if not force and out.exists() and stamp.exists() and stamp.read_text().strip() == digest:
        return out
    OUT.mkdir(parents=True, exist_ok=True)
    if spec["kind"] in ("hip", "hip_host"):
        cc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    else:
        cc = shutil.which("g++") or "g++"
    link = list(spec["link"])
    if spec["kind"] == "hip_host":
        link = [f"-L{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'lib'}"] + link + ["-lamdhip64"]
    tmp = out.with_suffix(f".so.tmp{os.getpid()}")
    cmd = [cc, *flags, *map(str, srcs), "-o", str(tmp), *link]
    if verbose:
        print(" ".join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"native build of {name} failed:\n{' '.join(cmd)}\n{proc.stderr[-6000:]}")
    os.replace(tmp, out)
    stamp.write_text(digest)
    return out


def _stale(name: str) -> bool:
    spec = LIBRARIES[name]
    stamp = lib_path(name).with_suffix(".so.sha")
    if not stamp.exists():
        return False  # shipped without a stamp: trust it
    try:
        digest = _digest([CSRC / s for s in spec["sources"]], _flags(spec["kind"]) + spec["link"])
    except OSError:
        return False
    return stamp.read_text().strip() != digest


def build_all(force: bool = False, verbose: bool = False) -> List[Path]:
    return [build(n, force=force, verbose=verbose) for n in LIBRARIES]


def available(name: str) -> bool:
    return lib_path(name).exists()


_SIZES: Dict[tuple, int] = {}


_COUNTERS: Dict[tuple, object] = {}


def capturing() -> bool:
    """Is the current HIP stream being captured into a hipGraph?"""
    import torch

    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def cached(cache: dict, key, make, ok=None):
    """``cache[key]`` (when ``ok(value)`` holds), else ``make()``.  A device buffer allocated while a stream is being
    captured comes from that graph's private memory pool and dangles once the graph is freed, so such a value is
    never stored: during capture a cached buffer is reused when present, else a fresh one serves this launch only
    (its allocation and initialisation are part of the graph).  Long-lived buffers -- zero pages, last-arriver
    tickets, workspaces -- therefore always live in the default pool."""
    v = cache.get(key)
    if v is not None and (ok is None or ok(v)):
        return v
    v = make()
    if not capturing():
        cache[key] = v
    return v


def counters(device, key: str, n: int = 4096):
    """A zeroed int32 counter array per (device, op) for the last-arriver kernels: each arriver that finishes a
    reduction resets its own counter, so the array is reused by every stream-ordered launch of that op."""
    import torch

    return cached(_COUNTERS, (str(device), key), lambda: torch.zeros(n, dtype=torch.int32, device=device))


def current_stream() -> int:
    """Raw handle of the current HIP stream of the current device: two C calls, against ~8 us for
    ``torch.cuda.current_stream().cuda_stream`` (a Python Stream object and device-index resolution per call) --
    every op's launch path asks for it, ~160 times per ResNet-50 step."""
    import torch

    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def size(libname: str, fn: str, *args: int) -> int:
    """Memoised integer query (workspace sizes, block counts): pure functions of their int arguments (and of
    knobs fixed at load time), called from every op's host path -- the ctypes round trip is not free there."""
    key = (fn,) + args
    v = _SIZES.get(key)
    if v is None:
        v = _SIZES[key] = int(getattr(lib(libname), fn)(*args))
    return v


def lib(name: str) -> ctypes.CDLL:
    """Load (building on first use if a compiler is present) the named native library."""
    with _lock:
        if name in _loaded:
            return _loaded[name]
        path = lib_path(name)
        # rebuild when the sources changed since the .so was built (digest stamp), or when forced
        if not path.exists() or os.environ.get("PLX_NATIVE_REBUILD") == "1" or _stale(name):
            build(name, force=os.environ.get("PLX_NATIVE_REBUILD") == "1")
        handle = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        _declare(name, handle)
        if name == "plx_conv" and os.environ.get("PLX_WGRAD_ATOMIC"):  # A/B knob: 0 = slab reducer (deterministic)
            handle.plx_set_tn_atomic(int(os.environ["PLX_WGRAD_ATOMIC"]))
        if name == "plx_gemm" and os.environ.get("PLX_GEMM_WAVES"):  # 8 = ping-pong kernel, 4 = AGPR 4-wave kernel
            handle.plx_gemm256_set_waves(int(os.environ["PLX_GEMM_WAVES"]))
        _loaded[name] = handle
        return handle


# ----------------------------------------------------------------------------- signatures
_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_U64 = ctypes.c_uint64
_F = ctypes.c_float
_D = ctypes.c_double

SIGNATURES: Dict[str, Dict[str, list]] = {
    "plx_train": {
        "plx_sgd_flat": [_P, _P, _P, _L, _L, _P, _P, _P],
        "plx_adamw_flat": [_P, _P, _P, _P, _L, _L, _P, _P, _P],
        "plx_adamw_mixed": [_P, _P, _P, _P, _P, _L, _I, _P, _P, _P],
        "plx_cast_lp": [_P, _P, _L, _P],
        "plx_init_flat": [_P, _P, _P, _P, _I, _P, _P, _U64, _P],
        "plx_zero_flat": [_P, _L, _P],
        "plx_record_metric": [_P, _I, _P, _P, _I, _P],
        "plx_commit_metric": [_P, _P, _I, _I, _P, _I, _P],
        "plx_synth_images": [_P, _P, _I, _I, _I, _P, _I, _I, _F, _U64, _P, _P],
        "plx_set_adamw_grid_cap": [_I],
        "plx_set_adamw_wide": [_I],
    },
    "plx_bn": {
        "plx_bn_workspace": [_L, _I],
        "plx_bn_forward": [_P, _P, _P, _L, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P],
        "plx_bn_apply": [_P, _P, _P, _L, _I, _P, _I, _P],
        "plx_bn_l2_workspace": [_I, _I],
        "plx_bn_forward_from_partials": [_P, _P, _P, _L, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _I, _P, _P,
                                         _I, _P, _P, _P],
        "plx_bn_backward": [_P, _P, _P, _P, _P, _L, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P],
        "plx_bn_dx_blocks": [_L, _I],
        "plx_bn_backward_from_partials": [_P, _P, _P, _P, _P, _L, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _I, _I, _P,
                                          _P, _P],
        "plx_stem_bn_pool_forward": [_P, _P, _P, _I, _I, _I, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P, _I, _P,
                                     _P],
        "plx_stem_bn_pool_bwd_workspace": [_I, _I, _I, _I],
        "plx_stem_bn_pool_backward": [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P],
    },
    "plx_procmon": {
        "plx_pm_create": [],
        "plx_pm_destroy": [_P],
        "plx_pm_spawn": [_P, _P, _P, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(_I)],
        "plx_pm_wait": [_P, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)],
        "plx_pm_wake": [_P],
        "plx_pm_signal": [_P, _I, _I, _I],
        "plx_pm_count": [_P],
    },
    "plx_gp": {
        "plx_gp_kmat": [_P, _P, _I, _I, _I, _P, _I, _I, _F, _F, _F, _I, _F, _P, _P, _D, _I, _P],
        "plx_gp_chol": [_P, _I, _I, _P, _P],
        "plx_gp_kmat_batch_f64": [_P, _I, _I, _P, _I, _P, _I, _L, _I, _D, _D, _D, _P, _P, _D, _I, _P],
        "plx_gp_matern_table": [_D, _D, _D, _I, _P, _P, _P],
        "plx_gp_chol_aug_f64": [_P, _I, _I, _I, _L, _I, _P, _P, _P],
        "plx_gp_chol_scratch_doubles": [],
        "plx_gp_lml_f64": [_P, _I, _I, _L, _I, _P, _P, _P],
        "plx_gp_acq_rows": [_P, _I, _I, _P, _F, _I, _F, _F, _F, _P, _P, _P, _P],
        "plx_gp_predict_acq": [_P, _I, _P, _I, _I, _P, _I, _P, _I, _F, _F, _F, _F, _I, _F, _F, _F, _P, _P, _P, _P,
                               _P, _P, _P, _D, _I, _P],
        "plx_gp_ascent": [_P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _I, _F, _F, _F, _F, _I, _F, _F, _F, _I, _P, _P, _D, _I,
                          _P],
    },
    "plx_conv": {
        "plx_gemm_nt": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _P],
        "plx_gemm_nt_rows_per_block": [_I],
        "plx_gemm_tn_workspace": [_I, _I, _I, _I],
        "plx_set_tn_v2": [_I, _I],
        "plx_set_tn2_stem": [_I],
        "plx_set_tn2_c64": [_I],
        "plx_set_tn_atomic": [_I],
        "plx_tn_plan_slices": [_I, _I, _I, _I, _I],
        "plx_gemm_tn": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P],
        "plx_weight_prep": [_P, _P, _P, _I, _I, _P],
        "plx_weight_prepk": [_P, _L, _L, _L, _L, _P, _P, _I, _I, _I, _P],
        "plx_weight_prep_all": [_P, _P, _P, _P, _I, _I, _P],
        "plx_stem_pack_input": [_P, _P, _I, _I, _I, _P],
        "plx_stem_pack_weight": [_P, _L, _L, _L, _L, _P, _I, _P],
        "plx_stem_conv_rows_per_block": [],
        "plx_stem_conv_fwd": [_P, _P, _P, _I, _I, _I, _P, _P, _P],
        "plx_stem_conv_wgrad_workspace": [_I, _I, _I, _I],
        "plx_stem_conv_wgrad": [_P, _P, _P, _L, _L, _L, _L, _P, _I, _I, _I, _P, _I, _I, _P],
        "plx_conv_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P],
        "plx_conv_dgrad": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P],
        "plx_conv_dgrad_blocks": [_I, _I, _I, _I, _I, _I, _I],
        "plx_conv_wgrad_workspace": [_I, _I, _I, _I, _I, _I, _I, _I],
        "plx_conv_wgrad": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P],
    },
    "plx_lm": {
        "plx_qkv_rope_fwd": [_P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _I, _I, _P],
        "plx_qkv_rope_bwd": [_P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _I, _I, _P],
        "plx_swiglu_fwd": [_P, _P, _L, _I, _P],
        "plx_swiglu_bwd": [_P, _P, _P, _L, _I, _P],
        "plx_xent_fwd": [_P, _P, _P, _P, _I, _I, _I, _P],
        "plx_xent_bwd": [_P, _P, _P, _P, _P, _I, _I, _I, _P],
        "plx_xent_cls_fwd": [_P, _P, _P, _P, _I, _I, _P],
        "plx_xent_cls_bwd": [_P, _P, _P, _P, _P, _I, _I, _F, _P],
        "plx_colsum_splits": [_L, _I],
        "plx_colsum": [_P, _L, _I, _P, _P, _P, _I, _P],
        "plx_gelu_bwd_colsum": [_P, _P, _P, _L, _I, _P, _P, _P, _I, _P],
    },
    "plx_gemm": {
        "plx_gemm256": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _I, _P],
        "plx_gemm256_bias": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P],
        "plx_gemm256_ex": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P, _P],
        "plx_gemm256_exv": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P, _I, _P],
        "plx_gemm256_splits": [_I, _I, _I],
        "plx_gemm256_set_split_target": [_I],
        "plx_gemm256_set_waves": [_I],
        "plx_gemm256_set_group": [_I],
        "plx_gemm256_tile": [],
        "plx_gemm256_sk_ws": [_I, _I, _I],
        "plx_gemm256_sk_plan": [_I, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)],
        "plx_gemm256_set_sk_force": [_I],
        "plx_gemm256_sk": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _P, _P, _P, _P],
    },
    "plx_attn": {
        "plx_attn_fwd": [_P, _I, _P],
        "plx_attn_bwd": [_P, _I, _P, _P],
        "plx_attn_bwd_workspace": [_I, _I, _I, _I, _I],
        "plx_attn_args_size": [],
        "plx_attn_set_fwd_waves": [_I],
        "plx_attn_set_dq_waves": [_I],
        "plx_attn_set_dkdv_waves": [_I],
    },
    "plx_pool": {
        "plx_maxpool3s2_forward": [_P, _P, _P, _I, _I, _I, _I, _P],
        "plx_gap_forward": [_P, _P, _I, _I, _I, _P],
        "plx_gap_backward": [_P, _P, _I, _I, _I, _P],
        "plx_maxpool3s2_backward": [_P, _P, _P, _I, _I, _I, _I, _P],
    },
    "plx_rms": {
        "plx_rms_forward": [_P, _P, _P, _P, _L, _I, _F, _P],
        "plx_rms_bwd_blocks": [_L],
        "plx_ln_bwd_blocks": [_L, _I],
        "plx_add_ln_forward": [_P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _F, _P],
        "plx_add_rms_forward": [_P, _P, _P, _P, _P, _P, _L, _I, _F, _P],
        "plx_add_rms_backward": [_P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
        "plx_add_ln_backward": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
        "plx_partial_colsum_workspace": [_I, _I, _I],
        "plx_partial_colsum": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _P],
        "plx_rms_backward": [_P, _P, _P, _P, _P, _P, _L, _I, _P],
        "plx_ln_forward": [_P, _P, _P, _P, _P, _P, _L, _I, _F, _P],
        "plx_ln_backward": [_P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    },
    "plx_rccl": {
        "plx_rccl_unique_id": [ctypes.c_char_p],
        "plx_rccl_init": [ctypes.c_char_p, _I, _I, _I, _L, _L, ctypes.POINTER(_I)],
        "plx_rccl_all_reduce": [_P, _P, _P, _L, _I, _I, _P],
        "plx_rccl_all_gather": [_P, _P, _P, _L, _I, _P],
        "plx_rccl_reduce_scatter": [_P, _P, _P, _L, _I, _I, _P],
        "plx_rccl_broadcast": [_P, _P, _P, _L, _I, _I, _P],
        "plx_rccl_bus_bw": [_P, _P, _L, _I, _P, ctypes.POINTER(_D), ctypes.POINTER(_D)],
        "plx_rccl_destroy": [_P],
        "plx_rccl_status": [_P],
        "plx_rccl_pending": [_P],
        "plx_rccl_set_timeout": [_P, _L],
        "plx_rccl_abort": [_P],
        "plx_rccl_error": [_I],
    },
    "plx_polytune": {
        "plx_topk_brackets": [_P, _P, _I, _I, _I, _I, _P, _P],
        "plx_philox_sample": [_P, _P, _I, _L, _L, ctypes.c_uint64, _P, _P],
        "plx_philox_desc_size": [],
        "plx_early_stop_any": [_P, _I, _I, _P, _P, _P, _I, _P, _P],
    },
}


RESTYPES: Dict[str, object] = {"plx_attn_bwd_workspace": ctypes.c_longlong, "plx_conv_wgrad_workspace": _L, "plx_bn_workspace": _L, "plx_bn_l2_workspace": _L, "plx_partial_colsum_workspace": _L, "plx_stem_bn_pool_bwd_workspace": _L, "plx_gemm_tn_workspace": _L, "plx_gemm256_sk_ws": ctypes.c_longlong, "plx_stem_conv_wgrad_workspace": _L, "plx_pm_create": _P, "plx_pm_destroy": None, "plx_set_tn_v2": None, "plx_set_tn2_stem": None, "plx_set_tn2_c64": None, "plx_set_tn_atomic": None, "plx_set_adamw_grid_cap": None, "plx_set_adamw_wide": None, "plx_attn_set_fwd_waves": None, "plx_attn_set_dq_waves": None, "plx_attn_set_dkdv_waves": None, "plx_gemm256_set_split_target": None,
                               "plx_pm_wake": None, "plx_rccl_init": _P, "plx_rccl_error": ctypes.c_char_p}


def _declare(name: str, handle: ctypes.CDLL) -> None:
    for fn, argtypes in SIGNATURES.get(name, {}).items():
        f = getattr(handle, fn)
        f.argtypes = argtypes
        f.restype = RESTYPES.get(fn, _I)


class ResBnArgs(ctypes.Structure):
    """Host image of ``ResBn`` (csrc/bn_kernels.hip): the residual BatchNorm whose reduction partials the dx pass
    of the BatchNorm consuming its output also produces."""
    _fields_ = [("x", _P), ("mask", _P), ("mean", _P), ("invstd", _P), ("part", _P)]


class BnBwdArgs(ctypes.Structure):
    """Host image of ``BnBwd`` (csrc/conv_gemm.hip): fused BatchNorm-backward partials in a dgrad GEMM epilogue."""
    _fields_ = [("x", _P), ("mask", _P), ("mean", _P), ("invstd", _P), ("part", _P), ("part_ld", _I),
                ("blk_off", _I), ("skip_h", _I), ("skip_w", _I)]


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")
