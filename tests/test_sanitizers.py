"""Native host code under sanitizers: the process supervisor (csrc/procmon.cpp) stress-tested
with AddressSanitizer + UndefinedBehaviorSanitizer and with ThreadSanitizer (host compiler, no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "procmon_stress.cpp")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_procmon_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "procmon_stress")
    flags = ["-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer"]
    if "undefined" in san:
        flags.append("-fno-sanitize-recover=undefined")
    build = subprocess.run([cxx, *flags, SRC, "-o", exe], capture_output=True, text=True, timeout=180)
    if build.returncode != 0 and "sanitize" in build.stderr and "unsupported" in build.stderr:
        pytest.skip(f"{san} sanitizer unsupported here")
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "150"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "bad 0 left 0" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
