"""VERDICT r05 item 4 -- the reference's `go test -race` (/root/reference/Makefile:104,
SURVEY.md section 5) mapped onto the C++ host runtime: the library's .cpp files built with
ThreadSanitizer and with AddressSanitizer (host code only; kraken_amd/csrc/Makefile targets
tsan / asan), then

* tests/native/host_race.cpp: 16 threads at once through every device-free entry point
  (piece sums and verification over pageable buffers on the host pool and CPU tokens, host
  Digesters and piece streams, the InfoHash batch, the window scheduler, the planners with
  rates injected and re-set concurrently, the CPU budget), each result checked against the
  oracle, plus the gather's page registry with its helper threads against a recording
  stand-in for hipHostRegister (the copy-out hazard present before release, gone after);
* this CPU suite's C-ABI tests with the sanitizer runtime preloaded into Python and the
  instrumented library selected by KRK_LIB_PATH.

A sanitizer report fails the run (halt_on_error, a distinct exit code).  CPU only: no GPU
is touched (without a device the library's device paths return KRK_ENODEV)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "kraken_amd", "csrc")
NATIVE = os.path.join(ROOT, "tests", "native")
OPTS = {"tsan": ("TSAN_OPTIONS", "halt_on_error=1:exitcode=66:report_signal_unsafe=0"),
        "asan": ("ASAN_OPTIONS", "halt_on_error=1:exitcode=67:detect_leaks=1")}


def _runtime(kind):
    rt = glob.glob(f"/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.{kind}-x86_64.so")
    if not rt:
        pytest.skip(f"no clang {kind} runtime in this image")
    return rt[0]


def _build(kind):
    _runtime(kind)
    jobs = str(min(8, os.cpu_count() or 4))
    r = subprocess.run(["make", "-s", "-j", jobs, "-C", CSRC, kind], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_host_race_driver_clean(kind):
    _build(kind)
    env = dict(os.environ)
    key, val = OPTS[kind]
    env[key] = val
    r = subprocess.run([os.path.join(NATIVE, f"host_race_{kind}"), "16", "3"], capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-6000:]
    assert "host_race: 16 threads x 3 rounds" in out and out.rstrip().endswith("ok"), out[-2000:]


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_cpu_suite_under_sanitizer(kind):
    """The C-ABI CPU tests with the instrumented library and the sanitizer runtime preloaded
    (Python itself is not instrumented; every report comes from libkraken_hip's host code)."""
    _build(kind)
    env = dict(os.environ)
    key, val = OPTS[kind]
    env[key] = val.replace("detect_leaks=1", "detect_leaks=0")  # CPython's own allocations
    env["LD_PRELOAD"] = _runtime(kind)
    env["KRK_LIB_PATH"] = os.path.join(ROOT, "kraken_amd", "lib", kind, "libkraken_hip.so")
    tests = [os.path.join(ROOT, "tests", t) for t in ("test_capi_cpu.py", "test_host_logic.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        *tests], capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-6000:]
    assert " passed" in out, out[-2000:]
