"""The native core under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer
(host code only — GPU sanitizers are not used on this pool). Builds csrc/tests/
core_selftest.cpp with the scheduler core, the HBM arena, and the step runner's action loop over
the loopback p2p pairing (csrc/runtime/p2p_match.h: one thread per rank, 2 / 4 / 8 ranks),
cached by source hash."""
import hashlib
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["csrc/tests/core_selftest.cpp", "csrc/core/scheduler.cpp", "csrc/core/partition.cpp", "csrc/runtime/arena.cpp"]
HDRS = ["csrc/core/scheduler.h", "csrc/runtime/arena.h", "csrc/runtime/p2p_match.h"]
FLAGS = {
    "asan": ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-O1", "-g", "-fsanitize=thread"],
}


def _build(kind):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    h = hashlib.sha1(" ".join(FLAGS[kind]).encode())
    for f in SRCS + HDRS:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    out_dir = os.path.join(ROOT, "build", "sanitizers")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, f"core_selftest_{kind}_{h.hexdigest()[:12]}")
    if not os.path.exists(exe):
        cmd = [cxx, "-std=c++17", *FLAGS[kind], *[os.path.join(ROOT, s) for s in SRCS],
               f"-I{os.path.join(ROOT, 'csrc')}", "-o", exe + ".tmp", "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            if "sanitize" in r.stderr and "unrecognized" in r.stderr:
                pytest.skip(f"{kind} unsupported by this compiler")
            raise AssertionError(r.stderr[-3000:])
        os.replace(exe + ".tmp", exe)
    return exe


@pytest.mark.parametrize("kind,args", [("asan", ["--instances", "60"]), ("tsan", ["--instances", "15", "--threads", "4"])])
def test_core_under_sanitizers(kind, args):
    exe = _build(kind)
    # verify_asan_link_order=0: the environment may preload libraries ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, *args], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ok (0 failures)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr
