import faulthandler
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# A test marked ``isolated`` runs in a FRESH child pytest process (one per test), spawned by
# this process: the multi-rank-in-one-process harness tests (parallel/loopback.py) capture
# hipGraphs on several threads at once and need more hardware queues than HIP's default, so
# they get their own process with GPU_MAX_HW_QUEUES=16 while the rest of the suite runs under
# the pool's default. An abort inside one of them fails that test — it cannot end the suite.
CHILD_ENV = "DLS_ISOLATED_CHILD"
IN_CHILD = os.environ.get(CHILD_ENV) == "1"
ISOLATED_QUEUES = "16"  # 4 ranks x (compute, copy, capture stream) + the default; pool limit 32
ISOLATED_TIMEOUT_S = int(os.environ.get("DLS_ISOLATED_TIMEOUT_S", "300"))

_GPU = None


def _has_gpu() -> bool:
    global _GPU
    if _GPU is None:
        try:
            import torch
            _GPU = torch.cuda.is_available()
        except Exception:  # pragma: no cover
            _GPU = False
    return _GPU


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "isolated: runs in a fresh child process of its own (see conftest.py)")
    if not faulthandler.is_enabled():
        faulthandler.enable(file=sys.__stderr__, all_threads=True)


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def pytest_runtest_logstart(nodeid, location):
    """GPU sessions: name every test on the terminal, flushed, BEFORE it runs — if the process
    dies inside a test, the output's last line names it (round 5's driver record ended mid-line
    after 1,035 dots and did not)."""
    if not (_GPU and not IN_CHILD):
        return
    sys.__stdout__.write(f"\n[start] {nodeid}\n")
    sys.__stdout__.flush()


@pytest.fixture(autouse=True)
def _release_native_garbage():
    """Between tests, on the main thread: destroy the hipGraphs / runners / buffers of executors
    that died during the test (parallel/lifetime.py defers them to such quiesce points)."""
    yield
    if _GPU:
        from distributed_llm_scheduler_amd.parallel import lifetime
        lifetime.release()


def pytest_pyfunc_call(pyfuncitem):
    """``isolated`` tests on the GPU: run the test's node id in a child pytest process."""
    if IN_CHILD or pyfuncitem.get_closest_marker("isolated") is None or not _has_gpu():
        return None
    env = dict(os.environ)
    env[CHILD_ENV] = "1"
    env["GPU_MAX_HW_QUEUES"] = ISOLATED_QUEUES
    env["PYTHONUNBUFFERED"] = "1"
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "--timeout",
           str(ISOLATED_TIMEOUT_S - 30), "--timeout-method", "thread", pyfuncitem.nodeid]
    try:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           timeout=ISOLATED_TIMEOUT_S, text=True)
    except subprocess.TimeoutExpired as e:
        out = e.stdout or ""
        pytest.fail(f"isolated child timed out after {ISOLATED_TIMEOUT_S} s:\n{out[-6000:]}", pytrace=False)
    out = r.stdout or ""
    if r.returncode != 0 or " passed" not in out:
        pytest.fail(f"isolated child exited {r.returncode}:\n{out[-6000:]}", pytrace=False)
    return True
