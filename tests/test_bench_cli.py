"""The bench.py driver contract on the CPU fake device: one JSON line from rank 0 with the
BASELINE metric fields, single process and under torch.distributed.run (gloo, 2 ranks)."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "tiny-gpt2", "--seq", "32", "--steps", "2", "--warmup", "1"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _run(cmd):
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return _json_lines(r.stdout)


def _check(line, n):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["n_gpus"] == n and line["steps"] == 2 and line["warmup"] == 1
    assert line["higher_is_better"] is False and line["scaling"] == "weak"
    assert line["value"] > 0 and line["config"]["model"] == "tiny-gpt2"
    assert "synthetic" in line["data"]


def test_bench_single_process():
    lines = _run([sys.executable, "bench.py", "--gpus", "1", *ARGS])
    assert len(lines) == 1
    _check(lines[0], 1)


@pytest.mark.timeout(300)
def test_bench_two_ranks_gloo():
    lines = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                  "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", *ARGS])
    assert len(lines) == 1  # rank 0 only
    _check(lines[0], 2)
