"""Device-loss injection + re-plan onto the survivors (multi-process, gloo on CPU)."""
import torch

from distributed_llm_scheduler_amd.models import reference
from distributed_llm_scheduler_amd.parallel import runtime
from distributed_llm_scheduler_amd.parallel.elastic import run_elastic
from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens


def test_device_loss_replans_and_completes():
    kw = dict(model="tiny-gpt2", seq=16, replicas=3, placement="replica")
    out = run_elastic(world=3, steps=2, fail_rank=1, fail_step=1, timeout=240, **kw)
    assert out["attempts"][0] == {"world": 3, "lost": [1], "devices": [0, 1, 2]}
    # the survivors keep their physical devices: new ranks 0, 1 -> devices 0, 2
    assert out["attempts"][1] == {"world": 2, "lost": [], "devices": [0, 2]} and out["world"] == 2
    sums = {}
    for r in out["results"]:
        assert r["ok"]
        assert r["device"] == [0, 2][r["rank"]]
        sums.update(r.get("logits_sum", {}))
    assert sorted(sums) == ["r0/output_projection", "r1/output_projection", "r2/output_projection"]
    p = runtime.plan(world=2, **kw)
    store = runtime.make_store(p)
    for rid in ("r0/", "r1/", "r2/"):
        tok = synthetic_tokens(f"{rid}@tokens", 16, p.cfg.vocab_size).view(1, 16)
        ref = float(reference.forward(p.cfg, store, tok).sum())
        assert abs(sums[f"{rid}output_projection"] - ref) < 0.02 * abs(ref) + 1.0


def test_no_failure_single_attempt():
    out = run_elastic(world=2, steps=1, timeout=240, model="tiny-llama", seq=16, replicas=2)
    assert out["attempts"] == [{"world": 2, "lost": [], "devices": [0, 1]}]
