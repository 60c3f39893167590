"""The unified CLI (python -m distributed_llm_scheduler_amd ...), CPU paths."""
import json

from distributed_llm_scheduler_amd import cli


def test_cli_plan_save_and_run_resume(tmp_path, capsys):
    path = str(tmp_path / "plan.json")
    assert cli.main(["plan", "--model", "tiny-gpt2", "--seq", "16", "--devices", "1", "--save", path]) == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["tasks_completed"] == out["tasks_total"] == 19
    trace = str(tmp_path / "t.json")
    assert cli.main(["run", "--device", "cpu", "--model", "tiny-gpt2", "--seq", "16", "--steps", "1", "--warmup", "0",
                     "--resume", path, "--trace", trace]) == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["tasks_completed"] == 19 and res["ms_per_step"] > 0
    assert any(e["ph"] == "X" for e in json.load(open(trace))["traceEvents"])


def test_cli_reference_cost_model_plan(capsys):
    assert cli.main(["plan", "--model", "gpt2", "--devices", "4", "--scheduler", "MRU_spec", "--cost-model",
                     "reference", "--hbm-cap-gb", "8"]) == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["tasks_total"] == 99 and out["tasks_completed"] == 99


def test_cli_extract_and_models(tmp_path, capsys):
    path = str(tmp_path / "g.json")
    assert cli.main(["extract", "--out", path]) == 0
    assert len(json.load(open(path))["tasks"]) == 99
    assert cli.main(["models"]) == 0
    assert "llama3-8b" in capsys.readouterr().out


def test_cli_simulate_execute(tmp_path, capsys):
    out = str(tmp_path / "ev")
    assert cli.main(["simulate", "--execute", "--model", "tiny-llama", "--seq", "16", "--steps", "1", "--warmup", "1",
                     "--regimes", "1.0,0.8", "--schedulers", "DFS,EFT", "--out", out]) == 0
    import pandas as pd
    df = pd.read_csv(f"{out}/raw_results.csv")
    assert len(df) == 4 and (df["wall_makespan_ms"] > 0).all()
    eft = df[(df.scheduler_name == "EFT") & (df.memory_regime == 0.8)].iloc[0]
    assert eft.completed_tasks == eft.total_tasks
