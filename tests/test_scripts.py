"""scripts/make_graphs (C17) and scripts/benchmark_test.sh (C20/C21) end to end
on the CPU tiers: the harness must extract a time in seconds and confirm the
hop count against the .json ground truth for every graph."""
import csv
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_make_graphs_and_harness(tmp_path, native):
    env = dict(os.environ, SIZES="1000 10000", SEED="3", BACKEND="native")
    subprocess.run([os.path.join(ROOT, "scripts", "make_graphs"), str(tmp_path)], check=True, env=env,
                   capture_output=True, timeout=300)
    for g in ("1k", "10k"):
        assert (tmp_path / f"{g}.bin").stat().st_size > 8
        assert (tmp_path / f"{g}.json").exists()
    out = tmp_path / "res.csv"
    env = dict(os.environ, TIERS="v1 v2", GRAPHS="1k 10k", REPEAT="3", NP="2",
               LOGDIR=str(tmp_path / "logs"), CSV=str(out))
    r = subprocess.run([os.path.join(ROOT, "scripts", "benchmark_test.sh"), str(tmp_path)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    rows = list(csv.DictReader(open(out)))
    assert len(rows) == 4
    for row in rows:
        assert row["time_sec"] != "ERROR", row
        assert float(row["time_sec"]) < 1.0
        assert row["hops_ok"] == "yes", row
        assert row["timing"] == "hot median x3", row
        assert row["ranks"] == ("2" if row["version"] == "v2" else "1"), row
    assert "| version" in r.stdout
    # MODE=cold: one run per cell, no warm-up, as the reference harness did
    env.update(MODE="cold", TIERS="v1")
    r = subprocess.run([os.path.join(ROOT, "scripts", "benchmark_test.sh"), str(tmp_path)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    rows = list(csv.DictReader(open(out)))
    assert len(rows) == 2 and all(x["timing"] == "cold x1" and x["hops_ok"] == "yes" for x in rows), rows
