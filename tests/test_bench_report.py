"""bench.py's output line (driver contract) built from synthetic per-config
numbers, no GPU: required keys, whole-job value, weak vs strong scaling,
vs_baseline only for the 100k headline graph."""
import argparse
import json

import bench


def _head(n=100000, gteps=4.5, ms=0.024):
    return {"n": n, "m": 110201, "seed": 6, "gteps": gteps, "ms_per_step": ms, "device_ms_per_query": 0.017,
            "gteps_inspected": 0.08, "mean_hops": 14.3, "build_ms": 80.0, "batched": None}


def _args(mode="replicated", steps=400, warmup=50):
    return argparse.Namespace(mode=mode, steps=steps, warmup=warmup, no_resident=False)


def test_report_contract_keys_and_baseline():
    out = bench.report(_args(), 8, _head(gteps=36.0), {}, {})
    json.dumps(out)  # one JSON line
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 8 and out["steps"] == 400 and out["warmup"] == 50
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["data"] == "synthetic"
    assert out["value"] == 36.0
    assert abs(out["vs_baseline"] - 36.0 / bench.BASELINE_100K_GTEPS) < 1e-3
    assert out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 8


def test_report_partitioned_is_strong_scaling_and_other_graph_has_no_baseline():
    out = bench.report(_args(mode="partitioned"), 2, _head(n=1000000), {}, {})
    assert out["scaling"] == "strong" and out["vs_baseline"] is None
    assert out["config"]["parallelism"] == "vertex-partition2" and out["config"]["global_batch"] == 1


def test_spawn_path_forwards_rank0_line_and_status(capsys):
    """`bench.py --gpus N` without a launcher runs the ranks as a child job
    (mocked here by a child that prints a line) and forwards its status."""
    import sys

    line = json.dumps({"metric": "m", "value": 1.0, "n_gpus": 8})
    ok = [sys.executable, "-c", f"print('noise'); print({line!r})"]
    assert bench.spawn_ranks(8, [], cmd=ok) == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert out == [line]
    bad = [sys.executable, "-c", f"print({line!r}); raise SystemExit(3)"]
    assert bench.spawn_ranks(8, [], cmd=bad) == 3
    silent = [sys.executable, "-c", "pass"]
    assert bench.spawn_ranks(8, [], cmd=silent) == 1


def test_launcher_command_and_world_check(monkeypatch):
    """The self-launch uses torch.distributed.run on 127.0.0.1 with one rank per
    GPU; a launcher-provided WORLD_SIZE that disagrees with --gpus fails fast
    (before torch is imported)."""
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "3"])
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.main(["--gpus", "4"]) == 2
    monkeypatch.delenv("WORLD_SIZE")
    called = {}

    def fake_spawn(n, argv):
        called["n"], called["argv"] = n, argv
        return 0

    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    assert bench.main(["--gpus", "8", "--steps", "2"]) == 0
    assert called == {"n": 8, "argv": ["--gpus", "8", "--steps", "2"]}


def test_world_scaled_partitioned_config():
    """kron:auto: Kronecker 27 on one GPU (the single-GPU engine is its
    reference); for N >= 2 a graph that does NOT fit one GPU -- its CSR is
    ~1.35x one GPU's HBM -- while every rank's shard stays within ~70% of it."""
    import bench

    H = 288 * 10**9
    assert bench.world_scaled("kron:auto", 1, H) == "kron:27:16:1"
    for w in (2, 4, 8):
        spec = bench.world_scaled("kron:auto", w, H)
        assert spec.startswith("kron:30:")
        total = bench.csr_bytes(spec)
        assert total > 1.25 * H, (spec, total)
        assert total / w < 0.72 * H, (spec, total / w)
    assert bench.world_scaled("kron:auto", 8, H) == "kron:30:44:1"
    assert bench.world_scaled("gnp:1000000::2", 8, H) == "gnp:1000000::2"
    assert bench.csr_bytes("kron:27:16:1") == 8 * ((1 << 27) + 1) + 8 * (16 << 27)


def test_secondary_errors_listed_without_touching_the_headline():
    """A failed, unverified or unfinished secondary config is named in
    detail.secondary_errors; the headline fields are unchanged."""
    extra = {"gnp:10000000::1": {"ms_per_step": 0.09}, "kron:22:16:1": {"error": "RuntimeError('x')"}}
    part = {"gnp:1000000::2": {"verified": False}, "kron:30:16:1": None, "kron:22:16:1": {"verified": True}}
    out = bench.report(_args(), 8, _head(gteps=36.0), extra, part)
    assert out["detail"]["secondary_errors"] == ["gnp:1000000::2", "kron:22:16:1", "kron:30:16:1"]
    assert out["value"] == 36.0
    assert bench.report(_args(), 1, _head(), {}, {})["detail"]["secondary_errors"] == []


def test_reporting_hygiene_fields_and_exit_status():
    """Round-4 reporting fields: the headline carries the timed loop's tiny-
    server fallbacks; a partitioned entry reports communicator bootstrap
    apart from the graph build; wrong answers always fail the run."""
    head = dict(_head(), tiny_overflows=3)
    part = {"gnp:1000000::2": {"verified": True, "build_ms": 70.0}}
    out = bench.report(_args(), 1, head, {}, part, comm_init_ms=3650.0)
    assert out["detail"]["tiny_overflows"] == 3
    p = out["detail"]["partitioned"]["gnp:1000000::2"]
    assert "build_ms" in p
    # one communicator for every partitioned config, its bootstrap reported once
    assert out["detail"]["partitioned_comm_init_ms"] == 3650.0
    assert bench.exit_status(part, False, False) == 0
    assert bench.exit_status({"x": {"verified": False}}, False, False) == 5
    assert bench.exit_status({"x": {"error": "timeout"}}, True, False) == 0
    assert bench.exit_status({"x": {"error": "timeout"}}, True, True) == 4


def test_cpu_comparison_fields_for_every_replicated_config():
    """Round-5 fields: every replicated config (headline and extras) carries
    the serial CPU engine's time on the SAME graph and pairs, the speedup over
    it, and how many of its pairs a unidirectional host BFS re-derived."""
    f = bench.cpu_fields(0.9, 1.0, 1.2, 4, 2.5, 0.06)
    assert f == {"cpu_serial_ms": 0.9, "cpu_serial_mean_ms": 1.0, "cpu_serial_query_ms": 1.2,
                 "cpu_serial_first_pass_ms": 2.5, "speedup_vs_cpu_serial_query": 20.0, "cpu_oracle_checked_pairs": 4}
    extra = {"gnp:10000000::1": dict({"ms_per_step": 0.06}, **f)}
    out = bench.report(_args(), 1, _head(), extra, {})
    e = out["detail"]["extra"]["gnp:10000000::1"]
    assert e["cpu_serial_query_ms"] == 1.2 and e["cpu_oracle_checked_pairs"] == 4


def test_cpu_serial_reference_on_small_graph():
    """cpu_serial_ms runs the serial engine on the bench's graph and pairs and
    holds every hop count to it (and the first pairs to bfs_oracle)."""
    from bidirectional_bfs_amd import native

    spec = "gnp:20000::4"
    kind, n, p, seed = bench.parse_spec(spec)
    csr = native.build_csr(native.gen_gnp(n, p, seed))
    eng = native.SerialBiBfs(csr)
    pairs = []
    for s, d in [(0, n - 1), (5, 77), (100, 9000), (3, 19999)]:
        r = eng.search(s, d)
        if r.found and r.hops > 0:
            pairs.append((s, d, int(r.hops)))
    med, mean, e2e, ok, first = bench.cpu_serial_ms(spec, pairs, reps=2, oracle_pairs=2)
    assert med > 0 and mean > 0 and e2e > 0 and first > 0 and ok == min(2, len(pairs))


def test_partitioned_headline_fields_beside_the_replicated_value():
    """Round-6: the partitioned BASELINE config-3 numbers (1M G(n, p), one
    collective search per query) sit at the top level next to the replicated
    headline, so a scaling run over N reports the v4 engine too."""
    part = {"gnp:1000000::2": {"verified": True, "ms_per_query": 0.41, "speedup_vs_single_gpu": 0.09,
                               "gteps": 2.68, "collectives_per_round": 1.1}}
    out = bench.report(_args(), 4, _head(gteps=36.0), {}, part)
    assert out["value"] == 36.0 and out["scaling"] == "weak"
    assert out["partitioned_config"] == "gnp:1000000::2"
    assert out["partitioned_ms_per_query"] == 0.41 and out["partitioned_speedup_vs_single_gpu"] == 0.09
    assert out["partitioned_collectives_per_round"] == 1.1 and out["partitioned_verified"] is True
    failed = bench.report(_args(), 4, _head(), {}, {"gnp:1000000::2": {"error": "x"}})
    assert failed["partitioned_ms_per_query"] is None
    assert bench.report(_args(), 1, _head(), {}, {})["partitioned_ms_per_query"] is None


def _rehearsals():
    import glob
    import os

    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return sorted(glob.glob(os.path.join(here, "profiles", "r6_bench_[24]rank_1gpu_ipc*.json")))


def test_ipc_rehearsal_lines_carry_partitioned_fields():
    """The 2- and 4-rank IPC rehearsals (bench.py --gpus 2/4 on one GPU,
    measured on the GPU box and committed under profiles/) carry the
    top-level partitioned fields, verified, with every rank counted."""
    import pytest

    files = _rehearsals()
    if not files:
        pytest.skip("no round-6 rehearsal profiles committed")
    seen = set()
    for f in files:
        with open(f) as fh:
            line = [ln for ln in fh.read().splitlines() if ln.strip().startswith("{")][-1]
        d = json.loads(line)
        assert d["n_gpus"] in (2, 4), f
        seen.add(d["n_gpus"])
        assert d["partitioned_config"] == "gnp:1000000::2"
        assert d["partitioned_ms_per_query"] > 0 and d["partitioned_verified"] is True, f
        assert d["partitioned_speedup_vs_single_gpu"] is not None
        p = d["detail"]["partitioned"]["gnp:1000000::2"]
        assert p["ranks"] == d["n_gpus"] and p["ms_per_query"] == d["partitioned_ms_per_query"]
    assert seen == {2, 4}, seen
