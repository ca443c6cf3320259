"""One rank of :func:`bidirectional_bfs_amd.parallel.dist_proc_run`.

``python -m bidirectional_bfs_amd.parallel._proc_worker JOB.json RANK``: builds
a native ``DistBiBfs`` over the job's collective backend (``ipc`` by default:
every rank is its own process, several may share one GPU), loads its shard
(``.bin`` shard read or on-device generation), answers the queries and writes
``rank<R>.json`` into the job's output directory.  Any failure is reported in
that file and by a non-zero exit status.
"""
from __future__ import annotations

import json
import os
import sys
import time
import traceback


def _result(r) -> dict:
    return {"hops": int(r.hops), "found": bool(r.found), "path": [int(v) for v in r.path], "stats": r.stats,
            "total_ms": float(r.total_ms)}


def main(job_path: str, rank: int) -> int:
    with open(job_path) as f:
        job = json.load(f)
    out_path = os.path.join(job["out_dir"], f"rank{rank}.json")
    out = {"rank": rank, "pid": os.getpid()}
    try:
        if os.environ.get("BIBFS_PROC_TORCH", "1") != "0":
            import torch  # noqa: F401  (binds the HIP runtime first, as every GPU test does)

            if os.environ.get("BIBFS_PROC_TORCH", "1") == "2":  # also a torch device context (as bench.py)
                torch.cuda.set_device(int(job["device"]))
                torch.cuda.synchronize()

        from .. import native
        from ..ops import make_options
        from . import make_tuning

        eng = native.DistBiBfs(rank, int(job["size"]), int(job["device"]), bytes.fromhex(job["uid"]),
                               job.get("backend", "ipc"))
        # the first run's tuning holds for the build too (hbm_cap_bytes, timeout_s)
        eng.set_tuning(make_tuning(**(job["runs"][0].get("tuning") or {})))
        fault = job.get("fault")
        if fault and int(fault[0]) == rank:
            eng.inject_fault(int(fault[1]), int(fault[2]))
        t0 = time.perf_counter()
        g = job["graph"]
        if "bin" in g:
            eng.load_bin(g["bin"])
        else:
            from ..models import parse_spec

            kind, n, arg, seed = parse_spec(g["spec"])
            if kind == "gnp":
                eng.generate_gnp(n, float(arg), seed)
            else:
                eng.generate_rmat(n, int(arg), seed)
        out["build_ms"] = (time.perf_counter() - t0) * 1e3
        out["local_nnz"] = int(eng.local_nnz)
        out["shard_bytes"] = int(eng.shard_bytes)
        out["gen_peak_bytes"] = int(eng.gen_peak_bytes)
        out["resident_bytes"] = int(eng.resident_bytes)
        out["owned"] = [int(eng.lo), int(eng.hi)]
        out["backend"] = eng.backend
        verify = int(job.get("verify", 0))
        runs = []
        for run in job["runs"]:  # option / tuning sets, all on the same shards
            if run.get("tuning") is not None:
                eng.set_tuning(make_tuning(**run["tuning"]))
            o = dict(run.get("options", {}))
            catch = bool(o.pop("_catch", False))  # a failing query is recorded (hops -3) and the run goes on
            opt = make_options(**o)
            res, stats, valid, uni, qms = [], [], [], [], []
            for qi, (s, d) in enumerate(job["queries"]):
                if s >= eng.n or d >= eng.n:  # fails on every rank before any collective
                    try:
                        eng.search(int(s), int(d), opt)
                    except Exception:  # noqa: BLE001
                        res.append({"hops": -2, "found": False, "path": [], "stats": {}, "total_ms": 0.0})
                        stats.append({})
                        continue
                    raise RuntimeError("an out-of-range query did not raise")
                q0 = time.perf_counter()
                try:
                    r = eng.search(int(s), int(d), opt)
                except Exception as e:  # noqa: BLE001
                    if not catch:
                        raise
                    res.append({"hops": -3, "found": False, "path": [], "stats": {}, "total_ms": 0.0,
                                "error": str(e)})
                    stats.append({})
                    continue
                qms.append((time.perf_counter() - q0) * 1e3)
                res.append(_result(r))
                stats.append(eng.last_stats)
                if verify:
                    valid.append((1 if eng.validate_path(int(s), int(d), int(r.hops), list(r.path)) else 0)
                                 if r.found else -1)
                    uni.append(int(eng.search_unidirectional(int(s), int(d)).hops) if qi < verify else -2)
            runs.append({"results": res, "last_stats": stats, "path_valid": valid, "uni_hops": uni, "query_ms": qms})
        out["runs"] = runs
        eng.barrier()
        del eng
        rc = 0
    except BaseException as e:  # noqa: BLE001
        out["error"] = f"{type(e).__name__}: {e}"
        out["traceback"] = traceback.format_exc()
        sys.stderr.write(f"[rank {rank}] {out['error']}\n")
        rc = 3
    tmp = out_path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(out, f)
    os.replace(tmp, out_path)
    sys.stdout.flush()
    sys.stderr.flush()
    return rc


if __name__ == "__main__":
    # exit without tearing the interpreter down through the HIP runtime's
    # atexit handlers twice: the engine is already destroyed above
    os._exit(main(sys.argv[1], int(sys.argv[2])))
