"""Multi-GPU and multi-process execution (v2 / v4 capabilities).

* ``DistEngine``: one process per GPU, graph 1-D partitioned, every per-level
  exchange an RCCL collective over xGMI (native ``DistBiBfs``).  The round
  policy runs on the device and the host enqueues several rounds per wait
  (``DistTuning.spec_rounds``); dense or oversized levels are planned by the
  host, where one side's exchange overlaps the other side's expand.  The RCCL
  communicator is bootstrapped from a unique id broadcast over
  ``torch.distributed`` (``from_torch_distributed``) or over MPI by the
  ``mpi_bibfs`` CLI.  An error or a watchdog timeout on any rank aborts the
  communicator (``ncclCommAbort``) so no peer is left hanging.
* ``dist_proc_run``: the same native engine with P ranks as P separate
  PROCESSES, exchanging over the HIP-IPC transport (``backend="ipc"``,
  csrc/dist/ipc_comm.hip).  The processes may share one GPU -- the
  reference's own v4 launch, 4 MPI ranks on one machine's GPU
  (single_machine_bench.sh:9,52) -- or sit on different GPUs, where the same
  transport reads peer HBM over xGMI.
* ``dist_local_run``: the same native engine with P ranks as P threads on ONE
  GPU, exchanging through an in-process group instead of RCCL -- how the
  partition / exchange logic is tested with P > 1 on a one-GPU box.
* ``ReplicatedServer``: query-parallel serving -- every GPU holds the whole
  graph (a 10M-vertex graph is ~0.2 GB of a 288 GB HBM3E part) and answers its
  own share of queries; throughput scales with the number of GPUs.
* ``run_mpi``: launch the CPU MPI engines (``second_try`` = C3,
  ``mpi_queue_bibfs`` = C4) or ``mpi_bibfs`` under ``mpiexec``.
"""
from __future__ import annotations

import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time
from typing import List, Optional, Sequence

from .._lib import native, tool_path
from ..models import Graph, parse_spec
from ..ops import _DEFAULT_OPTIONS, HipEngine, make_options

MPIEXEC = os.environ.get("BIBFS_MPIEXEC", "/opt/conda/bin/mpiexec")


def gpu_count() -> int:
    """Visible HIP devices (0 without a GPU), from the native library."""
    return int(native.gpu_count())


def make_tuning(spec_rounds: Optional[int] = None, spec_cap_max: Optional[int] = None, cap: Optional[int] = None,
                nosync_bytes: Optional[int] = None, timeout_s: Optional[float] = None,
                walk_max: Optional[int] = None, solo: Optional[bool] = None,
                solo_edges: Optional[int] = None, owner_cap: Optional[int] = None,
                pipeline: Optional[bool] = None, spec_stall_edges: Optional[int] = None,
                stamps: Optional[bool] = None, hbm_cap_bytes: Optional[int] = None,
                world1_single: Optional[bool] = None, spill_cap: Optional[int] = None,
                dev_sync: Optional[bool] = None) -> "native.DistTuning":
    """Knobs of the partitioned engine; unset ones keep the production default.

    solo (one rank only): run the small rounds in one persistent workgroup
    (k_spec_solo) instead of one multi-workgroup launch per round, while each
    expanding side has at most ``solo_edges`` frontier edges (one CU's
    gather rate caps what it should take on; <= 8192).

    owner_cap (more than one rank): pairs per owner-addressed candidate block
    of a speculative round (0 = predicted per round from the last per-owner
    counts); candidates that do not fit are re-offered by a continuation round.

    pipeline (more than one rank, default on): ONE collective per speculative
    round -- each round's reduction travels in the header of the next round's
    candidate exchange, and each plan accounts the round before the last one
    (a finished search runs one extra round); the first stall (a spill, a big
    or dense frontier) drains the pipeline and the search goes on with exact
    plans.  Off: exact plans, a status allgather per round.

    stamps: per-round device stamps; ``last_stats`` then splits the
    speculative rounds into ``expand_us`` / ``claim_us`` (kernels) and
    ``exchange_us`` / ``status_us`` (the gaps the two collectives and the
    launches leave), summed over ``stamped_rounds``.  Diagnostics: one extra
    host wait and a copy per search.

    hbm_cap_bytes: a build that would make a rank hold more device memory
    than this throws (rehearses "does not fit one GPU" at small scale).

    spill_cap (test hook, 0 = the allocation): a smaller candidate spill
    list, so a round overflows it -- the search then raises on every rank
    and the group keeps serving.

    world1_single (default on): with ONE rank the shard is the whole graph,
    so queries are answered by the single-GPU engine over the same device CSR
    (no copy); off = the partitioned rounds (solo workgroup) at world size 1.

    dev_sync (default on; IPC ranks that share one GPU): a round's claim
    kernel waits for the peers' expansions on their flags in a device window
    instead of a host rendezvous (no effect on other transports)."""
    t = native.DistTuning()
    for k, v in (("spec_rounds", spec_rounds), ("spec_cap_max", spec_cap_max), ("cap", cap),
                 ("nosync_bytes", nosync_bytes), ("timeout_s", timeout_s), ("walk_max", walk_max),
                 ("solo", solo), ("solo_edges", solo_edges), ("owner_cap", owner_cap), ("pipeline", pipeline),
                 ("spec_stall_edges", spec_stall_edges), ("stamps", stamps), ("hbm_cap_bytes", hbm_cap_bytes),
                 ("world1_single", world1_single), ("spill_cap", spill_cap), ("dev_sync", dev_sync)):
        if v is not None:
            setattr(t, k, v)
    return t


class DistEngine:
    """Partitioned multi-GPU bidirectional BFS (collective API: call on every rank)."""

    def __init__(self, rank: int, world: int, device: int, unique_id: bytes, backend: str = "rccl"):
        self._e = native.DistBiBfs(int(rank), int(world), int(device), unique_id, backend)
        # the serving call goes straight to the native method (no Python frame
        # per query, as HipEngine.query); `query` below documents it
        self.query = self._e.query

    @staticmethod
    def unique_id(backend: str = "rccl") -> bytes:
        return native.dist_unique_id(backend)

    @classmethod
    def from_torch_distributed(cls, device: Optional[int] = None, backend: str = "rccl") -> "DistEngine":
        """Bootstrap from an initialised torch.distributed process group.

        backend "rccl": one rank per GPU; "ipc": the HIP-IPC transport, where
        several ranks may share a GPU (device defaults to LOCAL_RANK modulo
        the visible GPUs)."""
        import torch.distributed as dist

        rank, world = dist.get_rank(), dist.get_world_size()
        if backend == "ipc":
            # The IPC control plane is node-local shared memory with peer
            # liveness checked by local pid: every rank must share one host.
            hosts = [None] * world
            dist.all_gather_object(hosts, socket.gethostname())
            if len(set(hosts)) != 1:
                raise RuntimeError(f"backend 'ipc' needs all {world} ranks on one node, got hosts "
                                   f"{sorted(set(hosts))}; use backend 'rccl' (one rank per GPU)")
        obj = [native.dist_unique_id(backend) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", rank))
            if backend == "ipc":
                device %= max(1, gpu_count())
        return cls(rank, world, device, obj[0], backend)

    def query(self, src: int, dst: int):
        """Lean serving call: ``(hops, path)``, hops = -1 when unreachable
        (the stats stay in ``last_stats``, read outside any timed loop).  At
        world size 1 it is the single-GPU engine's own query (resident tiny /
        LDS server, GIL kept)."""
        return self._e.query(src, dst)

    def load(self, graph: Graph) -> "DistEngine":
        self._e.load_edges(graph.edges)
        return self

    def load_bin(self, path: str) -> "DistEngine":
        self._e.load_bin(path)
        return self

    def generate_gnp(self, n: int, p: Optional[float] = None, seed: int = 1) -> "DistEngine":
        self._e.generate_gnp(int(n), native.reference_p(int(n)) if p is None else float(p), int(seed))
        return self

    def generate_rmat(self, n: int, m: int, seed: int = 1) -> "DistEngine":
        self._e.generate_rmat(int(n), int(m), int(seed))
        return self

    def search(self, src: int, dst: int, options=None, **kw):
        if options is None:
            options = make_options(**kw) if kw else _DEFAULT_OPTIONS
        return self._e.search(int(src), int(dst), options)

    def barrier(self) -> None:
        self._e.barrier()

    def release(self) -> None:
        """Free this rank's graph shard and search state (the communicator stays)."""
        self._e.release()

    def set_tuning(self, tuning=None, **kw) -> "DistEngine":
        self._e.set_tuning(tuning if tuning is not None else make_tuning(**kw))
        return self

    def inject_fault(self, at: int, mode: int = 1) -> None:
        """Test hook: from round ``at`` on this rank throws (1) or stalls past the timeout (2)."""
        self._e.inject_fault(int(at), int(mode))

    @property
    def local_nnz(self) -> int:
        return self._e.local_nnz

    @property
    def shard_bytes(self) -> int:
        """Bytes of this rank's CSR shard (row offsets + columns)."""
        return self._e.shard_bytes

    @property
    def gen_peak_bytes(self) -> int:
        """Peak allocation of the last device generation on this rank: the
        shard plus one cursor array (the edge list is never materialised)."""
        return self._e.gen_peak_bytes

    @property
    def gen_hbm_peak_bytes(self) -> int:
        """The device's free-memory drop over the last build (hipMemGetInfo
        low-water mark); equals gen_peak_bytes up to allocator granularity
        with one rank per GPU."""
        return self._e.gen_hbm_peak_bytes

    @property
    def resident_bytes(self) -> int:
        """Device bytes this rank holds now (shard + search state)."""
        return self._e.resident_bytes

    def validate_path(self, src: int, dst: int, hops: int, path) -> bool:
        """Collective: each path edge looked up by the owner of its first
        vertex, one sum-allreduce (no copy of the graph anywhere)."""
        return bool(self._e.validate_path(int(src), int(dst), int(hops), [int(v) for v in path]))

    def search_unidirectional(self, src: int, dst: int):
        """Collective: a plain partitioned BFS from src (hop count only), an
        independent check of the bidirectional engine's distance."""
        return self._e.search_unidirectional(int(src), int(dst))

    def allreduce_max(self, x: float) -> float:
        return self._e.allreduce_max(float(x))

    @property
    def rank(self) -> int:
        return self._e.rank

    @property
    def world(self) -> int:
        return self._e.size

    @property
    def n(self) -> int:
        return self._e.n

    @property
    def m(self) -> int:
        return self._e.m_input

    @property
    def owned(self):
        return self._e.lo, self._e.hi

    @property
    def last_stats(self) -> dict:
        """Rounds, lockstep rounds, sparse / dense / overflow levels, exchanged bytes of the last search."""
        return self._e.last_stats

    @property
    def backend(self) -> str:
        return self._e.backend


def dist_local_run(ranks: int, graph: Graph, queries: Sequence, device: int = 0, options=None, tuning=None,
                   fault=None, return_stats: bool = False, **kw):
    """Partitioned native engine, ``ranks`` ranks as threads sharing one GPU (test harness).

    Every rank answers every query; the result list is rank 0's, after a check
    that all ranks agree.  ``tuning``: a ``native.DistTuning`` (see
    :func:`make_tuning`); ``fault``: ``(rank, at, mode)`` arms
    ``inject_fault`` on one rank.  With ``return_stats`` also returns rank 0's
    per-query ``last_stats`` dicts.
    """
    if options is None:
        options = make_options(**kw) if kw else _DEFAULT_OPTIONS
    q = [(int(s), int(d)) for s, d in queries]
    f = native.DistLocalFault()
    if fault is not None:
        f.rank, f.at, f.mode = (int(x) for x in fault)
    rs, st = native.dist_local_run(int(ranks), int(device), graph.edges, q, options,
                                   tuning if tuning is not None else native.DistTuning(), f)
    return (rs, st) if return_stats else rs


def dist_local_generate_run(ranks: int, spec: str, queries: Sequence, device: int = 0, options=None, tuning=None,
                            verify: int = 0, **kw):
    """Like :func:`dist_local_run`, but every rank generates ``spec``
    (``gnp:``/``rmat:``/``kron:``) on the device and keeps only its own CSR
    shard, as the multi-GPU bench does.  Returns ``(results, timing)`` with
    ``timing = {"build_ms", "query_ms": [rank 0 wall per query], "local_nnz": [per rank], ...}``.
    ``verify`` > 0: every found path is also checked collectively
    (``timing["path_valid"]``) and the first ``verify`` queries are re-run as
    a unidirectional partitioned BFS (``timing["uni_hops"]``).
    """
    if options is None:
        options = make_options(**kw) if kw else _DEFAULT_OPTIONS
    kind, n, arg, seed = parse_spec(spec)
    q = [(int(s), int(d)) for s, d in queries]
    return native.dist_local_generate_run(int(ranks), int(device), kind, n, float(arg), seed, q, options,
                                          tuning if tuning is not None else native.DistTuning(), int(verify))


class ProcResult:
    """One query's answer from :func:`dist_proc_run` (the fields of ``native.SearchResult`` the tests read)."""

    __slots__ = ("hops", "found", "path", "stats", "total_ms")

    def __init__(self, d: dict):
        self.hops, self.found, self.path = int(d["hops"]), bool(d["found"]), list(d["path"])
        self.stats, self.total_ms = d.get("stats", {}), float(d.get("total_ms", 0.0))

    def __repr__(self) -> str:
        return f"ProcResult(found={self.found}, hops={self.hops})"


class ProcRunError(RuntimeError):
    """A multi-process run failed; ``returncodes`` / ``outputs`` / ``elapsed_s`` say how."""

    def __init__(self, msg: str, returncodes, outputs, elapsed_s: float):
        super().__init__(msg)
        self.returncodes, self.outputs, self.elapsed_s = returncodes, outputs, elapsed_s


def dist_proc_launch(ranks: int, graph, queries: Sequence, runs: Sequence = ((None, None),), device: int = 0,
                     fault=None, verify: int = 0, backend: str = "ipc", timeout: float = 300.0, env=None):
    """Run the partitioned engine as ``ranks`` separate processes and return
    ``(returncodes, outputs, elapsed_s)``: ``outputs[r]`` is rank r's report
    (build sizes and ``runs[i] = {"results", "last_stats", ...}``, or
    ``error``).  ``graph`` is a :class:`Graph` (written once as ``.bin``;
    every rank reads only its shard) or a ``gnp:``/``rmat:``/``kron:`` spec
    (every rank generates its rows on its GPU).  ``runs``: ``(options,
    tuning)`` keyword dicts of :func:`make_options` / :func:`make_tuning`,
    each answering every query on the same shards (tuning None = keep the
    previous); ``fault``: ``(rank, round, mode)`` for ``inject_fault``
    (3 = that rank's process kills itself)."""
    tmp = tempfile.mkdtemp(prefix="bibfs_proc_")
    try:
        if isinstance(graph, str):
            gdesc = {"spec": graph}
        else:
            path = os.path.join(tmp, "graph.bin")
            graph.save_bin(path)
            gdesc = {"bin": path}
        job = {"size": int(ranks), "device": int(device), "uid": native.dist_unique_id(backend).hex(),
               "backend": backend, "graph": gdesc, "queries": [[int(s), int(d)] for s, d in queries],
               "runs": [{"options": dict(o or {}), "tuning": None if t is None else dict(t)} for o, t in runs],
               "fault": list(fault) if fault else None,
               "verify": int(verify), "out_dir": tmp}
        job_path = os.path.join(tmp, "job.json")
        with open(job_path, "w") as f:
            json.dump(job, f)
        e = dict(os.environ)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if int(ranks) > 1:
            # every rank on the one device: one hardware queue per process.  With
            # HIP's 4 each, the GPU time-slices the processes' queues: G(1M) at
            # 8 ranks 137-157 -> 1.4-2.2 ms per query, 4 ranks 0.54 -> 0.51 ms
            # (profiles/r6_hw_queues_procs.jsonl)
            e["GPU_MAX_HW_QUEUES"] = "1"
        if env:
            e.update(env)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
        t0 = time.monotonic()
        procs = [subprocess.Popen([sys.executable, "-m", "bidirectional_bfs_amd.parallel._proc_worker", job_path,
                                   str(r)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e)
                 for r in range(int(ranks))]
        logs = []
        for p in procs:
            left = max(1.0, timeout - (time.monotonic() - t0))
            try:
                logs.append(p.communicate(timeout=left)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                logs.append(p.communicate()[0])
        elapsed = time.monotonic() - t0
        rcs = [p.returncode for p in procs]
        outs = []
        for r in range(int(ranks)):
            fp = os.path.join(tmp, f"rank{r}.json")
            if os.path.exists(fp):
                with open(fp) as f:
                    outs.append(json.load(f))
            else:
                outs.append({"rank": r, "error": f"no report (exit status {rcs[r]})"})
            outs[-1]["log"] = (logs[r] or "")[-4000:]
        return rcs, outs, elapsed
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def dist_proc_matrix(ranks: int, graph, queries: Sequence, runs: Sequence, device: int = 0, verify: int = 0,
                     backend: str = "ipc", timeout: float = 300.0):
    """Every ``(options, tuning)`` of ``runs`` over the same ``ranks``-process
    group (see :func:`dist_proc_launch`).  Returns ``[(results, last_stats,
    run_report)]`` per run -- rank 0's, after checking that every rank
    returned the same hop counts and paths -- and the per-rank reports."""
    rcs, outs, elapsed = dist_proc_launch(ranks, graph, queries, runs, device, None, verify, backend, timeout)
    if any(rcs):
        errs = "; ".join(f"rank {o.get('rank')}: {o.get('error', '')}" for o in outs if o.get("error"))
        raise ProcRunError(f"dist_proc_run failed (exit statuses {rcs}): {errs}", rcs, outs, elapsed)
    got = []
    for i, run0 in enumerate(outs[0]["runs"]):
        for o in outs[1:]:
            for a, b in zip(run0["results"], o["runs"][i]["results"]):
                if a["hops"] != b["hops"] or a["path"] != b["path"]:
                    raise ProcRunError("dist_proc_run: ranks returned different results", rcs, outs, elapsed)
        got.append(([ProcResult(d) for d in run0["results"]], run0["last_stats"], run0))
    return got, outs


def dist_proc_run(ranks: int, graph, queries: Sequence, device: int = 0, options: Optional[dict] = None,
                  tuning: Optional[dict] = None, return_stats: bool = False, verify: int = 0,
                  backend: str = "ipc", timeout: float = 300.0, **kw):
    """Like :func:`dist_local_run`, with every rank its own process.  Returns
    rank 0's results; with ``return_stats`` also its per-query
    ``last_stats`` and the per-rank reports."""
    opts = dict(options or {})
    opts.update(kw)
    got, outs = dist_proc_matrix(ranks, graph, queries, [(opts, tuning or {})], device, verify, backend, timeout)
    rs, st, _ = got[0]
    return (rs, st, outs) if return_stats else rs


class ReplicatedServer:
    """Query-parallel serving: rank r answers queries r, r+W, r+2W, ... on its own GPU."""

    def __init__(self, rank: int, world: int, device: int):
        self.rank, self.world = int(rank), int(world)
        self.engine = HipEngine(device)

    def load(self, graph: Graph) -> "ReplicatedServer":
        self.engine.load(graph)
        return self

    def my_queries(self, pairs: Sequence) -> List:
        return list(pairs[self.rank :: self.world])

    def serve(self, pairs: Sequence, options=None) -> List:
        return [self.engine.search(s, d, options) for s, d in self.my_queries(pairs)]


def run_mpi(tool: str, args: Sequence[str], np: int = 2, timeout: float = 300.0, env=None) -> subprocess.CompletedProcess:
    """Run a native MPI tool (second_try, mpi_queue_bibfs, mpi_bibfs) under mpiexec."""
    cmd = [MPIEXEC, "-n", str(int(np)), tool_path(tool)] + [str(a) for a in args]
    e = dict(os.environ)
    if env:
        e.update(env)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)


__all__ = ["DistEngine", "ReplicatedServer", "dist_local_run", "dist_local_generate_run", "dist_proc_launch",
           "dist_proc_matrix", "dist_proc_run", "ProcResult", "ProcRunError", "make_tuning", "run_mpi", "MPIEXEC"]
