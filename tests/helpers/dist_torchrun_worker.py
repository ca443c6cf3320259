"""One rank of the multi-GPU correctness gate (tests/test_gpu_multi.py).

Launched by torch.distributed.run, one rank per GPU: checks the local-rank ->
device mapping, builds the partitioned engine through the torch.distributed
bootstrap (RCCL communicator of WORLD_SIZE ranks) on G(1M) and Kronecker-16,
and compares every answer with the host oracle.  Rank 0 prints one JSON line.

BIBFS_TEST_BACKEND=ipc: the ranks may outnumber the GPUs (they share them
round-robin); the process group is gloo and the engine's collectives go over
the HIP-IPC transport (tests/test_gpu_dist_proc.py).
"""
import json
import os
import random
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bidirectional_bfs_amd as bb  # noqa: E402
from bidirectional_bfs_amd import native  # noqa: E402
from bidirectional_bfs_amd.parallel import DistEngine  # noqa: E402


def main():
    backend = os.environ.get("BIBFS_TEST_BACKEND", "rccl")
    local = int(os.environ["LOCAL_RANK"])
    device = local % torch.cuda.device_count() if backend == "ipc" else local
    torch.cuda.set_device(device)
    if backend == "ipc":
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    assert torch.cuda.current_device() == device
    eng = DistEngine.from_torch_distributed(device, backend=backend)
    assert eng.world == world and eng.rank == rank and eng.backend == backend, (eng.world, eng.rank, eng.backend)
    checked, bad = 0, []
    for spec in ("gnp:1000000::2", "kron:16:16:3"):
        g = bb.from_spec(spec)  # host copy for the oracle (same edges as the device generator)
        kind, n, arg, seed = bb.models.parse_spec(spec)
        if kind == "gnp":
            eng.generate_gnp(n, arg, seed)
        else:
            eng.generate_rmat(n, int(arg), seed)
        per = -(-n // world)
        chunk = max(64, -(-per // 64) * 64)  # 1-D block partition, 64-aligned (dist_engine.hpp)
        assert eng.owned == (min(rank * chunk, n), min((rank + 1) * chunk, n)), eng.owned
        rnd = random.Random(7)
        qs = [(0, n - 1), (5, 5)] + [(rnd.randrange(n), rnd.randrange(n)) for _ in range(12)]
        for s, d in qs:
            r = eng.search(s, d)
            o = native.bfs_oracle(g.csr, s, d)
            ok = r.hops == o.hops
            if ok and r.found:
                ok, _ = native.validate_path(g.csr, s, d, r.hops, r.path)
            checked += 1
            if not ok:
                bad.append((spec, s, d, int(r.hops), int(o.hops)))
        eng.release()
    flag = torch.tensor([len(bad)], device="cuda" if backend != "ipc" else "cpu")
    dist.all_reduce(flag)
    if rank == 0:
        print(json.dumps({"world": world, "backend": backend, "checked": checked, "bad_total": int(flag.item()),
                          "bad": bad[:4]}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
