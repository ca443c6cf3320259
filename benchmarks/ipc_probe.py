"""Which HIP runtime setups let two processes on one GPU map each other's
staging buffers (csrc/dist/ipc_comm.hip)?  Runs a 2-process dist_proc_run on a
small graph per setup and prints one JSON line each:
  torch   -- workers import torch first (torch's bundled HIP runtime)
  rocm    -- workers do not import torch (/opt/rocm's HIP runtime via rpath)
  mpi     -- mpi_bibfs --comm ipc under mpiexec (/opt/rocm runtime)
"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bidirectional_bfs_amd as bb  # noqa: E402
from bidirectional_bfs_amd.parallel import MPIEXEC, dist_proc_launch  # noqa: E402


def main():
    g = bb.from_spec("gnp:20000::6")
    qs = [(0, g.n - 1), (3, 77)]
    for mode, env in (("rocm", {"BIBFS_PROC_TORCH": "0"}), ("torch", {"BIBFS_PROC_TORCH": "1"})):
        rcs, outs, el = dist_proc_launch(2, g, qs, env=env, timeout=120)
        print(json.dumps({"mode": mode, "rcs": rcs, "elapsed_s": round(el, 2),
                          "errors": [o.get("error") for o in outs],
                          "hops": [[r["hops"] for r in o["runs"][0]["results"]] if "runs" in o else None
                                   for o in outs]}), flush=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([MPIEXEC, "-n", "2", os.path.join(root, "build", "bin", "mpi_bibfs"), "gnp:20000::6", "0",
                        "19999", "--comm", "ipc", "--verify"], capture_output=True, text=True, timeout=120)
    print(json.dumps({"mode": "mpi", "rc": r.returncode, "out": r.stdout[-300:], "err": r.stderr[-300:]}), flush=True)


if __name__ == "__main__":
    main()
