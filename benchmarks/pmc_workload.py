#!/usr/bin/env python3
"""Fixed workload for rocprofv3 counter passes: 200 one-shot queries on the
100k G(n,p) bench graph (LDS engine) and 8 on Kronecker scale 22 (grid
top-down / bottom-up kernels)."""
import os
import random
import sys

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bidirectional_bfs_amd.ops import HipEngine  # noqa: E402

eng = HipEngine(0)
eng.generate_gnp(100000, 2.2000000001 / 100000, 6)
rnd = random.Random(5)
for i in range(200):
    eng.search(0, 99999) if i % 2 == 0 else eng.search(rnd.randrange(100000), rnd.randrange(100000))
eng.release()
eng.generate_rmat(1 << 22, 16 << 22, 1)
for i in range(8):
    eng.search(rnd.randrange(1 << 22), rnd.randrange(1 << 22))
print("pmc workload done", flush=True)
