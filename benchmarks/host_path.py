#!/usr/bin/env python3
"""Where a 100k serving query's time goes on the host side.

`HipEngine.query` on the tiny resident server (bench.py's timed call), with
the engine's host-path stamps on (HipBiBfs::set_host_stamps): steady-clock
marks at entry, request posted, first answer packet seen, every packet read,
return -- beside the Python-level time of the whole call and the device time
(request seen -> answer written, s_memrealtime).  The remainder
(python_call_us - the stamped parts) is the Python wrapper + pybind11 +
the path list; wait_first_packet_us - device_us is the mailbox round trip
(request over PCIe to the polling wave, answer packets back).

    python benchmarks/host_path.py [--graph gnp:100000::6] [--reps 30]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="gnp:100000::6")
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)

    import bench
    from bidirectional_bfs_amd.ops import HipEngine

    _, n, _, _ = bench.parse_spec(a.graph)
    eng = bench.generate(HipEngine(0), a.graph)
    eng.set_resident(True)
    pairs = bench.pick_pairs(eng, n, a.pairs, 12345)
    for s, d, _ in pairs[:16]:
        eng.query(s, d)
    for stamps in (False, True):
        eng._e.set_host_stamps(stamps)
        t_all, dev = [], []
        for _ in range(a.reps):
            for s, d, h in pairs:
                t0 = time.perf_counter()
                hh, path = eng.query(s, d)
                t_all.append(time.perf_counter() - t0)
                dev.append(eng.last_search_ms)
                assert hh == h and len(path) == h + 1
        rec = {"graph": a.graph, "host_stamps": stamps, "queries": len(t_all),
               "python_call_us": round(statistics.fmean(t_all) * 1e6, 3),
               "python_call_us_median": round(statistics.median(t_all) * 1e6, 3),
               "device_us": round(statistics.fmean(dev) * 1e3, 3)}
        if stamps:
            hs = eng._e.host_stamps()
            rec.update({k: round(v, 3) if isinstance(v, float) else v for k, v in hs.items()})
            native_us = hs["post_us"] + hs["wait_first_packet_us"] + hs["read_packets_us"] + hs["return_us"]
            rec["native_us"] = round(native_us, 3)
            rec["python_binding_list_us"] = round(rec["python_call_us"] - native_us, 3)
            rec["mailbox_and_publish_us"] = round(hs["wait_first_packet_us"] - rec["device_us"], 3)
        print(json.dumps(rec), flush=True)
    eng._e.set_host_stamps(False)
    eng.set_resident(False)
    eng.release()


if __name__ == "__main__":
    main()
