"""CPU model of the device-ordered exchange (csrc/dist/dist_engine.hip: DevSync,
dev_sync_wait, k_dev_barrier; docs/DESIGN.md §4.3).

Each rank is a thread that runs the protocol's rounds in stream order:

* expand(e): write this rank's owner blocks into its window half e & 1;
* claim(e):  raise this rank's flag to e, wait until every peer's flag is >= e,
             then read every peer's half e & 1 in place;
* after the last round of a search: a barrier epoch (flag raised, all waited).

Random delays stand in for the ranks' independent streams.  Every half
carries the epoch that last wrote it and a checksum of its payload, and a
reader asserts that the half it reads holds exactly round e's bytes: the
flag wait must order it after the writer's expand(e), and no writer may have
moved on to e + 2 (the same half) while it reads.  A single-buffered window
(one half) fails the same check under an adversarial schedule, which shows
the check can see the race the parity avoids.
"""
import random
import threading
import time

import pytest


class Window:
    def __init__(self, halves):
        self.flag = 0
        self.halves = [(0, None) for _ in range(halves)]  # (epoch, payload)


def run_model(ranks, searches, rounds_per_search, halves=2, seed=0, adversary=False):
    wins = [Window(halves) for _ in range(ranks)]
    errors = []
    lock = threading.Lock()  # (only guards the errors list)

    def payload(r, e, owner):
        return (r, e, owner, (r * 1000003 + e * 7919 + owner) & 0xffffffff)

    def rank_main(r):
        rnd = random.Random(seed * 97 + r)
        e = 0

        def jitter(scale=1.0):
            if adversary and r == 0:
                time.sleep(0.002 * scale)  # rank 0 lags: a single half gets rewritten under it
            elif rnd.random() < 0.3:
                time.sleep(rnd.random() * 0.0005 * scale)

        def wait_all(epoch):
            t0 = time.monotonic()
            for p in range(ranks):
                while wins[p].flag < epoch:
                    if time.monotonic() - t0 > 20:
                        raise TimeoutError(f"rank {r} waited for rank {p} at epoch {epoch}")
                    time.sleep(0)

        for _ in range(searches):
            for _ in range(rounds_per_search):
                e += 1
                jitter()
                # expand(e): this rank's blocks for every owner into half e % halves
                wins[r].halves[e % halves] = (e, [payload(r, e, o) for o in range(ranks)])
                jitter()
                # claim(e): raise own flag (the expand is complete: stream order), wait, read
                wins[r].flag = e
                wait_all(e)
                for p in range(ranks):
                    jitter(0.2)
                    got_e, blocks = wins[p].halves[e % halves]
                    if got_e != e or blocks[r] != payload(p, e, r):
                        with lock:
                            errors.append((r, p, e, got_e))
            # k_dev_barrier: one more epoch, nobody reads
            e += 1
            wins[r].flag = e
            wait_all(e)

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(ranks)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not any(t.is_alive() for t in threads), "a rank hung (flag protocol deadlock)"
    return errors


@pytest.mark.parametrize("ranks", [2, 3, 4])
def test_double_buffered_window_never_reads_a_stale_or_rewritten_half(ranks):
    errors = run_model(ranks, searches=6, rounds_per_search=12, halves=2, seed=ranks)
    assert errors == []


def test_double_buffered_window_survives_a_lagging_reader():
    assert run_model(3, searches=2, rounds_per_search=10, halves=2, seed=5, adversary=True) == []


def test_single_buffered_window_shows_the_race():
    """The same check over ONE half with a reader that lags: a fast writer
    rewrites the half for the next epoch while the slow rank still reads it --
    the race the two halves rule out (the check is not vacuous)."""
    errors = run_model(3, searches=2, rounds_per_search=10, halves=1, seed=5, adversary=True)
    assert errors, "expected the single-buffered window to expose a rewritten half"
