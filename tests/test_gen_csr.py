"""Generators (seeded, thread-count independent) and CSR construction."""
import numpy as np
import pytest

from bidirectional_bfs_amd import native


def test_gnp_deterministic_and_thread_independent():
    a = native.gen_gnp(20000, 3.0 / 20000, 9, threads=1).edges()
    b = native.gen_gnp(20000, 3.0 / 20000, 9, threads=7).edges()
    c = native.gen_gnp(20000, 3.0 / 20000, 10).edges()
    assert np.array_equal(a, b)
    assert not np.array_equal(a, c)


def test_gnp_structure_and_density():
    n, p = 50000, native.reference_p(50000)
    e = native.gen_gnp(n, p, 1).edges()
    assert (e[:, 0] < e[:, 1]).all()  # u < v, no self loops (networkx edge order)
    keys = e[:, 0].astype(np.int64) * n + e[:, 1]
    assert len(np.unique(keys)) == len(keys)  # simple graph
    expect = p * n * (n - 1) / 2
    assert abs(len(e) - expect) < 6 * np.sqrt(expect)


def test_gnp_extremes():
    assert native.gen_gnp(10, 0.0, 1).m == 0
    assert native.gen_gnp(10, 1.0, 1).m == 45
    assert native.gen_gnp(1, 0.5, 1).m == 0


def test_rmat_kronecker():
    el = native.gen_rmat(3000, 20000, 4)
    e = el.edges()
    assert el.m == 20000 and (e < 3000).all() and (e[:, 0] != e[:, 1]).all()
    assert np.array_equal(e, native.gen_rmat(3000, 20000, 4, threads=3).edges())
    k = native.gen_kronecker(10, 8, 2)
    assert k.n == 1024 and k.m == 8192
    deg = np.bincount(k.edges().ravel(), minlength=1024)
    assert deg.max() > 8 * deg.mean()  # skewed (power-law-ish) degrees


def test_csr_matches_scipy():
    from scipy.sparse import csr_matrix

    el = native.gen_gnp(3000, 0.002, 2)
    g = native.build_csr(el, sort_rows=True)
    e = el.edges().astype(np.int64)
    allv = np.vstack([e, e[:, ::-1]])
    A = csr_matrix((np.ones(len(allv)), (allv[:, 0], allv[:, 1])), shape=(3000, 3000))
    A.sort_indices()
    assert np.array_equal(g.row_off, A.indptr)
    assert np.array_equal(g.col, A.indices)
    assert g.nnz == 2 * el.m and g.m_input == el.m


def test_csr_dedup_and_self_loops():
    el = native.EdgeList.from_numpy(4, np.array([[0, 1], [1, 0], [2, 2], [1, 3], [0, 1]], dtype=np.uint32))
    g = native.build_csr(el, dedup=True)
    rows = [sorted(g.col[g.row_off[v]:g.row_off[v + 1]]) for v in range(4)]
    assert rows == [[1], [0, 3], [], [1]]
    g2 = native.build_csr(el)  # no dedup: multi-edges kept, self loop dropped
    assert g2.nnz == 8


@pytest.mark.parametrize("P", [1, 2, 3, 5])
def test_partition_rows_union(P):
    el = native.gen_gnp(1001, 0.005, 3)
    full = native.build_csr(el, sort_rows=True)
    cols = []
    for r in range(P):
        part = native.build_csr_rows(el, r, P)
        for i in range(part.n):
            cols.append(sorted(part.col[part.row_off[i]:part.row_off[i + 1]]))
    assert len(cols) == 1001
    assert cols == [sorted(full.col[full.row_off[v]:full.row_off[v + 1]]) for v in range(1001)]


def test_parse_spec_device_generator_args():
    from bidirectional_bfs_amd.models import parse_spec, reference_p

    assert parse_spec("kron:27") == ("rmat", 1 << 27, 16 << 27, 1)
    assert parse_spec("kron:20:8:3") == ("rmat", 1 << 20, 8 << 20, 3)
    assert parse_spec("rmat:65536:1048576:4") == ("rmat", 65536, 1048576, 4)
    kind, n, p, seed = parse_spec("gnp:100000::6")
    assert (kind, n, seed) == ("gnp", 100000, 6) and p == reference_p(100000)
    assert parse_spec("gnp:1000:0.01")[2] == 0.01
    import pytest

    with pytest.raises(ValueError):
        parse_spec("graph.bin")
