"""The root merge on the device (k_merge_lists, the RCCL path's compute_global_top_k,
src/mpi_helpers/metrics.rs:141-171) against the host merge (merge.cpp, itself checked against
the oracle in test_abi.py) and the oracle: bsr_global_top_k with every array in device memory."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device_merge(bsr_mod, li, ld, lc, k):
    import torch
    P, Q, k_in = li.shape
    d_i = torch.from_numpy(li.view(np.int64)).cuda()
    d_d = torch.from_numpy(ld).cuda()
    d_c = torch.from_numpy(lc.view(np.int32)).cuda()
    o_i = torch.empty((Q, k), dtype=torch.int64, device="cuda")
    o_d = torch.empty((Q, k), dtype=torch.float32, device="cuda")
    o_c = torch.empty(Q, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    st = bsr_mod.lib().bsr_global_top_k(d_i.data_ptr(), d_d.data_ptr(), d_c.data_ptr(), P, Q, k_in, k,
                                        o_i.data_ptr(), o_d.data_ptr(), o_c.data_ptr())
    if st != 0:
        raise bsr_mod.BsrError(st, bsr_mod.lib().bsr_last_error().decode())
    return (o_i.cpu().numpy().view(np.uint64), o_d.cpu().numpy(), o_c.cpu().numpy().view(np.uint32))


def _assert_same(a, b):
    ai, ad, ac = a
    bi, bd, bc = b
    assert np.array_equal(ac, bc)
    assert np.array_equal(ai, bi)
    assert np.array_equal(ad.view(np.uint32), bd.view(np.uint32))


def _random_lists(rng, P, Q, k_in, sorted_=True, overlap=True, signed_zero=False):
    vals = np.linspace(0, 1, 40, dtype=np.float32)  # few distinct distances: many ties
    ld = rng.choice(vals, (P, Q, k_in)).astype(np.float32)
    if signed_zero:
        z = rng.random((P, Q, k_in)) < 0.2
        ld[z] = np.where(rng.random(z.sum()) < 0.5, np.float32(-0.0), np.float32(0.0))
    if sorted_:
        ld = np.sort(ld, axis=2)
    span = 30 if overlap else 1_000_000
    li = (np.arange(P, dtype=np.uint64)[:, None, None] * (0 if overlap else span)
          + rng.integers(0, span, (P, Q, k_in)).astype(np.uint64))
    lc = rng.integers(0, k_in + 1, (P, Q)).astype(np.uint32)
    lc[rng.random((P, Q)) < 0.05] = k_in + 7  # counts above k_in read as k_in
    return li, ld, lc


@pytest.mark.parametrize("P", [1, 2, 3, 8])
@pytest.mark.parametrize("sorted_", [True, False])
def test_device_merge_matches_host(bsr_mod, P, sorted_):
    rng = np.random.default_rng(1000 + 10 * P + sorted_)
    for k_in, k in ((10, 10), (10, 4), (4, 16), (50, 50)):
        for overlap in (False, True):
            li, ld, lc = _random_lists(rng, P, 257, k_in, sorted_, overlap, signed_zero=True)
            _assert_same(_device_merge(bsr_mod, li, ld, lc, k), bsr_mod.merge_top_k_lists(li, ld, lc, k))


@pytest.mark.parametrize("P,k", [(8, 100), (4, 256), (64, 16)])
def test_device_merge_largest_lists(bsr_mod, P, k):
    rng = np.random.default_rng(7 + P)
    li, ld, lc = _random_lists(rng, P, 64, k, True, True)
    _assert_same(_device_merge(bsr_mod, li, ld, lc, k), bsr_mod.merge_top_k_lists(li, ld, lc, k))


def test_device_merge_vs_oracle(bsr_mod, oracle_mod):
    """Rank lists of the oracle over interval_by_rank blocks, cross-rank ties included."""
    rng = np.random.default_rng(5)
    rows = rng.uniform(-1, 1, (300, 24)).astype(np.float32)
    rows[250] = rows[3]
    rows[150:170] = rows[10]
    qs = rng.uniform(-1, 1, (6, 24)).astype(np.float32)
    qs[0] = rows[3]
    for P in (2, 5, 8):
        for k in (1, 10):
            li = np.zeros((P, len(qs), k), np.uint64)
            ld = np.zeros((P, len(qs), k), np.float32)
            lc = np.zeros((P, len(qs)), np.uint32)
            for r in range(P):
                for q in range(len(qs)):
                    i, d = oracle_mod.local_top_k(rows, r, P, k, qs[q])
                    li[r, q, :len(i)], ld[r, q, :len(d)], lc[r, q] = i, d, len(i)
            oi, od, oc = _device_merge(bsr_mod, li, ld, lc, k)
            wi, wd, wc = oracle_mod.parallel_top_k(rows, qs, k, size=P)
            assert np.array_equal(oc, wc)
            for q in range(len(qs)):
                c = int(wc[q])
                assert np.array_equal(oi[q, :c], wi[q, :c])
                assert np.array_equal(od[q, :c].view(np.uint32), wd[q, :c].view(np.uint32))
                assert (oi[q, c:] == np.uint64(2**64 - 1)).all() and np.isinf(od[q, c:]).all()


def test_device_merge_nan_is_an_error(bsr_mod):
    li = np.zeros((2, 3, 2), np.uint64)
    ld = np.full((2, 3, 2), 0.5, np.float32)
    ld[1, 2, 1] = np.nan
    ld[0, 1, 0] = np.nan
    lc = np.full((2, 3), 2, np.uint32)
    with pytest.raises(bsr_mod.BsrError) as e:
        _device_merge(bsr_mod, li, ld, lc, 2)
    assert e.value.status == -2 and "query 1" in str(e.value)


def test_device_merge_rejects_mixed_memory(bsr_mod):
    import torch
    li = torch.zeros((1, 1, 2), dtype=torch.int64, device="cuda")
    ld = torch.zeros((1, 1, 2), dtype=torch.float32, device="cuda")
    lc = torch.full((1, 1), 2, dtype=torch.int32, device="cuda")
    oi = np.empty((1, 2), np.uint64)
    od = np.empty((1, 2), np.float32)
    oc = np.empty(1, np.uint32)
    st = bsr_mod.lib().bsr_global_top_k(li.data_ptr(), ld.data_ptr(), lc.data_ptr(), 1, 1, 2, 2,
                                        oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
    assert st != 0


def test_host_merge_rejects_device_lists(bsr_mod):
    """Host counts with device lists or outputs: rejected (BSR_E_INVALID), never
    dereferenced on the CPU."""
    import torch
    li = torch.zeros((1, 1, 2), dtype=torch.int64, device="cuda")
    ld = torch.zeros((1, 1, 2), dtype=torch.float32, device="cuda")
    lc = np.full((1, 1), 2, np.uint32)
    oi = np.empty((1, 2), np.uint64)
    od = np.empty((1, 2), np.float32)
    oc = np.empty(1, np.uint32)
    st = bsr_mod.lib().bsr_global_top_k(li.data_ptr(), ld.data_ptr(), lc.ctypes.data, 1, 1, 2, 2,
                                        oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
    assert st == -1
    hi = np.zeros((1, 1, 2), np.uint64)
    hd = np.zeros((1, 1, 2), np.float32)
    doi = torch.empty((1, 2), dtype=torch.int64, device="cuda")
    st = bsr_mod.lib().bsr_global_top_k(hi.ctypes.data, hd.ctypes.data, lc.ctypes.data, 1, 1, 2, 2,
                                        doi.data_ptr(), od.ctypes.data, oc.ctypes.data)
    assert st == -1
