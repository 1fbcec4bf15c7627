"""f-1: the parquet vector store (lib/libbsr_vstore.so) against the reference's own tests
of PolarsVectorstore (src/vectorstore/polars.rs:256-394, restated one for one with the
fixture convention of src/utils.rs:8-35: 768-d U(-1,1) rows) and against parquet files laid
out as polars writes them (large_list, null rows, null elements, several row groups).
Host only: no GPU needed, except the last test (index load -> search vs the oracle)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

DIMENSION = 768  # src/utils.rs:8


def mock_embeddings(rng, n):
    return rng.uniform(-1.0, 1.0, (n, DIMENSION)).astype(np.float32)  # src/utils.rs:14-28


@pytest.fixture
def rng():
    return np.random.default_rng(1234)


# ---- src/vectorstore/polars.rs:256-394, one test each ---------------------------------
def test_new_vectorstore(bsr_mod, tmp_path, rng):
    store = bsr_mod.get_global_vstore(tmp_path, True)
    store.append_many(mock_embeddings(rng, 3))
    assert store.get_count() == 3


def test_append_vector(bsr_mod, tmp_path, rng):
    store = bsr_mod.get_global_vstore(tmp_path, True)
    sample = mock_embeddings(rng, 1)
    store.append_many(sample)
    store.append(mock_embeddings(rng, 1)[0])
    result = store.get_many(None)
    assert len(result) == 2
    assert np.array_equal(result[0], sample[0])


def test_append_many_vectors(bsr_mod, tmp_path, rng):
    store = bsr_mod.get_global_vstore(tmp_path, True)
    n = 3
    store.append_many(mock_embeddings(rng, n))
    new = mock_embeddings(rng, 2)
    store.append_many(new)
    result = store.get_many(bsr_mod.SliceArgs(n, len(new)))
    assert len(result) == 2
    assert np.array_equal(result[0], new[0]) and np.array_equal(result[1], new[1])


def test_read_slice(bsr_mod, tmp_path, rng):
    store = bsr_mod.get_global_vstore(tmp_path, True)
    sample = mock_embeddings(rng, 3)
    store.append_many(sample)
    result = store.get_many(bsr_mod.SliceArgs(1, 1))
    assert len(result) == 1 and np.array_equal(result[0], sample[1])
    result = store.get_many(None)
    assert len(result) == 3 and all(np.array_equal(result[i], sample[i]) for i in range(3))


def test_persist_and_reload(bsr_mod, tmp_path, rng):
    store = bsr_mod.get_global_vstore(tmp_path, True)
    sample = mock_embeddings(rng, 3)
    store.append_many(sample)
    extra = mock_embeddings(rng, 1)[0]
    store.append(extra)
    store.persist()
    new_store = bsr_mod.get_global_vstore(tmp_path, False)
    result = new_store.get_many(None)
    assert len(result) == 4
    assert np.array_equal(np.stack(result), np.vstack([sample, extra[None]]))


def test_empty_file_reload(bsr_mod, tmp_path):
    store = bsr_mod.get_global_vstore(tmp_path, True)
    with pytest.raises(bsr_mod.BsrError):
        store.reload(False)  # read_parquet creates an empty file; 0 rows without force is an error
    store.reload(True)
    assert store.get_count() == 0
    assert os.path.exists(os.path.join(tmp_path, "global.parquet"))


def test_large_dataset(bsr_mod, tmp_path, rng):
    store = bsr_mod.get_global_vstore(tmp_path, True)
    store.append_many(mock_embeddings(rng, 1000))
    assert len(store.get_many(bsr_mod.SliceArgs(0, 100))) == 100
    assert len(store.get_many(bsr_mod.SliceArgs(500, 200))) == 200
    assert len(store.get_many(None)) == 1000


# ---- files as polars writes them, and the slice / get semantics ------------------------
def write_polars_like(path, rows, *, large=True, row_group_size=None):
    """One "embeddings" column; rows: list of (None | list of float|None)."""
    typ = pa.large_list(pa.float32()) if large else pa.list_(pa.float32())
    pq.write_table(pa.table({"embeddings": pa.array(rows, type=typ)}), path,
                   row_group_size=row_group_size, compression="zstd")


def test_reads_polars_layout_with_nulls(bsr_mod, tmp_path, rng):
    data = mock_embeddings(rng, 10)
    rows = [list(map(float, r)) for r in data]
    rows[3] = None                      # null row: counted, dropped by get_many
    rows[6] = list(rows[6])
    rows[6][5] = None                   # null element: skipped (flatten)
    path = os.path.join(tmp_path, "global.parquet")
    write_polars_like(path, rows, row_group_size=4)
    store = bsr_mod.get_global_vstore(tmp_path, False)
    assert store.get_count() == 10
    got = store.get_many(None)
    assert len(got) == 9
    assert np.array_equal(got[2], data[2]) and np.array_equal(got[3], data[4])
    assert len(got[5]) == DIMENSION - 1 and np.array_equal(got[5], np.delete(data[6], 5))
    # a dense slab of the block needs every row to be 768 long
    with pytest.raises(bsr_mod.BsrError) as e:
        store.get_many_array(None)
    assert e.value.status == -6
    assert np.array_equal(store.get_many_array(bsr_mod.SliceArgs(0, 6)), np.delete(data[:6], 3, axis=0))


def test_slice_semantics_negative_and_clamped(bsr_mod, tmp_path, rng):
    data = mock_embeddings(rng, 7)
    store = bsr_mod.get_global_vstore(tmp_path, True)
    store.append_many(data)
    assert np.array_equal(np.stack(store.get_many(bsr_mod.SliceArgs(-3, 2))), data[4:6])
    assert np.array_equal(np.stack(store.get_many(bsr_mod.SliceArgs(5, 100))), data[5:])
    assert store.get_many(bsr_mod.SliceArgs(7, 1)) == []
    assert store.get_many(bsr_mod.SliceArgs(100, 5)) == []       # interval_by_rank's empty blocks
    # polars slice_offsets clamps start and stop independently
    assert store.get_many(bsr_mod.SliceArgs(-100, 2)) == []
    assert np.array_equal(np.stack(store.get_many(bsr_mod.SliceArgs(-100, 95))), data[:2])
    assert np.array_equal(store.get(6), data[6])
    with pytest.raises(bsr_mod.BsrError):
        store.get(7)                                             # "Index not found"


def test_missing_file_is_created_and_paths(bsr_mod, tmp_path):
    d = os.path.join(tmp_path, "a", "b")
    store = bsr_mod.get_local_vstore(d, 3, False)
    assert store.path.endswith(os.path.join("a", "b", "rank_3.parquet"))
    assert os.path.exists(store.path) and store.get_count() == 0
    assert pq.read_table(store.path).num_rows == 0


def test_persist_mixed_file_and_appended_rows_roundtrip(bsr_mod, tmp_path, rng):
    data = mock_embeddings(rng, 6)
    rows = [list(map(float, r)) for r in data[:4]]
    rows[1] = None
    write_polars_like(os.path.join(tmp_path, "global.parquet"), rows, large=False)
    store = bsr_mod.get_global_vstore(tmp_path, False)
    store.append_many(data[4:])
    store.persist()
    t = pq.read_table(os.path.join(tmp_path, "global.parquet"))
    assert t.num_rows == 6 and t.column("embeddings").null_count == 1
    again = bsr_mod.get_global_vstore(tmp_path, False)
    assert again.get_count() == 6
    assert np.array_equal(again.get_many_array(None), np.delete(data, 1, axis=0))


@pytest.mark.gpu
def test_index_load_vstore_blocks_search_like_reference(bsr_mod, oracle_mod, gpu, tmp_path, rng):
    # the rank's block of global.parquet into HBM (mpi_helpers/metrics.rs:23-33), P = 3
    # ranks, merged: identical to the oracle's whole-store search
    data = mock_embeddings(rng, 5000)
    store = bsr_mod.get_global_vstore(tmp_path, True)
    store.append_many(data)
    store.persist()
    qs = mock_embeddings(rng, 20)
    qs[0] = data[17]
    P, k = 3, 10
    li = np.zeros((P, 20, k), np.uint64)
    ld = np.zeros((P, 20, k), np.float32)
    lc = np.zeros((P, 20), np.uint32)
    for r in range(P):
        vs = bsr_mod.get_global_vstore(tmp_path, False)
        ix = bsr_mod.Index(DIMENSION, max_k=k, device=0)
        bsr_mod.load_index_from_vstore(ix, vs, r, P)
        li[r], ld[r], lc[r] = ix.local_top_k(qs, k)
    got = bsr_mod.merge_top_k_lists(li, ld, lc, k)
    wi, wd, wc = oracle_mod.parallel_top_k(data, qs, k, size=P)
    assert np.array_equal(got[2], wc) and np.array_equal(got[0], wi)
    assert np.array_equal(got[1].view(np.uint32), wd.view(np.uint32))


# ---- f-3: src/mpi_helpers/tasks.rs:181-217 (merge_vector_stores) ------------------------
def _write_local_stores(bsr_mod, tmp_path, rng, counts):
    parts = []
    for r, n in enumerate(counts):
        vs = bsr_mod.get_local_vstore(tmp_path, r, True)
        rows = mock_embeddings(rng, n)
        if n:
            vs.append_many(rows)
        vs.persist()
        vs.close()
        parts.append(rows)
    return np.concatenate(parts)


def test_merge_vector_stores_rank_order_skips_empty(bsr_mod, tmp_path, rng):
    want = _write_local_stores(bsr_mod, tmp_path, rng, [5, 0, 7, 3])  # rank 1 empty (skipped)
    merged = bsr_mod.merge_vector_stores(4, tmp_path)
    assert merged.get_count() == 15
    assert np.array_equal(merged.get_many_array(None, DIMENSION), want)
    assert merged.path.endswith("global.parquet")
    merged.close()


@pytest.mark.gpu
def test_merge_vector_stores_into_index_matches_host_merge(bsr_mod, oracle_mod, gpu, tmp_path, rng):
    want = _write_local_stores(bsr_mod, tmp_path, rng, [900, 0, 1300, 451])
    ix = bsr_mod.Index(DIMENSION, max_k=16, device=0)
    assert bsr_mod.merge_vector_stores_into_index(ix, 4, tmp_path) == len(want)
    assert ix.get_count() == len(want)
    qs = mock_embeddings(rng, 5)
    qs[0] = want[1000]
    got = ix.local_top_k(qs, 10)
    wi, wd, wc = oracle_mod.parallel_top_k(want, qs, 10)
    assert np.array_equal(got[2], wc) and np.array_equal(got[0], wi)
    assert np.array_equal(got[1].view(np.uint32), wd.view(np.uint32))
    assert got[0][0, 0] == 1000
