"""ctypes loader for the C oracle (oracle/bsr_oracle.c) plus an independent numpy restatement.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.  Parity status: "parity unpinned"
against the reference binary (Rust toolchain absent); pinned by the
hand-derived known answers in tests/golden/known_answers.json and by agreement between the
two independent restatements here (C and numpy).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libbsr_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        f32p = ctypes.POINTER(ctypes.c_float)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.bsr_oracle_cosine_distance.restype = ctypes.c_float
        L.bsr_oracle_cosine_distance.argtypes = [f32p, ctypes.c_size_t, f32p, ctypes.c_size_t]
        L.bsr_oracle_interval_by_rank.restype = None
        L.bsr_oracle_interval_by_rank.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                                  u64p, u64p]
        L.bsr_oracle_local_top_k.restype = ctypes.c_size_t
        L.bsr_oracle_local_top_k.argtypes = [f32p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_uint32, f32p, u64p, f32p]
        L.bsr_oracle_global_top_k.restype = ctypes.c_size_t
        L.bsr_oracle_global_top_k.argtypes = [u64p, f32p, ctypes.c_size_t, ctypes.c_uint32, u64p, f32p]
        L.bsr_oracle_parallel_top_k_batch.restype = None
        L.bsr_oracle_parallel_top_k_batch.argtypes = [f32p, ctypes.c_uint64, ctypes.c_uint32,
                                                      ctypes.c_int32, ctypes.c_uint32, f32p,
                                                      ctypes.c_uint32, u64p, f32p, u32p,
                                                      ctypes.c_int32]
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def cosine_distance(a, b) -> float:
    a, b = _f32(a).ravel(), _f32(b).ravel()
    return float(np.float32(lib().bsr_oracle_cosine_distance(_p(a, ctypes.c_float), a.size,
                                                             _p(b, ctypes.c_float), b.size)))


def interval_by_rank(rank: int, size: int, count: int):
    s, e = ctypes.c_uint64(), ctypes.c_uint64()
    lib().bsr_oracle_interval_by_rank(rank, size, count, ctypes.byref(s), ctypes.byref(e))
    return s.value, e.value


def local_top_k(rows, rank, size, top_k, query):
    rows = _f32(rows)
    q = _f32(query).ravel()
    oi = np.zeros(max(top_k, 1), np.uint64)
    od = np.zeros(max(top_k, 1), np.float32)
    n = lib().bsr_oracle_local_top_k(_p(rows, ctypes.c_float), rows.shape[0], rows.shape[1], rank,
                                     size, top_k, _p(q, ctypes.c_float), _p(oi, ctypes.c_uint64),
                                     _p(od, ctypes.c_float))
    if n == ctypes.c_size_t(-1).value:
        raise FloatingPointError("NaN distance (reference panics)")
    return oi[:n].copy(), od[:n].copy()


def global_top_k(indices, distances, top_k):
    idx = np.ascontiguousarray(indices, np.uint64)
    dist = _f32(distances)
    oi = np.zeros(max(top_k, 1), np.uint64)
    od = np.zeros(max(top_k, 1), np.float32)
    n = lib().bsr_oracle_global_top_k(_p(idx, ctypes.c_uint64), _p(dist, ctypes.c_float), idx.size,
                                      top_k, _p(oi, ctypes.c_uint64), _p(od, ctypes.c_float))
    if n == ctypes.c_size_t(-1).value:
        raise FloatingPointError("NaN distance (reference panics)")
    return oi[:n].copy(), od[:n].copy()


def parallel_top_k(rows, queries, top_k, size=1, threads=1):
    """Batch of queries -> (idx [Q,k] uint64, dist [Q,k] float32, count [Q] uint32)."""
    rows = _f32(rows)
    qs = _f32(queries)
    if qs.ndim == 1:
        qs = qs[None, :]
    nq = qs.shape[0]
    k = max(top_k, 1)
    oi = np.zeros((nq, k), np.uint64)
    od = np.zeros((nq, k), np.float32)
    oc = np.zeros(nq, np.uint32)
    lib().bsr_oracle_parallel_top_k_batch(_p(rows, ctypes.c_float), rows.shape[0], rows.shape[1],
                                          size, top_k, _p(qs, ctypes.c_float), nq,
                                          _p(oi, ctypes.c_uint64), _p(od, ctypes.c_float),
                                          _p(oc, ctypes.c_uint32), threads)
    return oi[:, :top_k], od[:, :top_k], oc


# ----------------------------------------------------------------------------------------
# Independent numpy restatement (vectorised over rows).  np.add.accumulate with
# dtype=float32 is a strictly sequential f32 running sum, i.e. Rust's fold; np.sum is
# pairwise and would NOT match.  Used to cross-check the C oracle bit-for-bit.
# ----------------------------------------------------------------------------------------

def np_cosine_distances(rows, query):
    """src/metrics.rs:143-165 for every row of `rows` against `query` (a = row, b = query)."""
    rows = _f32(rows)
    q = _f32(query).ravel()
    n, d = rows.shape
    if d != q.size or d == 0:
        return np.ones(n, np.float32)
    with np.errstate(all="ignore"):
        ident = np.all(np.abs(rows - q[None, :]) <= np.float32(1e-10), axis=1)
        prods = rows * q[None, :]
        dot = np.add.accumulate(prods, axis=1, dtype=np.float32)[:, -1]
        ma = np.sqrt(np.add.accumulate(rows * rows, axis=1, dtype=np.float32)[:, -1])
        mb = np.sqrt(np.add.accumulate(q * q, dtype=np.float32)[-1])
        denom = (ma * mb).astype(np.float32)
        s = (dot / denom).astype(np.float32)
        s = np.fmax(s, np.float32(-1.0))
        s = np.fmin(s, np.float32(1.0))
        out = (np.float32(1.0) - s).astype(np.float32)
    out = np.where((ma == 0) | (mb == 0), np.float32(1.0), out)
    out = np.where(ident, np.float32(0.0), out)
    return out.astype(np.float32)


def np_top_k(rows, query, top_k):
    """Global (dist asc, idx asc) top-k: the order parallel_top_k_similarity_search returns
    for any rank count."""
    d = np_cosine_distances(rows, query)
    order = np.lexsort((np.arange(d.size), d))[:top_k]
    return order.astype(np.uint64), d[order]
