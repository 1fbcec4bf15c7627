"""Host-side mirror of better-search-rag-rust's search-path interface over the C ABI.

Every function here is a thin ctypes call into ``lib/libbsr.so`` (include/bsr.h); the
compute runs in the gfx950 HIP kernels.  There is no CPU fallback: if the library or a GPU
is missing the calls raise :class:`BsrError`.  Names and argument meaning follow the
reference (paths relative to nichmorgan/better-search-rag-rust):

=====================================  ===============================================
``cosine_distance(a, b)``              src/metrics.rs:143-165
``interval_by_rank(rank, size, n)``    src/mpi_helpers/load_balance.rs:24-42
``Index`` (get_count/get_many/get)     src/vectorstore/polars.rs:79-169,243-246
``compute_local_top_k``                src/mpi_helpers/metrics.rs:16-53
``gather_top_k_results``               src/mpi_helpers/metrics.rs:56-138
``compute_global_top_k``               src/mpi_helpers/metrics.rs:141-171
``gather_global_top_k``                src/mpi_helpers/metrics.rs:56-171 (a-4 + a-5)
``parallel_top_k_similarity_search``   src/mpi_helpers/metrics.rs:174-206
``Comm`` (RCCL / host transport)       the MPI world; ``Comm.broadcast``: src/main.rs:123-125
``run_search_stage``                   src/main.rs:109-163
``similarity_search_report``           src/mpi_helpers/benchmark.rs:131-413
``calculate_accuracy_metrics``         src/mpi_helpers/metrics.rs:217-249
``PolarsVectorstore`` (lib/libbsr_vstore.so, include/bsr_vstore.h)
                                       src/vectorstore/polars.rs:7-247
``get_global_vstore/get_local_vstore`` src/mpi_helpers/vectorstore.rs:5-20
=====================================  ===============================================
"""
from __future__ import annotations

import ctypes
import os
import warnings
import weakref
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# (BSR_LIB: another build of the same ABI, for A/B measurements)
LIB_PATH = os.environ.get("BSR_LIB") or os.path.join(os.path.dirname(_PKG), "lib", "libbsr.so")
VSTORE_LIB_PATH = os.environ.get("BSR_VSTORE_LIB") or os.path.join(os.path.dirname(_PKG), "lib", "libbsr_vstore.so")

BSR_OK = 0
BSR_PARTIAL = 1  # parallel search root: valid result without its own block (include/bsr.h)
BSR_F32 = 0
BSR_BF16 = 1
BSR_MAX_K = 256
BSR_FLAG_EXACT_ONLY = 1
BSR_FLAG_PROFILE = 2
BSR_FLAG_FILTER_BF16 = 4   # retired (round 4): bsr_index_create returns BSR_E_INVALID
# SearchStats.search_path bits (include/bsr.h)
BSR_PATH_COLLECTIVE = 1
BSR_PATH_GLOBAL_TAU = 2
BSR_PATH_DIRECT_OUT = 4
BSR_PATH_DEVICE_MERGE = 8
BSR_PATH_FALLBACK = 16
BSR_PATH_SKINNY_TOP = 32
BSR_PATH_TOP_RERUN = 64
FILTER_I8 = 0
ROOT = 0  # src/mpi_helpers/mod.rs:8


class BsrError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{_status_name(status)}: {message}")
        self.status = status


class _Config(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_uint32), ("dtype", ctypes.c_uint32), ("max_k", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("device", ctypes.c_int32)]


class _Interval(ctypes.Structure):
    _fields_ = [("start_index", ctypes.c_uint64), ("end_index", ctypes.c_uint64)]


class SearchStats(ctypes.Structure):
    _fields_ = [("n_queries", ctypes.c_uint32), ("n_exact_direct", ctypes.c_uint32),
                ("n_fallback", ctypes.c_uint32), ("n_candidates", ctypes.c_uint32),
                ("n_emitted", ctypes.c_uint64), ("filter_op", ctypes.c_uint32),
                ("row_ebound", ctypes.c_float), ("n_rescued", ctypes.c_uint32),
                ("graph_replay", ctypes.c_uint32), ("search_path", ctypes.c_uint32)]


class Profile(ctypes.Structure):
    _fields_ = [("gemm_emit_ms", ctypes.c_double), ("gemm_emit_launches", ctypes.c_uint64),
                ("gemm_sample_ms", ctypes.c_double), ("gemm_sample_launches", ctypes.c_uint64),
                ("select_ms", ctypes.c_double), ("select_launches", ctypes.c_uint64),
                ("rescore_ms", ctypes.c_double), ("rescore_launches", ctypes.c_uint64),
                ("scan_ms", ctypes.c_double), ("scan_launches", ctypes.c_uint64),
                ("search_ms", ctypes.c_double), ("searches", ctypes.c_uint64)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


_lib = None
_P = ctypes.c_void_p
# int (*)(const void* send, void* recv, uint64_t bytes, void* user)  (include/bsr.h)
_HOST_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_void_p)


def lib() -> ctypes.CDLL:
    """Load libbsr.so (raises if it has not been built: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BsrError(-3, f"{LIB_PATH} not built (run __graft_entry__.build()); no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    u32, u64, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    sig = {
        "bsr_last_error": (ctypes.c_char_p, []),
        "bsr_status_string": (ctypes.c_char_p, [ctypes.c_int]),
        "bsr_version": (ctypes.c_char_p, []),
        "bsr_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "bsr_cosine_distance": (ctypes.c_int, [_P, u32, _P, u32, ctypes.POINTER(ctypes.c_float)]),
        "bsr_interval_by_rank": (ctypes.c_int, [i32, i32, u64, ctypes.POINTER(_Interval)]),
        "bsr_index_create": (ctypes.c_int, [ctypes.POINTER(_Config), ctypes.POINTER(_P)]),
        "bsr_index_destroy": (None, [_P]),
        "bsr_index_load": (ctypes.c_int, [_P, _P, u64, u64]),
        "bsr_index_append": (ctypes.c_int, [_P, _P, u64]),
        "bsr_index_count": (ctypes.c_int, [_P, ctypes.POINTER(u64)]),
        "bsr_index_dim": (ctypes.c_int, [_P, ctypes.POINTER(u32)]),
        "bsr_index_global_offset": (ctypes.c_int, [_P, ctypes.POINTER(u64)]),
        "bsr_index_get_many": (ctypes.c_int, [_P, u64, u64, _P]),
        "bsr_local_top_k": (ctypes.c_int, [_P, _P, u32, u32, _P, _P, _P]),
        "bsr_global_top_k": (ctypes.c_int, [_P, _P, _P, u32, u32, u32, u32, _P, _P, _P]),
        "bsr_comm_unique_id": (ctypes.c_int, [_P]),
        "bsr_comm_init": (ctypes.c_int, [_P, i32, i32, i32, ctypes.POINTER(_P)]),
        "bsr_comm_destroy": (None, [_P]),
        "bsr_comm_rank": (ctypes.c_int, [_P, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "bsr_gather_top_k": (ctypes.c_int, [_P, _P, _P, _P, u32, u32, _P, _P, _P]),
        "bsr_comm_init_host": (ctypes.c_int, [i32, i32, _HOST_ALLGATHER, _P, ctypes.POINTER(_P)]),
        "bsr_gather_global_top_k": (ctypes.c_int, [_P, _P, _P, _P, u32, u32, _P, _P, _P]),
        "bsr_comm_init_loopback": (ctypes.c_int, [i32, i32, i32, u32, _P, _P, ctypes.POINTER(_P)]),
        "bsr_comm_loopback_stats": (ctypes.c_int, [_P, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "bsr_host_alloc": (ctypes.c_int, [u64, ctypes.POINTER(_P)]),
        "bsr_host_free": (None, [_P]),
        "bsr_broadcast": (ctypes.c_int, [_P, _P, u64, i32]),
        "bsr_allgather_bytes": (ctypes.c_int, [_P, _P, _P, u64]),
        "bsr_parallel_top_k_similarity_search": (ctypes.c_int, [_P, _P, _P, u32, u32, _P, _P, _P]),
        "bsr_index_last_stats": (ctypes.c_int, [_P, ctypes.POINTER(SearchStats)]),
        "bsr_index_profile": (ctypes.c_int, [_P, ctypes.POINTER(Profile), ctypes.c_int]),
        "bsr_index_set_profile": (ctypes.c_int, [_P, ctypes.c_int]),
        "bsr_synth_uniform": (ctypes.c_int, [_P, u64, u64, u32, u64]),
    }
    optional = {"bsr_host_alloc", "bsr_host_free"}  # (absent in older builds used for A/B runs)
    for name, (res, args) in sig.items():
        if name in optional and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _status_name(s: int) -> str:
    try:
        return lib().bsr_status_string(s).decode()
    except Exception:  # library missing
        return f"status {s}"


def _check(status: int):
    if status != BSR_OK:
        raise BsrError(status, lib().bsr_last_error().decode())


def _ptr(a) -> Optional[int]:
    """Data pointer of a numpy array or a torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    raise TypeError(f"unsupported buffer type {type(a)}")


class _PinnedOwner:
    def __init__(self, p):
        self.p = p

    def __del__(self):
        try:
            lib().bsr_host_free(self.p)
        except Exception:
            pass


def host_array(shape, dtype) -> np.ndarray:
    """A numpy array in coherent pinned host memory (bsr_host_alloc; freed with the array).  Root
    outputs there are written by the GPU directly on the global-threshold path (include/bsr.h)."""
    dtype = np.dtype(dtype)
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    if not hasattr(lib(), "bsr_host_alloc"):  # (an older build: pageable memory)
        return np.empty(shape, dtype)
    n = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
    p = _P()
    _check(lib().bsr_host_alloc(max(n, 1), ctypes.byref(p)))
    buf = (ctypes.c_uint8 * max(n, 1)).from_address(p.value)
    buf._owner = _PinnedOwner(p.value)  # (the array's base keeps the allocation alive)
    return np.frombuffer(buf, dtype=dtype, count=n // dtype.itemsize).reshape(shape)


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(lib().bsr_device_count(ctypes.byref(n)))
    return n.value


def version() -> str:
    return lib().bsr_version().decode()


# ---- a-1 --------------------------------------------------------------------------------
def cosine_distance(a, b) -> float:
    """src/metrics.rs:143-165 (a = stored row, b = query), computed on the GPU."""
    a = np.ascontiguousarray(a, np.float32).ravel()
    b = np.ascontiguousarray(b, np.float32).ravel()
    out = ctypes.c_float(0.0)
    _check(lib().bsr_cosine_distance(_ptr(a) if a.size else None, a.size,
                                     _ptr(b) if b.size else None, b.size, ctypes.byref(out)))
    return float(np.float32(out.value))


# ---- a-3 --------------------------------------------------------------------------------
@dataclass
class RankInterval:
    """src/mpi_helpers/load_balance.rs:8-17."""
    start_index: int
    end_index: int

    def get_count(self) -> int:
        # The reference's release build wraps end - start when end < start and then slices
        # nothing; the effective count is therefore max(0, end - start).
        return max(0, self.end_index - self.start_index)


def interval_by_rank(rank: int, size: int, count: int) -> RankInterval:
    out = _Interval()
    _check(lib().bsr_interval_by_rank(rank, size, count, ctypes.byref(out)))
    return RankInterval(out.start_index, out.end_index)


@dataclass
class SliceArgs:
    """src/vectorstore/polars.rs:12-15."""
    offset: int
    length: int


# ---- the rank's shard ---------------------------------------------------------------------
class Index:
    """One rank's corpus block resident in HBM (read side of PolarsVectorstore)."""

    def __init__(self, dim: int = 768, max_k: int = 64, device: int = -1, dtype: int = BSR_F32,
                 flags: int = 0):
        cfg = _Config(dim, dtype, max_k, flags, device)
        h = _P()
        _check(lib().bsr_index_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.dim = dim
        self.max_k = max_k
        self.dtype = dtype

    def close(self):
        if getattr(self, "_h", None):
            lib().bsr_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _rows(self, rows):
        if isinstance(rows, np.ndarray):
            want = np.uint16 if self.dtype == BSR_BF16 else np.float32
            rows = np.ascontiguousarray(rows, want)
            if rows.ndim == 1:
                rows = rows.reshape(1, -1)
            n = rows.shape[0]
            if n and rows.shape[1] != self.dim:
                raise BsrError(-6, f"row length {rows.shape[1]} != dim {self.dim}")
            return rows, n
        n = int(rows.shape[0]) if rows.dim() > 1 else 1
        want = 2 if self.dtype == BSR_BF16 else 4
        if rows.element_size() != want or not rows.is_contiguous():
            raise BsrError(-1, f"rows must be a contiguous {want}-byte tensor for this index dtype")
        if n and int(rows.shape[-1]) != self.dim:
            raise BsrError(-6, f"row length {int(rows.shape[-1])} != dim {self.dim}")
        return rows, n

    def load(self, rows, global_offset: int = 0):
        rows, n = self._rows(rows)
        _check(lib().bsr_index_load(self._h, _ptr(rows) if n else None, n, global_offset))
        return self

    def append_many(self, rows):
        """PolarsVectorstore::append_many (src/vectorstore/polars.rs:101-119)."""
        rows, n = self._rows(rows)
        _check(lib().bsr_index_append(self._h, _ptr(rows) if n else None, n))

    def append(self, vector):
        self.append_many(np.asarray(vector).reshape(1, -1))

    def get_count(self) -> int:
        n = ctypes.c_uint64()
        _check(lib().bsr_index_count(self._h, ctypes.byref(n)))
        return n.value

    def global_offset(self) -> int:
        n = ctypes.c_uint64()
        _check(lib().bsr_index_global_offset(self._h, ctypes.byref(n)))
        return n.value

    def get_many(self, slice_args: Optional[SliceArgs] = None) -> np.ndarray:
        count = self.get_count()
        if slice_args is None:
            off, length = 0, count
        else:
            off = min(max(slice_args.offset, 0), count)
            length = min(slice_args.length, count - off)
        out = np.empty((length, self.dim), np.float32)
        _check(lib().bsr_index_get_many(self._h, off, length, _ptr(out) if length else None))
        return out

    def get(self, index: int) -> np.ndarray:
        rows = self.get_many(SliceArgs(index, 1))
        if rows.shape[0] == 0:
            raise BsrError(-1, "Index not found")
        return rows[0]

    def local_top_k(self, queries, k: int):
        """Batched compute_local_top_k -> (idx [Q,k] u64, dist [Q,k] f32, count [Q] u32)."""
        q = np.ascontiguousarray(queries, np.float32)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        if q.shape[1] != self.dim:
            raise BsrError(-6, f"query length {q.shape[1]} != dim {self.dim}")
        nq = q.shape[0]
        oi = np.empty((nq, k), np.uint64)
        od = np.empty((nq, k), np.float32)
        oc = np.empty(nq, np.uint32)
        _check(lib().bsr_local_top_k(self._h, _ptr(q), nq, k, _ptr(oi), _ptr(od), _ptr(oc)))
        return oi, od, oc

    def local_top_k_device(self, queries, nq: int, k: int, out_idx, out_dist, out_count):
        """Zero-copy variant on device buffers (torch tensors or raw pointers)."""
        _check(lib().bsr_local_top_k(self._h, _ptr(queries), nq, k, _ptr(out_idx), _ptr(out_dist),
                                     _ptr(out_count)))

    def last_stats(self) -> SearchStats:
        s = SearchStats()
        _check(lib().bsr_index_last_stats(self._h, ctypes.byref(s)))
        return s

    def set_profile(self, level: int) -> None:
        """Event recording of a profiled index: 0 none, 1 filter/scan kernels, 2 every stage."""
        _check(lib().bsr_index_set_profile(self._h, int(level)))

    def profile(self, reset: bool = False) -> Profile:
        p = Profile()
        _check(lib().bsr_index_profile(self._h, ctypes.byref(p), int(reset)))
        return p


# ---- communicator -----------------------------------------------------------------------
class Comm:
    """The rank group of the exchange step -- replaces the MPI world.

    ``Comm(unique_id, rank, size, device)``: RCCL over xGMI, one GPU per rank.
    ``Comm.host(group)``: the same gather + merge code over a host transport, here a
    torch.distributed process group (gloo on CPU, or any backend): the library calls back
    into Python for each all-gather of packed host bytes."""

    def __init__(self, unique_id: bytes, rank: int, size: int, device: int = -1):
        h = _P()
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        _check(lib().bsr_comm_init(buf, rank, size, device, ctypes.byref(h)))
        self._h = h
        self.rank = rank
        self.size = size
        self.transport = "rccl"

    @classmethod
    def host(cls, group=None) -> "Comm":
        """`record` (attribute): set it to a list and every all-gather appends its receive
        buffer [size * bytes] to it (the script of Comm.loopback)."""
        import torch
        import torch.distributed as dist

        rank, size = dist.get_rank(group), dist.get_world_size(group)

        def allgather(send, recv, nbytes, _user):
            try:
                n = int(nbytes)
                src = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(send)) if n else np.zeros(0, np.uint8)
                t = torch.from_numpy(src.copy())
                parts = [torch.empty(n, dtype=torch.uint8) for _ in range(size)]
                dist.all_gather(parts, t, group=group)
                dst = np.ctypeslib.as_array((ctypes.c_uint8 * (n * size)).from_address(recv)) if n else None
                for r, p in enumerate(parts):
                    if n:
                        dst[r * n:(r + 1) * n] = p.numpy()
                if self.record is not None and n:
                    self.record.append(dst.copy())
                return 0
            except Exception:  # the library reports a transport failure
                return 1

        self = cls.__new__(cls)
        self.record = None
        self._cb = _HOST_ALLGATHER(allgather)  # kept alive as long as the comm
        h = _P()
        _check(lib().bsr_comm_init_host(rank, size, self._cb, None, ctypes.byref(h)))
        self._h = h
        self.rank = rank
        self.size = size
        self.transport = "host"
        return self

    @classmethod
    def loopback(cls, rank: int, size: int, device: int = -1, script=None) -> "Comm":
        """One process acting as rank `rank` of `size` (measurement and tests): every
        all-gather is one device kernel on the stream where ncclAllGather would sit.  `script`
        (optional): the all-gathers of one parallel search recorded in a real size-rank run,
        a list of [size * bytes] uint8 arrays in call order (see Comm.host's `record`); the
        searches then replay them, this rank's own slot live (include/bsr.h)."""
        script = list(script or [])
        nb = np.array([len(x) // size for x in script] or [0], np.uint64)
        data = np.ascontiguousarray(np.concatenate([np.frombuffer(bytes(x), np.uint8) for x in script])
                                    if script else np.zeros(1, np.uint8))
        self = cls.__new__(cls)
        h = _P()
        _check(lib().bsr_comm_init_loopback(rank, size, device, len(script), _ptr(nb), _ptr(data), ctypes.byref(h)))
        self._h = h
        self.rank = rank
        self.size = size
        self.transport = "loopback"
        return self

    def loopback_stats(self) -> Tuple[int, int]:
        """(all-gathers replayed from the script, calls that missed it) of a loopback Comm."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().bsr_comm_loopback_stats(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        _check(lib().bsr_comm_unique_id(buf))
        return bytes(buf)

    def broadcast(self, array, root: int = 0):
        """src/main.rs:123-125 process_at_rank(root).broadcast_into(array) (in place)."""
        _check(lib().bsr_broadcast(self._h, _ptr(array), int(array.nbytes if isinstance(array, np.ndarray)
                                                              else array.numel() * array.element_size()), root))
        return array

    def allgather_bytes(self, data: bytes) -> List[bytes]:
        n = len(data)
        src = np.frombuffer(data, np.uint8).copy() if n else np.zeros(1, np.uint8)
        dst = np.empty(max(n * self.size, 1), np.uint8)
        _check(lib().bsr_allgather_bytes(self._h, _ptr(src), _ptr(dst), n))
        return [dst[r * n:(r + 1) * n].tobytes() for r in range(self.size)]

    def close(self):
        if getattr(self, "_h", None):
            lib().bsr_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _as_comm(world) -> Optional[Comm]:
    """A Comm for `world`: a Comm as is, None (one rank) as None, a torch.distributed
    group (or the default group, passed as a group object) as a cached host-transport Comm.
    The cache holds the group weakly: a destroyed group's Comm is never handed to a new
    group that reuses its id()."""
    if world is None or isinstance(world, Comm):
        return world
    try:
        c = _HOST_COMMS.get(world)
    except TypeError:  # a group object that cannot be weakly referenced: no caching
        return Comm.host(world)
    if c is None:
        c = Comm.host(world)
        _HOST_COMMS[world] = c
    return c


_HOST_COMMS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


# ---- a-2 ... a-6 (reference-shaped, single query) -------------------------------------
def compute_local_top_k(index: Index, rank: int, size: int, top_k: int, target_vector
                        ) -> List[Tuple[int, float]]:
    """src/mpi_helpers/metrics.rs:16-53.  `index` holds this rank's block, loaded with the
    global offset interval_by_rank(rank, size, N).start_index."""
    idx, dist, cnt = index.local_top_k(np.asarray(target_vector, np.float32).reshape(1, -1), top_k)
    return [(int(idx[0, i]), float(dist[0, i])) for i in range(int(cnt[0]))]


def compute_global_top_k(global_indices: Sequence[int], global_distances: Sequence[float],
                         top_k: int) -> List[Tuple[int, float]]:
    """src/mpi_helpers/metrics.rs:141-171 (stable sort by distance, dedupe, keep top_k)."""
    gi = np.ascontiguousarray(global_indices, np.uint64).ravel()
    gd = np.ascontiguousarray(global_distances, np.float32).ravel()
    n = gi.size
    cnt = np.array([n], np.uint32)
    if n == 0:  # keep the pointers valid; the count says there is nothing to read
        gi, gd = np.zeros(1, np.uint64), np.zeros(1, np.float32)
    oi = np.empty(max(top_k, 1), np.uint64)
    od = np.empty(max(top_k, 1), np.float32)
    oc = np.empty(1, np.uint32)
    _check(lib().bsr_global_top_k(_ptr(gi), _ptr(gd), _ptr(cnt), 1, 1, max(n, 1), top_k, _ptr(oi),
                                  _ptr(od), _ptr(oc)))
    return [(int(oi[i]), float(od[i])) for i in range(int(oc[0]))]


def merge_top_k_lists(idx, dist, count, top_k: int):
    """compute_global_top_k for many queries at once: idx/dist [L,Q,k_in], count [L,Q]."""
    idx = np.ascontiguousarray(idx, np.uint64)
    dist = np.ascontiguousarray(dist, np.float32)
    count = np.ascontiguousarray(count, np.uint32)
    L, Q, k_in = idx.shape
    oi = np.empty((Q, top_k), np.uint64)
    od = np.empty((Q, top_k), np.float32)
    oc = np.empty(Q, np.uint32)
    _check(lib().bsr_global_top_k(_ptr(idx), _ptr(dist), _ptr(count), L, Q, k_in, top_k, _ptr(oi),
                                  _ptr(od), _ptr(oc)))
    return oi, od, oc


def gather_top_k_results(world, rank: int, local_top_k: List[Tuple[int, float]]):
    """src/mpi_helpers/metrics.rs:56-138: rank-order concatenation at the root, through the
    C ABI's exchange (bsr_gather_top_k) over `world` (a Comm, a torch.distributed group or
    None for one rank).  Non-root ranks get empty lists, like the reference."""
    local_idx = [int(i) for i, _ in local_top_k]
    local_dist = [float(d) for _, d in local_top_k]
    comm = _as_comm(world)
    if comm is None:
        return local_idx, local_dist
    # every rank sends a fixed-size slot: the largest local count (all-gathered first, as
    # the reference's all_gather_into of the counts, :67-68)
    counts = np.frombuffer(b"".join(comm.allgather_bytes(np.uint32(len(local_idx)).tobytes())), np.uint32)
    kk = max(int(counts.max()), 1)
    li = np.zeros((1, kk), np.uint64)
    ld = np.zeros((1, kk), np.float32)
    li[0, :len(local_idx)] = local_idx
    ld[0, :len(local_dist)] = local_dist
    lc = np.array([len(local_idx)], np.uint32)
    P = comm.size
    ri = np.zeros((P, 1, kk), np.uint64)
    rd = np.zeros((P, 1, kk), np.float32)
    rc = np.zeros((P, 1), np.uint32)
    _check(lib().bsr_gather_top_k(comm._h, _ptr(li), _ptr(ld), _ptr(lc), 1, kk, _ptr(ri), _ptr(rd), _ptr(rc)))
    if rank != ROOT:
        return [], []
    gi, gd = [], []
    for r in range(P):  # rank order
        c = int(rc[r, 0])
        gi.extend(int(x) for x in ri[r, 0, :c])
        gd.extend(float(x) for x in rd[r, 0, :c])
    return gi, gd


def gather_global_top_k(world, local_idx, local_dist, local_count, top_k: int):
    """a-4 + a-5 composed (the exchange step of parallel_top_k_similarity_search,
    src/mpi_helpers/metrics.rs:194-202) for a batch: local lists [Q, top_k] (+ counts [Q]) of
    this rank, or all None for an empty contribution.  Root: (idx, dist, count) of the
    global top-k; other ranks: None.  `world` None (one rank): the local lists merged alone."""
    q, err = None, None
    if local_idx is not None:
        local_idx = np.ascontiguousarray(local_idx, np.uint64)
        local_dist = np.ascontiguousarray(local_dist, np.float32)
        local_count = np.ascontiguousarray(local_count, np.uint32)
        q = local_idx.shape[0] if local_idx.ndim else 0
        # the library reads Q * top_k entries of each list and Q counts
        if local_idx.shape != (q, top_k) or local_dist.shape != (q, top_k) or local_count.shape != (q,):
            err = (f"local lists must be [Q, top_k] = [{q}, {top_k}] (+ counts [Q]); got "
                   f"{local_idx.shape}, {local_dist.shape}, {local_count.shape}")
    comm = _as_comm(world)
    if comm is None:
        if err:
            raise BsrError(-1, err)
        if q is None:
            raise BsrError(-1, "one rank (world=None) with no local lists: nothing to merge")
        return merge_top_k_lists(local_idx[None], local_dist[None], local_count[None], top_k)
    # Every rank's {has lists, Q, top_k, valid} first, and every check after it: a rank that
    # raised before the exchange would leave the others blocked in it, and ranks that disagree
    # on the batch shape must all fail before any list moves (as the C parallel search does).
    mine = np.array([q is not None, q or 0, top_k, err is not None], np.uint32)
    hdr = np.frombuffer(b"".join(comm.allgather_bytes(mine.tobytes())), np.uint32).reshape(comm.size, 4)
    bad = [r for r in range(comm.size) if hdr[r, 3]]
    if bad:
        raise BsrError(-1, err if err else f"rank(s) {bad} passed invalid local lists; no rank exchanged lists")
    shapes = {int(hdr[r, 1]) for r in range(comm.size) if hdr[r, 0]}
    if len(shapes) > 1 or len({int(x) for x in hdr[:, 2]}) > 1:
        raise BsrError(-1, f"ranks disagree on the batch shape (Q per rank {hdr[:, 1].tolist()}, top_k per rank "
                           f"{hdr[:, 2].tolist()}); no rank exchanged lists")
    nq = shapes.pop() if shapes else 0
    oi = np.empty((nq, top_k), np.uint64)
    od = np.empty((nq, top_k), np.float32)
    oc = np.empty(nq, np.uint32)
    _check(lib().bsr_gather_global_top_k(comm._h, _ptr(local_idx), _ptr(local_dist), _ptr(local_count), nq,
                                         top_k, _ptr(oi), _ptr(od), _ptr(oc)))
    if comm.rank != ROOT:
        return None
    return oi, od, oc


def _check_parallel(status: int, rank: int) -> None:
    """Status of bsr_parallel_top_k_similarity_search: BSR_PARTIAL on the root is the
    reference's Some(..) after a local error (src/mpi_helpers/metrics.rs:185-202): the result
    stands (it covers the other ranks) and the error is reported as a warning, as the
    reference prints it."""
    if status == BSR_PARTIAL and rank == ROOT:
        warnings.warn(lib().bsr_last_error().decode(), RuntimeWarning, stacklevel=3)
        return
    _check(status)


def parallel_top_k_similarity_search(world, rank: int, size: int, index: Index, top_k: int,
                                     target_vector) -> Optional[List[Tuple[int, float]]]:
    """src/mpi_helpers/metrics.rs:174-206, one query: the local search on this rank's shard
    (GPU), the exchange over `world` (a Comm -- RCCL or host transport --, a
    torch.distributed group, or None for one rank) and the root's merge, all inside the
    library (bsr_parallel_top_k_similarity_search).  Root: the global top-k; others: None."""
    res = parallel_top_k_similarity_search_batch(world, index, np.asarray(target_vector, np.float32).reshape(1, -1),
                                                 top_k, rank=rank)
    if res is None:
        return None
    oi, od, oc = res
    return [(int(oi[0, i]), float(od[0, i])) for i in range(int(oc[0]))]


def parallel_top_k_similarity_search_batch(world, index: Optional[Index], queries, top_k: int,
                                           rank: Optional[int] = None):
    """The same for a batch of queries [Q, dim] (host array or device tensor): Q independent
    reference searches in one collective call.  Root: (idx [Q, top_k] u64, dist [Q, top_k]
    f32, count [Q] u32); other ranks: None.  A non-root rank whose local step fails raises
    after the exchange; the root then warns and returns the other ranks' global top-k.
    Local argument checks never return before the collective: a rank whose
    queries are unusable still takes part, with an empty contribution (the library's null-index
    path), and raises -- or, on the root, warns -- afterwards, as the library does for a failed
    local search (src/mpi_helpers/metrics.rs:185-202)."""
    comm = _as_comm(world)
    if rank is None:
        rank = comm.rank if comm is not None else ROOT
    err = None  # (status, message) of this rank's local checks
    if isinstance(queries, np.ndarray) or not hasattr(queries, "data_ptr"):
        try:
            queries = np.ascontiguousarray(queries, np.float32)
        except (TypeError, ValueError) as e:
            err, queries = (-1, f"queries are not a float32 array: {e}"), np.zeros((0, 0), np.float32)
    if queries.ndim == 1:
        queries = queries.reshape(1, -1)
    if err is None and queries.ndim != 2:
        err = (-1, f"queries must be [Q, dim]; got shape {tuple(queries.shape)}")
    if err is None and not isinstance(queries, np.ndarray):
        import torch
        if queries.dtype != torch.float32 or not queries.is_contiguous():
            err = (-1, "query tensors must be contiguous float32")
    if err is None and index is not None and int(queries.shape[1]) != index.dim:
        err = (-6, f"query length {int(queries.shape[1])} != dim {index.dim}")
    nq = int(queries.shape[0]) if queries.ndim >= 1 else 0
    if err is not None and comm is None:
        raise BsrError(*err)
    oi = np.empty((nq, top_k), np.uint64)
    od = np.empty((nq, top_k), np.float32)
    oc = np.empty(nq, np.uint32)
    # (a rank with an error passes no index: an empty contribution; the batch shape it passes is
    # still agreed with the others, so a rank whose Q differs makes every rank fail together)
    st = lib().bsr_parallel_top_k_similarity_search(comm._h if comm else None,
                                                    index._h if (index and err is None) else None,
                                                    _ptr(queries) if err is None else None, nq, top_k,
                                                    _ptr(oi), _ptr(od), _ptr(oc))
    if err is not None:
        if rank == ROOT and st == BSR_PARTIAL:
            warnings.warn(f"{_status_name(err[0])}: {err[1]} (this rank's block is missing from the result)",
                          RuntimeWarning, stacklevel=2)
            return oi, od, oc
        msg = lib().bsr_last_error().decode()
        extra = "" if st in (BSR_OK, BSR_PARTIAL) or "null index" in msg else f"; the collective: {msg}"
        raise BsrError(err[0], err[1] + extra)
    _check_parallel(st, rank)
    if rank != ROOT:
        return None
    return oi, od, oc


def calculate_accuracy_metrics(top_k_results, query_idx: int, top_k: int):
    """src/mpi_helpers/metrics.rs:217-249 (MRR, recall@k, overlap of the query row)."""
    position = 0
    for i, (idx, _) in enumerate(top_k_results):
        if idx == query_idx:
            position = i + 1
            break
    mrr = 1.0 / position if position > 0 else 0.0
    recall = 1.0 if 0 < position <= top_k else 0.0
    overlap = 1.0 if position > 0 else 0.0
    return mrr, recall, overlap


def print_top_k_results(top_k_results, out=None) -> None:
    """src/mpi_helpers/metrics.rs:209-214 (Rust's `{}` of an f32 is its shortest round-trip
    form, as Python's repr of the same float32)."""
    import sys as _sys
    w = (out or _sys.stdout).write
    w(f"Global top-{len(top_k_results)} results:\n")
    for i, (idx, dist) in enumerate(top_k_results):
        w(f"  {i + 1}. Index: {idx}, Distance: {_rust_f32(dist)}\n")


def _rust_f32(x) -> str:
    """Rust's Display of an f32: the shortest round-trip digits, positional, no exponent."""
    return np.format_float_positional(np.float32(x), unique=True, trim="-")


def similarity_search_report(world, rank: int, seconds: float) -> str:
    """The "similarity_search" entry of the reference's performance report
    (src/mpi_helpers/benchmark.rs:131-293 gathers every rank's timing to the root;
    :296-413 prints min (first rank attaining it), max (last rank attaining it, as Rust's
    max_by) and the average, {:.4} seconds).  Root: the report text; other ranks: ""."""
    comm = _as_comm(world)
    if comm is None:
        secs = [float(seconds)]
    else:
        parts = comm.allgather_bytes(np.float64(seconds).tobytes())
        secs = [float(np.frombuffer(p, np.float64)[0]) for p in parts]
    if rank != ROOT:
        return ""
    mn, mx = min(secs), max(secs)
    min_rank = secs.index(mn)
    max_rank = len(secs) - 1 - secs[::-1].index(mx)
    return ("==== PARALLEL PERFORMANCE REPORT ====\n\n"
            "Operation: similarity_search\n"
            f"  Min time: {mn:.4f} sec (Rank {min_rank})\n"
            f"  Max time: {mx:.4f} sec (Rank {max_rank})\n"
            f"  Avg time: {sum(secs) / len(secs):.4f} sec\n")


def run_search_stage(world, rank: int, size: int, index: "Index", target_vector=None, top_k: int = 50,
                     query_idx: int = 0, out=None, report: bool = True):
    """The driver's search stage (src/main.rs:109-163).  The "similarity_search" timer starts
    first (:114); unless the caller passes `target_vector`, the root reads row `query_idx` of
    its own store (rank 0's shard starts at global row 0, :117-121) and broadcasts it to every
    rank (:123-125); then the parallel top-k search (:130-131).  On the root the result list
    and the accuracy metrics are printed in the reference's format (:141-163), followed by
    the report's similarity_search entry.  Returns (results, metrics, seconds) on the root,
    (None, None, seconds) elsewhere.  Collective: every rank calls it."""
    import sys as _sys
    import time as _time
    w = (out or _sys.stdout).write
    comm = _as_comm(world)
    t0 = _time.perf_counter()
    if target_vector is None:
        target_vector = np.zeros(index.dim, np.float32)
        if rank == ROOT:
            target_vector = np.ascontiguousarray(index.get(query_idx), np.float32)
        if comm is not None:
            comm.broadcast(target_vector, ROOT)
    res = parallel_top_k_similarity_search(comm, rank, size, index, top_k, target_vector)
    secs = _time.perf_counter() - t0
    rep = similarity_search_report(comm, rank, secs) if report else ""
    if rank != ROOT:
        return None, None, secs
    if res is None:
        w("Error: Failed to compute global top-k results\n")
        return None, None, secs
    print_top_k_results(res, out)
    mrr, recall, overlap = calculate_accuracy_metrics(res, query_idx, top_k)
    w("Accuracy Metrics:\n")
    w(f"  Mean Reciprocal Rank (MRR): {mrr:.4f}\n")
    w(f"  Recall@{top_k}: {recall:.4f}\n")
    w(f"  Top-k Overlap: {overlap:.4f}\n")
    if rep:
        w(rep)
    return res, (mrr, recall, overlap), secs


def synth_uniform(dev_ptr: int, row0: int, n_rows: int, dim: int, seed: int):
    """Fill device memory with the synthetic U(-1,1) corpus rows [row0, row0+n_rows)."""
    _check(lib().bsr_synth_uniform(dev_ptr, row0, n_rows, dim, seed))


def synth_uniform_np(row0: int, n_rows: int, dim: int, seed: int) -> np.ndarray:
    """Host replica of bsr_synth_uniform (splitmix64 of (seed, global element index))."""
    with np.errstate(over="ignore"):
        g = (np.uint64(row0) * np.uint64(dim) + np.arange(n_rows * dim, dtype=np.uint64))
        x = np.uint64(seed) * np.uint64(0xD1B54A32D192ED03) + g
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    v = (x >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 8388608.0) - np.float32(1.0)
    return v.reshape(n_rows, dim)


# ---- f-1: the parquet vector store (src/vectorstore/polars.rs) ------------------------------
_vlib = None


def vstore_lib() -> ctypes.CDLL:
    """Load libbsr_vstore.so (Arrow C++ / Parquet; host only)."""
    global _vlib
    if _vlib is not None:
        return _vlib
    lib()  # libbsr.so first (the adapter links it and shares its error state)
    if not os.path.exists(VSTORE_LIB_PATH):
        raise BsrError(-3, f"{VSTORE_LIB_PATH} not built (run __graft_entry__.build())")
    L = ctypes.CDLL(VSTORE_LIB_PATH)
    u32, u64, i32, i64 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int64
    sig = {
        "bsr_vstore_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(_P)]),
        "bsr_vstore_close": (None, [_P]),
        "bsr_vstore_path": (ctypes.c_char_p, [_P]),
        "bsr_vstore_get_count": (ctypes.c_int, [_P, ctypes.POINTER(u64)]),
        "bsr_vstore_get_many": (ctypes.c_int, [_P, i64, u64, _P, u64, _P, u64, ctypes.POINTER(u64),
                                               ctypes.POINTER(u64)]),
        "bsr_vstore_read_slab": (ctypes.c_int, [_P, i64, u64, u32, _P, u64, ctypes.POINTER(u64)]),
        "bsr_vstore_get": (ctypes.c_int, [_P, u64, _P, u32, ctypes.POINTER(u32)]),
        "bsr_vstore_append_many": (ctypes.c_int, [_P, _P, u64, u32]),
        "bsr_vstore_persist": (ctypes.c_int, [_P]),
        "bsr_vstore_reload": (ctypes.c_int, [_P, ctypes.c_int]),
        "bsr_vstore_reset": (ctypes.c_int, [_P]),
        "bsr_vstore_global_path": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]),
        "bsr_vstore_local_path": (ctypes.c_int, [ctypes.c_char_p, i32, ctypes.c_char_p, ctypes.c_size_t]),
        "bsr_index_load_vstore": (ctypes.c_int, [_P, _P, i32, i32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _vlib = L
    return L


class PolarsVectorstore:
    """src/vectorstore/polars.rs:7-247 over libbsr_vstore.so: one parquet file, one column
    "embeddings" of List(Float32).  Rows come back as lists of numpy float32 arrays (the
    reference's Vec<Vec<f32>>); `get_many_array` gives a dense [rows][dim] array."""

    def __init__(self, path: str, empty: bool):
        h = _P()
        _check(vstore_lib().bsr_vstore_open(os.fsencode(path), 1 if empty else 0, ctypes.byref(h)))
        self._h = h

    @property
    def path(self) -> str:
        return vstore_lib().bsr_vstore_path(self._h).decode()

    def close(self):
        if getattr(self, "_h", None):
            vstore_lib().bsr_vstore_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_count(self) -> int:
        n = ctypes.c_uint64(0)
        _check(vstore_lib().bsr_vstore_get_count(self._h, ctypes.byref(n)))
        return n.value

    def _slice(self, s: Optional[SliceArgs]) -> Tuple[int, int]:
        if s is None:
            return 0, self.get_count()
        return int(s.offset), int(s.length)

    def get_many(self, slice_args: Optional[SliceArgs] = None) -> List[np.ndarray]:
        off, length = self._slice(slice_args)
        L = vstore_lib()
        rows, floats = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(L.bsr_vstore_get_many(self._h, off, length, None, 0, None, 0, ctypes.byref(rows), ctypes.byref(floats)))
        vals = np.empty(max(floats.value, 1), np.float32)
        lens = np.empty(max(rows.value, 1), np.uint32)
        _check(L.bsr_vstore_get_many(self._h, off, length, vals.ctypes.data, vals.size, lens.ctypes.data, lens.size,
                                     ctypes.byref(rows), ctypes.byref(floats)))
        out, pos = [], 0
        for n in lens[:rows.value]:
            out.append(vals[pos:pos + int(n)].copy())
            pos += int(n)
        return out

    def get_many_array(self, slice_args: Optional[SliceArgs] = None, dim: int = 768) -> np.ndarray:
        off, length = self._slice(slice_args)
        cap = max(0, min(length, self.get_count()))
        out = np.empty((max(cap, 1), dim), np.float32)
        got = ctypes.c_uint64(0)
        _check(vstore_lib().bsr_vstore_read_slab(self._h, off, length, dim, out.ctypes.data, cap, ctypes.byref(got)))
        return out[:got.value]

    def get(self, index: int) -> np.ndarray:
        n = ctypes.c_uint32(0)
        L = vstore_lib()
        _check(L.bsr_vstore_get(self._h, index, None, 0, ctypes.byref(n)))
        out = np.empty(max(n.value, 1), np.float32)
        _check(L.bsr_vstore_get(self._h, index, out.ctypes.data, out.size, ctypes.byref(n)))
        return out[:n.value]

    def append(self, vector) -> None:
        self.append_many([vector])

    def append_many(self, vectors) -> None:
        if len(vectors) == 0:
            return
        a = np.ascontiguousarray(np.asarray(vectors, np.float32))
        if a.ndim != 2:
            raise BsrError(-6, "append_many takes equal-length rows")
        _check(vstore_lib().bsr_vstore_append_many(self._h, a.ctypes.data, a.shape[0], a.shape[1]))

    def persist(self) -> None:
        _check(vstore_lib().bsr_vstore_persist(self._h))

    def reload(self, force: bool) -> None:
        _check(vstore_lib().bsr_vstore_reload(self._h, 1 if force else 0))

    def reset(self) -> None:
        _check(vstore_lib().bsr_vstore_reset(self._h))


def get_global_vstore(vstore_dir: str, empty: bool) -> PolarsVectorstore:
    """src/mpi_helpers/vectorstore.rs:16-20: <dir>/global.parquet."""
    buf = ctypes.create_string_buffer(4096)
    _check(vstore_lib().bsr_vstore_global_path(os.fsencode(str(vstore_dir)), buf, len(buf)))
    return PolarsVectorstore(buf.value.decode(), empty)


def get_local_vstore(vstore_dir: str, rank: int, empty: bool) -> PolarsVectorstore:
    """src/mpi_helpers/vectorstore.rs:5-13: <dir>/rank_{rank}.parquet."""
    buf = ctypes.create_string_buffer(4096)
    _check(vstore_lib().bsr_vstore_local_path(os.fsencode(str(vstore_dir)), rank, buf, len(buf)))
    return PolarsVectorstore(buf.value.decode(), empty)


def merge_vector_stores(size: int, vstore_dir: str) -> PolarsVectorstore:
    """src/mpi_helpers/tasks.rs:181-217: an empty global store, then every rank's local store
    appended in rank order (empty ones skipped); the order defines the global row indices the
    search returns.  Like the reference, the merged store is returned, not persisted."""
    global_vs = get_global_vstore(vstore_dir, True)
    total = 0
    for r in range(size):
        local = get_local_vstore(vstore_dir, r, False)
        try:
            n = local.get_count()
            if n == 0:
                continue
            rows = local.get_many_array(None, dim=len(local.get(0)))
            global_vs.append_many(rows)
            total += rows.shape[0]
        finally:
            local.close()
    return global_vs


def merge_vector_stores_into_index(index: "Index", size: int, vstore_dir: str) -> int:
    """f-3 on the device: the rank-order concatenation of merge_vector_stores built directly
    as a GPU-resident shard (each local store's rows appended to the index's HBM slab with
    bsr_index_append), without materialising the global parquet store.  Returns the row count."""
    total = 0
    for r in range(size):
        local = get_local_vstore(vstore_dir, r, False)
        try:
            n = local.get_count()
            if n == 0:
                continue
            index.append_many(local.get_many_array(None, dim=index.dim))
            total += n
        finally:
            local.close()
    return total


def load_index_from_vstore(index: "Index", vstore: PolarsVectorstore, rank: int, size: int) -> None:
    """The read half of compute_local_top_k (src/mpi_helpers/metrics.rs:23-33): this rank's
    interval_by_rank block of the store, straight into the index's HBM shard."""
    _check(vstore_lib().bsr_index_load_vstore(index._h, vstore._h, rank, size))
