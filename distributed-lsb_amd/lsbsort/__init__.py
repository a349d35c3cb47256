"""Python front end of the MI355X-native distributed LSD radix sort.

A thin ctypes binding of the C ABI in ``include/lsb.h`` (library
``distributed-lsb_amd/build/liblsb.so``), mirroring the reference's own
seams so tests read like the reference program:

  ==========================  ==============================================
  reference                   here
  ==========================  ==============================================
  DistributedArray::create    ``World(n, ranks)`` / ``World.rank(...)``
  (mpi/mpi_lsbsort.cpp:137)   (block partition per = ceil(n/P))
  PCG init (:643-666)         ``World.generate()``
  mySort(A, B) (:580-585)     ``World.my_sort()``   (alias ``mySort``)
  globalShuffle (:481-577)    ``World.global_shuffle(d)`` (alias ``globalShuffle``)
  verify (:710-738)           ``World.verify()``
  checkSorted (shmem :180)    ``World.check_sorted()``
  A.print(10) (:171-200)      ``World.print_lines("A", 10)``
  ==========================  ==============================================

Errors from the library raise :class:`LsbError` (the reference aborts on
MPI errors, mpi/mpi_lsbsort.cpp:17-19).  There is no CPU fallback: if the
HIP library is missing or no GPU is present, calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os
import sys
from typing import Optional, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)
# LSB_LIBRARY: another build of the same ABI (A/B timing of kernel variants).
LIB_PATH = os.environ.get("LSB_LIBRARY") or os.path.join(ROOT_DIR, "build", "liblsb.so")
HARNESS_PATH = os.path.join(ROOT_DIR, "build", "hip_lsbsort")
HEADER_PATH = os.path.join(os.path.dirname(ROOT_DIR), "include", "lsb.h")

ELEM_DTYPE = np.dtype([("key", "<u8"), ("val", "<u8")])
UNIQUE_ID_BYTES = 128

LSB_OK = 0
LSB_ERR_VERIFY = 5
DIST_UNIFORM, DIST_ZIPF = 0, 1
K_UPSWEEP, K_SCAN, K_SCATTER, K_EXCHANGE, K_PLACE, K_SORT, K_SEGSORT, K_WIRE, K_PLACE_TAIL = range(9)
KERNEL_NAMES = ("upsweep", "scan", "scatter", "exchange", "place", "sort", "segsort", "wire", "place_tail")
MAX_RANKS = 64
OPT_TIMING, OPT_FORCE_EXCHANGE, OPT_SKIP_CONSTANT_DIGITS, OPT_EXCHANGE_SLICES, OPT_EXCHANGE_P2P = 0, 1, 2, 3, 4
OPT_EXCHANGE_PEER = 5
OPT_ONESWEEP = 6
OPT_EXCHANGE_SELF = 7
OPT_ONESWEEP_SPLIT = 8
OPT_HYBRID = 9
OPT_EXCHANGE_GATHER = 10
OPT_FAIL_ONESWEEP = 11
OPT_REGION_FIRST = 12
OPT_EXCHANGE_CHUNKS = 13
FIRST_COUNT, FIRST_REGIONAL, FIRST_REGIONAL_REDONE = 0, 1, 2
MAX_PASSES = 16


class LsbError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = _lib().lsb_strerror(code).decode()
        super().__init__(f"{where}: lsb error {code}: {msg}")
        self.code = code


_L = None


# -- host collectives (lsb_comm_ops_t) -------------------------------------
_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_size_t)
_ALLTOALLV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                              ctypes.POINTER(ctypes.c_size_t))
_ALLREDUCE_MIN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64))
_BARRIER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


class ExchangeStats(ctypes.Structure):
    """lsb_exchange_stats_t."""
    _fields_ = [("exchanges", ctypes.c_int64), ("calls", ctypes.c_int64),
                ("sent_bytes", ctypes.c_int64 * 64), ("recv_bytes", ctypes.c_int64 * 64),
                ("wire_ms", ctypes.c_double), ("plan_ms", ctypes.c_double), ("place_ms", ctypes.c_double),
                ("place_tail_ms", ctypes.c_double), ("place_bytes", ctypes.c_int64),
                ("placed_records", ctypes.c_int64), ("counted_records", ctypes.c_int64)]


class CommOps(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allgather", _ALLGATHER), ("alltoallv", _ALLTOALLV),
                ("allreduce_min_i64", _ALLREDUCE_MIN), ("barrier", _BARRIER)]


def _bytes_at(ptr, n):
    if n == 0:
        return np.zeros(0, dtype=np.uint8)
    return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ptr))


def _make_comm_ops(comm, P):
    """lsb_comm_ops_t whose callbacks call the Python object `comm`."""
    def guard(fn):
        def wrapped(*a):
            try:
                fn(*a)
                return 0
            except Exception as e:  # a failed collective is an error code, not a crash
                print(f"lsbsort comm callback failed: {e!r}", file=sys.stderr)
                return 1
        return wrapped

    def allgather(_u, send, recv, nbytes):
        _bytes_at(recv, nbytes * P)[:] = comm.allgather(_bytes_at(send, nbytes).copy())

    def alltoallv(_u, send, sc, sd, recv, rc, rd):
        scn = [sc[i] for i in range(P)]
        sdn = [sd[i] for i in range(P)]
        rcn = [rc[i] for i in range(P)]
        rdn = [rd[i] for i in range(P)]
        send_len = max([d + c for d, c in zip(sdn, scn) if c] or [0])
        recv_len = max([d + c for d, c in zip(rdn, rcn) if c] or [0])
        comm.alltoallv(_bytes_at(send, send_len), scn, sdn, _bytes_at(recv, recv_len), rcn, rdn)

    def allreduce_min(_u, v):
        v[0] = int(comm.allreduce_min(int(v[0])))

    def barrier(_u):
        comm.barrier()

    keep = (_ALLGATHER(guard(allgather)), _ALLTOALLV(guard(alltoallv)),
            _ALLREDUCE_MIN(guard(allreduce_min)), _BARRIER(guard(barrier)))
    ops = CommOps(None, *keep)
    return ops, keep


def _lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"HIP library {LIB_PATH} is not built; run `make -C distributed-lsb_amd` "
                "(or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, vp, cp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p
        P64 = ctypes.POINTER(ctypes.c_int64)
        sig = {
            "lsb_per_rank": (i64, [i64, i32]),
            "lsb_here": (i64, [i64, i32, i32]),
            "lsb_create": (i32, [ctypes.POINTER(vp), i64, i32, ctypes.POINTER(ctypes.c_int), i32]),
            "lsb_get_unique_id": (i32, [ctypes.c_char_p]),
            "lsb_device_count": (i32, [ctypes.POINTER(ctypes.c_int)]),
            "lsb_create_rank": (i32, [ctypes.POINTER(vp), i64, i32, i32, i32, i32, ctypes.c_char_p]),
            "lsb_create_rank_ops": (i32, [ctypes.POINTER(vp), i64, i32, i32, i32, i32,
                                          ctypes.POINTER(CommOps)]),
            "lsb_destroy": (None, [vp]),
            "lsb_set_option": (i32, [vp, i32, i64]),
            "lsb_get_last_sort": (i32, [vp, vp, vp, vp]),
            "lsb_get_first_pass": (i32, [vp, vp]),
            "lsb_local_ranks": (i32, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
            "lsb_generate": (i32, [vp]),
            "lsb_generate_ex": (i32, [vp, i32, ctypes.c_double]),
            "lsb_copy_in": (i32, [vp, i32, i64, i64, vp]),
            "lsb_copy_out": (i32, [vp, i32, i64, i64, vp]),
            "lsb_sort": (i32, [vp]),
            "lsb_pass": (i32, [vp, i32]),
            "lsb_sync": (i32, [vp]),
            "lsb_barrier": (i32, [vp]),
            "lsb_verify": (i32, [vp, P64]),
            "lsb_check_sorted": (i32, [vp, ctypes.POINTER(ctypes.c_int)]),
            "lsb_get_kernel_stats": (i32, [vp, i32, P64, ctypes.POINTER(ctypes.c_double)]),
            "lsb_reset_kernel_stats": (i32, [vp]),
            "lsb_get_scatter_elems": (i32, [vp, P64]),
            "lsb_get_pass_stats": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int), P64, P64,
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
            "lsb_get_exchange_bytes": (i32, [vp, P64, P64, P64]),
            "lsb_get_exchange_stats": (i32, [vp, ctypes.POINTER(ExchangeStats)]),
            "lsb_get_placement": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
            "lsb_get_pass_exchange": (i32, [vp, i32, P64, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double)]),
            "lsb_build_info": (cp, []),
            "lsb_rank_footprint": (i32, [i64, i32, i32, i32, P64, P64]),
            "lsb_device_memory": (i32, [i32, P64, P64]),
            "lsb_plan_exchange": (i32, [i64, i32, i32, i32, vp, vp, vp, vp, vp, vp]),
            "lsb_plan_exchange_device": (i32, [i32, i64, i32, i32, i32, vp, vp, vp, vp, vp, vp]),
            "lsb_plan_merge": (i32, [i64, i32, i32, vp, vp, vp, vp, vp, vp]),
            "lsb_strerror": (cp, [i32]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _L = L
    return _L


def _check(code: int, where: str) -> None:
    if code != LSB_OK:
        raise LsbError(code, where)


def per_rank(n: int, P: int) -> int:
    return int(_lib().lsb_per_rank(n, P))


def here(n: int, P: int, r: int) -> int:
    return int(_lib().lsb_here(n, P, r))


def rank_footprint(n: int, P: int, radix_bits: int = 8, with_recv: bool = False) -> dict:
    """lsb_rank_footprint: device bytes one rank of lsb_create(n, P, radix_bits)
    holds ({"bytes"}), and the optional placement probe's transient on top
    ({"probe_bytes"}, from LSB_PLACEMENT_CANDIDATES as set now).  Host
    arithmetic only."""
    b, pb = ctypes.c_int64(), ctypes.c_int64()
    _check(_lib().lsb_rank_footprint(n, P, radix_bits, int(with_recv), ctypes.byref(b), ctypes.byref(pb)),
           "lsb_rank_footprint")
    return {"bytes": b.value, "probe_bytes": pb.value}


def device_memory(dev: int = 0) -> tuple:
    """(free, total) device bytes of device dev (lsb_device_memory)."""
    f, t = ctypes.c_int64(), ctypes.c_int64()
    _check(_lib().lsb_device_memory(dev, ctypes.byref(f), ctypes.byref(t)), "lsb_device_memory")
    return f.value, t.value


def build_info() -> dict:
    """{"sha256": digest of the sources the loaded library was built from,
    "host": build host, "rccl": ncclGetVersion of the loaded RCCL}
    (lsb_build_info)."""
    info = _lib().lsb_build_info().decode()
    return dict(kv.split("=", 1) for kv in info.split())


def source_files() -> list:
    """The library's sources, in the order the Makefile hashes them (its
    SOURCES line, with the RT list of runtime units expanded)."""
    import re
    mk = open(os.path.join(ROOT_DIR, "Makefile")).read()
    rt = re.search(r"^RT\s*:=\s*(.*)$", mk, re.M).group(1).split()
    files = []
    for tok in re.search(r"^SOURCES\s*:=\s*(.*)$", mk, re.M).group(1).split():
        if tok.startswith("$(RT:"):
            files += [f"csrc/{u}.cpp" for u in rt]
        else:
            files.append(tok)
    return files


def source_digest() -> str:
    """sha256 of the library's sources as they are in this tree, in the
    order the Makefile hashes them (SOURCES)."""
    import hashlib
    h = hashlib.sha256()
    for rel in source_files():
        with open(os.path.join(ROOT_DIR, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def get_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _check(_lib().lsb_get_unique_id(buf), "lsb_get_unique_id")
    return buf.raw


def plan_exchange(n: int, P: int, rank: int, hist: np.ndarray, device: Optional[int] = None) -> dict:
    """Exchange plan of rank `rank` for a P x nbuckets count matrix: the host
    planner, or (device=d) the device kernels the runtime runs."""
    hist = np.ascontiguousarray(hist, dtype=np.int64)
    if hist.ndim != 2 or hist.shape[0] != P:
        raise ValueError("hist must be P x nbuckets")
    nb = hist.shape[1]
    out = {k: np.zeros(P, dtype=np.int64) for k in
           ("send_counts", "send_displs", "recv_counts", "recv_displs")}
    out["place_off"] = np.zeros((P, nb), dtype=np.int64)
    args = (n, P, rank, nb, hist.ctypes.data, out["send_counts"].ctypes.data,
            out["send_displs"].ctypes.data, out["recv_counts"].ctypes.data,
            out["recv_displs"].ctypes.data, out["place_off"].ctypes.data)
    if device is None:
        _check(_lib().lsb_plan_exchange(*args), "lsb_plan_exchange")
    else:
        _check(_lib().lsb_plan_exchange_device(device, *args), "lsb_plan_exchange_device")
    return out


def plan_merge(n: int, P: int, rank: int, below: np.ndarray, upto: np.ndarray) -> dict:
    """Whole-key exchange plan of rank `rank` (lsb_plan_merge): below/upto are
    P x (P-1) counts of keys <, <= the key at global position q * per."""
    below = np.ascontiguousarray(below, dtype=np.int64).reshape(P, max(P - 1, 0))
    upto = np.ascontiguousarray(upto, dtype=np.int64).reshape(P, max(P - 1, 0))
    out = {k: np.zeros(P, dtype=np.int64) for k in
           ("send_counts", "send_displs", "recv_counts", "recv_displs")}
    _check(_lib().lsb_plan_merge(n, P, rank, below.ctypes.data, upto.ctypes.data,
                                 out["send_counts"].ctypes.data, out["send_displs"].ctypes.data,
                                 out["recv_counts"].ctypes.data, out["recv_displs"].ctypes.data),
           "lsb_plan_merge")
    return out


class World:
    """One sort context: a block-distributed pair of arrays A, B over P ranks.

    ``World(n, ranks=P)`` drives all P ranks from this process (logical
    ranks; ``devices[r]`` per rank, default all on device 0).
    ``World.rank(n, P, r, device, uid)`` is one rank of a multi-process RCCL
    world (one process per GPU).
    """

    def __init__(self, n: int, ranks: int = 1, devices: Optional[Sequence[int]] = None,
                 radix_bits: int = 8, _handle=None, _P=None):
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
            self.P = _P
        else:
            devs = None
            if devices is not None:
                if len(devices) != ranks:
                    raise ValueError("one device per rank")
                devs = (ctypes.c_int * ranks)(*devices)
            _check(_lib().lsb_create(ctypes.byref(self._h), n, ranks, devs, radix_bits),
                   "lsb_create")
            self.P = ranks
        self.n = n
        self.per = per_rank(n, self.P)
        self.radix_bits = radix_bits
        first, nl = ctypes.c_int(), ctypes.c_int()
        _check(_lib().lsb_local_ranks(self._h, ctypes.byref(first), ctypes.byref(nl)),
               "lsb_local_ranks")
        self.local_ranks = list(range(first.value, first.value + nl.value))

    @classmethod
    def rank(cls, n: int, num_ranks: int, rank: int, device: int, unique_id: bytes,
             radix_bits: int = 8) -> "World":
        h = ctypes.c_void_p()
        _check(_lib().lsb_create_rank(ctypes.byref(h), n, num_ranks, rank, device, radix_bits,
                                      unique_id), "lsb_create_rank")
        return cls(n, _handle=h, _P=num_ranks, radix_bits=radix_bits)

    @classmethod
    def rank_ops(cls, n: int, num_ranks: int, rank: int, device: int, comm,
                 radix_bits: int = 8) -> "World":
        """One rank per process with host collectives instead of RCCL.

        `comm` provides (numpy uint8 buffers, host memory):
          allgather(send) -> P * len(send) bytes, rank-major
          alltoallv(send, send_counts, send_displs, recv, recv_counts, recv_displs)  (bytes)
          allreduce_min(int) -> int
          barrier()
        Any transport works (MPI, gloo, sockets); see lsb_create_rank_ops.
        """
        ops, keep = _make_comm_ops(comm, num_ranks)
        h = ctypes.c_void_p()
        _check(_lib().lsb_create_rank_ops(ctypes.byref(h), n, num_ranks, rank, device, radix_bits,
                                          ctypes.byref(ops)), "lsb_create_rank_ops")
        w = cls(n, _handle=h, _P=num_ranks, radix_bits=radix_bits)
        w._comm_keep = (ops, keep)  # the callbacks must outlive the context
        return w

    # -- lifecycle --------------------------------------------------------
    def close(self) -> None:
        if self._h:
            _lib().lsb_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, opt: int, value: int) -> None:
        _check(_lib().lsb_set_option(self._h, opt, value), "lsb_set_option")

    # -- data ---------------------------------------------------------------
    def here(self, r: int) -> int:
        return here(self.n, self.P, r)

    def generate(self, dist: str = "uniform", s: float = 1.1) -> None:
        """pcg64(rank) input; dist "zipf" maps each draw to a skewed key."""
        if dist == "uniform":
            _check(_lib().lsb_generate(self._h), "lsb_generate")
        elif dist == "zipf":
            _check(_lib().lsb_generate_ex(self._h, DIST_ZIPF, s), "lsb_generate_ex")
        else:
            raise ValueError(dist)

    def copy_in(self, rank: int, arr: np.ndarray, off: int = 0) -> None:
        arr = np.ascontiguousarray(arr, dtype=ELEM_DTYPE)
        _check(_lib().lsb_copy_in(self._h, rank, off, arr.size, arr.ctypes.data if arr.size else None),
               "lsb_copy_in")

    def copy_out(self, rank: int, off: int = 0, cnt: Optional[int] = None) -> np.ndarray:
        if cnt is None:
            cnt = self.here(rank) - off
        out = np.empty(cnt, dtype=ELEM_DTYPE)
        _check(_lib().lsb_copy_out(self._h, rank, off, cnt, out.ctypes.data if cnt else None),
               "lsb_copy_out")
        return out

    def scatter_global(self, arr: np.ndarray) -> None:
        """Load a global array of n records into the block partition."""
        arr = np.ascontiguousarray(arr, dtype=ELEM_DTYPE)
        if arr.size != self.n:
            raise ValueError("need exactly n records")
        for r in self.local_ranks:
            h = self.here(r)
            if h:
                self.copy_in(r, arr[r * self.per: r * self.per + h])

    def gather_global(self) -> np.ndarray:
        """A[0:n] in global order (every rank must be local)."""
        if len(self.local_ranks) != self.P:
            raise RuntimeError("gather_global needs all ranks in this process")
        parts = [self.copy_out(r) for r in range(self.P)]
        return np.concatenate(parts) if parts else np.empty(0, dtype=ELEM_DTYPE)

    # -- the hot path -------------------------------------------------------
    def my_sort(self) -> None:
        _check(_lib().lsb_sort(self._h), "lsb_sort")

    def global_shuffle(self, digit: int) -> None:
        _check(_lib().lsb_pass(self._h, digit), "lsb_pass")

    mySort = my_sort
    globalShuffle = global_shuffle

    def sync(self) -> None:
        _check(_lib().lsb_sync(self._h), "lsb_sync")

    def barrier(self) -> None:
        _check(_lib().lsb_barrier(self._h), "lsb_barrier")

    # -- checks ---------------------------------------------------------------
    def verify(self):
        """(ok, first_bad_global_index) of the O(n) stable-sort invariant."""
        bad = ctypes.c_int64(-1)
        rc = _lib().lsb_verify(self._h, ctypes.byref(bad))
        if rc not in (LSB_OK, LSB_ERR_VERIFY):
            _check(rc, "lsb_verify")
        return rc == LSB_OK, int(bad.value)

    def check_sorted(self) -> bool:
        s = ctypes.c_int(0)
        _check(_lib().lsb_check_sorted(self._h, ctypes.byref(s)), "lsb_check_sorted")
        return bool(s.value)

    checkSorted = check_sorted

    def print_lines(self, name: str = "A", n_per_rank: int = 10):
        """The lines DistributedArray::print emits (mpi/mpi_lsbsort.cpp:171-200)."""
        lines = []
        if n_per_rank * self.P >= self.n:
            lines.append(f"{name}: displaying all {self.n} elements")
        else:
            lines.append(f"{name}: displaying first {n_per_rank} elements on each rank"
                         f" out of {self.n} elements")
        for r in self.local_ranks:
            h = self.here(r)
            k = min(n_per_rank, h)
            for i, e in enumerate(self.copy_out(r, 0, k)):
                lines.append(f"{name}[{r * self.per + i}] = ({int(e['key']):016x},{int(e['val'])})")
            if k < h:
                lines.append("...")
        return lines

    # -- measurement ----------------------------------------------------------
    def set_timing(self, on: bool = True) -> None:
        self.set_option(OPT_TIMING, 1 if on else 0)

    def last_sort(self) -> tuple:
        """(local 8-bit passes, exchanges, varying key bits) of the last my_sort."""
        lp, ex, vb = ctypes.c_int(), ctypes.c_int(), ctypes.c_uint64()
        _check(_lib().lsb_get_last_sort(self._h, ctypes.byref(lp), ctypes.byref(ex), ctypes.byref(vb)),
               "lsb_get_last_sort")
        return int(lp.value), int(ex.value), int(vb.value)

    def first_pass(self) -> int:
        """How the last my_sort began (lsb_get_first_pass): FIRST_COUNT,
        FIRST_REGIONAL or FIRST_REGIONAL_REDONE."""
        f = ctypes.c_int()
        _check(_lib().lsb_get_first_pass(self._h, ctypes.byref(f)), "lsb_get_first_pass")
        return int(f.value)

    def kernel_stats(self) -> dict:
        out = {}
        for kid, name in enumerate(KERNEL_NAMES):
            n = ctypes.c_int64()
            ms = ctypes.c_double()
            _check(_lib().lsb_get_kernel_stats(self._h, kid, ctypes.byref(n), ctypes.byref(ms)),
                   "lsb_get_kernel_stats")
            out[name] = (int(n.value), float(ms.value))
        return out

    def pass_stats(self) -> list:
        """Per local pass that ran since the last reset (lsb_get_pass_stats):
        dicts with pass, shift, launches, elems and the device ms of its count,
        scatter, exchange and placement work, summed over launches."""
        out = []
        for p in range(MAX_PASSES):
            sh, la, el = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64()
            ms = [ctypes.c_double() for _ in range(4)]
            _check(_lib().lsb_get_pass_stats(self._h, p, ctypes.byref(sh), ctypes.byref(la), ctypes.byref(el),
                                             *[ctypes.byref(x) for x in ms]), "lsb_get_pass_stats")
            if sh.value < 0:
                continue
            xb, wire, tail = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            _check(_lib().lsb_get_pass_exchange(self._h, p, ctypes.byref(xb), ctypes.byref(wire),
                                                ctypes.byref(tail)), "lsb_get_pass_exchange")
            out.append({"pass": p, "shift": int(sh.value), "launches": int(la.value), "elems": int(el.value),
                        "ms_count": ms[0].value, "ms_scatter": ms[1].value, "ms_exchange": ms[2].value,
                        "ms_place": ms[3].value, "exchange_bytes": int(xb.value), "ms_wire": wire.value,
                        "ms_place_tail": tail.value})
        return out

    def placement(self, rank: Optional[int] = None) -> dict:
        """lsb_get_placement: how rank's A and B were chosen among candidate
        buffers (candidates 0: allocated as they came) and the probe copy's ms
        for the chosen pair, the first two allocated and the slowest pair."""
        r = self.local_ranks[0] if rank is None else rank
        k = ctypes.c_int()
        ms = [ctypes.c_double() for _ in range(3)]
        _check(_lib().lsb_get_placement(self._h, r, ctypes.byref(k), *[ctypes.byref(x) for x in ms]),
               "lsb_get_placement")
        return {"candidates": int(k.value), "chosen_ms": round(ms[0].value, 4),
                "first_pair_ms": round(ms[1].value, 4), "worst_ms": round(ms[2].value, 4)}

    def exchange_stats(self) -> dict:
        """lsb_get_exchange_stats: the exchange steps since the last reset
        (bytes per peer, wire / plan / placement / tail ms, placement bytes)."""
        st = ExchangeStats()
        _check(_lib().lsb_get_exchange_stats(self._h, ctypes.byref(st)), "lsb_get_exchange_stats")
        return {"exchanges": int(st.exchanges), "calls": int(st.calls),
                "sent_bytes": [int(x) for x in st.sent_bytes[:self.P]],
                "recv_bytes": [int(x) for x in st.recv_bytes[:self.P]],
                "wire_ms": st.wire_ms, "plan_ms": st.plan_ms, "place_ms": st.place_ms,
                "place_tail_ms": st.place_tail_ms, "place_bytes": int(st.place_bytes),
                "placed_records": int(st.placed_records), "counted_records": int(st.counted_records)}

    def reset_kernel_stats(self) -> None:
        _check(_lib().lsb_reset_kernel_stats(self._h), "lsb_reset_kernel_stats")

    def scatter_elems(self) -> int:
        e = ctypes.c_int64()
        _check(_lib().lsb_get_scatter_elems(self._h, ctypes.byref(e)), "lsb_get_scatter_elems")
        return int(e.value)

    def exchange_bytes(self) -> tuple:
        """(calls, bytes, largest call's bytes) handed to the all-to-all collective."""
        c, b, mx = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _check(_lib().lsb_get_exchange_bytes(self._h, ctypes.byref(c), ctypes.byref(b), ctypes.byref(mx)),
               "lsb_get_exchange_bytes")
        return int(c.value), int(b.value), int(mx.value)


def mySort(world: World) -> None:  # noqa: N802 - reference name
    world.my_sort()


def globalShuffle(world: World, digit: int) -> None:  # noqa: N802 - reference name
    world.global_shuffle(digit)
