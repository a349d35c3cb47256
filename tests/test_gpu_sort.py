"""Parity of the HIP path against the oracle and the reference's own outputs.

Everything here calls through the C ABI (build/liblsb.so) on the GPU.
Bar: bit-exact (integer / index work).  Multi-rank cases run P logical ranks
on one GPU (lsb_create): the same kernels, plan and placement as the RCCL
path, with the all-to-all done by device copies — the single-GPU analogue of
`mpirun -n P mpi_lsbsort` on one host.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = np.dtype([("key", "<u8"), ("val", "<u8")])


def _records(rows):
    a = np.zeros(len(rows), dtype=DT)
    for i, r in enumerate(rows):
        a[i] = (int(r[1], 16), r[2])
    return a


def _sorted_world(lsbsort, arr, P):
    w = lsbsort.World(arr.size, ranks=P)
    w.scatter_global(arr)
    w.my_sort()
    out = w.gather_global()
    return w, out


# --------------------------------------------------------------- generation
@pytest.mark.parametrize("n,P", [(1, 1), (20, 2), (4097, 1), (100_003, 4), (17, 8), (3, 4)])
def test_generate_matches_reference_input(lsb_built, oracle_mod, n, P):
    with lsb_built.World(n, ranks=P) as w:
        w.generate()
        assert np.array_equal(w.gather_global(), oracle_mod.generate(n, P))


# --------------------------------------------------------------- golden rows
@pytest.mark.parametrize("row", range(5))
def test_golden_digests(lsb_built, oracle_mod, digests, row):
    d = digests["rows"][row]
    with lsb_built.World(d["n"], ranks=d["P"]) as w:
        w.generate()
        assert oracle_mod.digest(w.gather_global()) == d["input"]
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == d["output"]
        ok, bad = w.verify()
        assert ok and bad == -1
        assert w.check_sorted()


def test_reference_print_vectors(lsb_built, ref_vectors):
    for case in ref_vectors["cases"]:
        n, P = case["n"], case["P"]
        with lsb_built.World(n, ranks=P) as w:
            w.generate()
            before = w.gather_global()
            w.my_sort()
            after = w.gather_global()
            for rows, arr in ((case["input"], before), (case["output"], after)):
                idx = [r[0] for r in rows]
                np.testing.assert_array_equal(arr[idx], _records(rows))


def test_print_lines_match_reference_format(lsb_built, ref_vectors):
    case = next(c for c in ref_vectors["cases"] if c["n"] == 20 and c["P"] == 2)
    with lsb_built.World(20, ranks=2) as w:
        w.generate()
        w.my_sort()
        lines = w.print_lines("A", 10)
    assert lines[0] == "A: displaying all 20 elements"
    expect = [f"A[{i}] = ({k},{v})" for i, k, v in case["output"]]
    assert lines[1:] == expect


# ------------------------------------------------------------- single pass
@pytest.mark.parametrize("n", [1, 63, 4095, 4096, 4097, 300_001])
def test_single_pass_matches_local_shuffle(lsb_built, oracle_mod, n):
    rng = np.random.default_rng(n)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    with lsb_built.World(n, ranks=1) as w:
        w.copy_in(0, a)
        cur = a
        for d in (0, 3, 7):
            w.global_shuffle(d)
            cur, _ = oracle_mod.local_pass(cur, 8, d)
            assert np.array_equal(w.copy_out(0), cur)


# ------------------------------------------------------- adversarial inputs
def _dist(name, n, rng):
    a = np.zeros(n, dtype=DT)
    a["val"] = np.arange(n, dtype=np.uint64)
    if name == "all_equal":
        a["key"] = np.uint64(0xDEADBEEF12345678)
    elif name == "two_keys":
        a["key"] = np.where(rng.random(n) < 0.5, 7, 0xFFFFFFFFFFFFFFFF).astype(np.uint64)
    elif name == "hot_bucket":
        k = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
        hot = rng.random(n) < 0.9
        k[hot] = (k[hot] & ~np.uint64(0xFF00FF)) | np.uint64(0x2A002A)
        a["key"] = k
    elif name == "high_bits_only":
        a["key"] = rng.integers(0, 256, n, dtype=np.uint64) << np.uint64(56)
    elif name == "zipf":
        z = np.minimum(rng.zipf(1.1, n), 2**20).astype(np.uint64)
        a["key"] = z * np.uint64(0x9E3779B97F4A7C15)  # spread over all digits
    elif name == "sorted":
        a["key"] = np.sort(rng.integers(0, 2**64 - 1, n, dtype=np.uint64))
    elif name == "reverse":
        a["key"] = np.sort(rng.integers(0, 2**64 - 1, n, dtype=np.uint64))[::-1]
    elif name == "small_range":
        a["key"] = rng.integers(0, 3, n, dtype=np.uint64)
    else:
        raise KeyError(name)
    return a


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "high_bits_only",
                                  "zipf", "sorted", "reverse", "small_range"])
@pytest.mark.parametrize("P", [1, 3, 8])
def test_distributions_bit_exact(lsb_built, oracle_mod, name, P):
    rng = np.random.default_rng(hash((name, P)) & 0xFFFF)
    n = 200_003
    a = _dist(name, n, rng)
    _, out = _sorted_world(lsb_built, a, P)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


@pytest.mark.parametrize("n,P", [(0, 1), (0, 3), (1, 1), (1, 4), (2, 8), (5, 8), (9, 8),
                                 (4096 * 3 + 1, 2), (4096 * 513 + 7, 1)])
def test_ragged_and_tiny(lsb_built, oracle_mod, n, P):
    rng = np.random.default_rng(n * 31 + P)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64) & np.uint64(0xF0F0F0F0F0F0F0F0)
    a["val"] = np.arange(n, dtype=np.uint64)
    _, out = _sorted_world(lsb_built, a, P)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


# ------------------------------------------------- constant-digit skipping
def _masked_keys(n, mask, rng):
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64) & np.uint64(mask)
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


# (key mask, radix bits, P) -> 8-bit local passes and exchanges lsb_sort must
# run, with reduce-then-scan passes (digit 0 always runs: the key span comes
# out of its count kernel) and with single-read passes (k_subhist reads the
# span before any pass, so a constant digit 0 is skipped like any other, at
# P = 1 too).
@pytest.mark.parametrize("mask,bits,P,passes,exchanges,passes_os,exchanges_os", [
    (0xFFFFFFFF, 8, 1, 4, 0, 4, 0),                 # keys < 2^32: bytes 4..7 constant
    (0xFFFF0000000000FF, 8, 1, 3, 0, 3, 0),         # bytes 1..5 constant
    (0xFFFFFFFFFFFFFFFF, 8, 1, 8, 0, 8, 0),         # nothing to skip
    (0x0, 8, 1, 1, 0, 0, 0),                        # all keys 0: nothing (reduce-scan: the first pass)
    (0xFFFFFFFFFFFFFF00, 8, 1, 8, 0, 7, 0),         # byte 0 constant (keys multiples of 256)
    (0x0000000000FFFFFF, 8, 3, 3, 3, 3, 3),         # 3 digits, each with its exchange
    (0x0000000000FFFFFF, 16, 3, 3, 2, 3, 2),        # 16-bit: digits 0,1; byte 3 skipped
    (0xFF00000000000000, 16, 4, 3, 2, 1, 1),        # 16-bit: digit 3's high byte (+ digit 0 forced)
    (0x00000000FFFF0000, 16, 8, 4, 2, 2, 1),        # digit 1 (+ digit 0 forced)
    # 16-bit: digit 1's low byte constant, so the pass after exchange 0 is
    # digit 1's high byte, gathered and counting the 65536 digits
    # (k_onesweep<..., C16, GATHER>)
    (0x00000000FF00FFFF, 16, 3, 3, 2, 3, 2),
])
@pytest.mark.parametrize("onesweep", [1, 0])
def test_constant_digits_skipped(lsb_built, oracle_mod, mask, bits, P, passes, exchanges,
                                 passes_os, exchanges_os, onesweep):
    rng = np.random.default_rng(mask & 0xFFFF ^ P)
    a = _masked_keys(100_003, mask, rng)
    with lsb_built.World(a.size, ranks=P, radix_bits=bits) as w:
        w.set_option(lsb_built.OPT_ONESWEEP, onesweep)
        w.scatter_global(a)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))
        lp, ex, varying = w.last_sort()
        assert (lp, ex) == ((passes_os, exchanges_os) if onesweep else (passes, exchanges))
        assert varying & ~mask == 0


def test_constant_digit_skipping_can_be_disabled(lsb_built, oracle_mod):
    a = _masked_keys(50_000, 0xFFFF, np.random.default_rng(7))
    with lsb_built.World(a.size, ranks=2) as w:
        w.set_option(lsb_built.OPT_SKIP_CONSTANT_DIGITS, 0)
        w.scatter_global(a)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))
        assert w.last_sort() == (8, 8, 2**64 - 1)


def test_constant_digits_skipped_over_rccl(lsb_built, oracle_mod):
    """The span is all-gathered over RCCL before any digit is skipped."""
    a = _masked_keys(70_001, 0x00FF00FF, np.random.default_rng(11))
    uid = lsb_built.get_unique_id()
    w = lsb_built.World.rank(a.size, 1, 0, 0, uid, radix_bits=16)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.copy_in(0, a, 0)
        w.my_sort()
        w.sync()
        assert np.array_equal(w.copy_out(0), oracle_mod.stable_sort(a))
        # byte 0 (digit 0's high byte is constant), byte 2; digits 0 and 1
        assert w.last_sort()[:2] == (2, 2)
    finally:
        w.close()


def test_uniform_input_runs_every_pass(lsb_built):
    with lsb_built.World(1 << 20, ranks=1) as w:
        w.generate()
        w.my_sort()
        assert w.last_sort() == (8, 0, 2**64 - 1)
        assert w.verify() == (True, -1)


# ------------------------------------------------------------------ checks
def test_verify_catches_corruption(lsb_built):
    n, P = 100_000, 2
    with lsb_built.World(n, ranks=P) as w:
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        part = w.copy_out(1, 0, 8)
        part[[3, 4]] = part[[4, 3]]  # breaks order at global per+3
        w.copy_in(1, part, 0)
        ok, bad = w.verify()
        assert not ok and bad == w.per + 3
        assert not w.check_sorted()
        part[[3, 4]] = part[[4, 3]]
        part[5]["val"] ^= 1  # key no longer PCG(val): stable order broken
        w.copy_in(1, part, 0)
        ok, bad = w.verify()
        assert not ok and bad in (w.per + 4, w.per + 5)
        assert w.check_sorted()  # keys still in order


def test_check_sorted_rank_boundary(lsb_built):
    n, P = 10_000, 4
    with lsb_built.World(n, ranks=P) as w:
        w.generate()
        w.my_sort()
        last = w.copy_out(0, w.per - 1, 1)
        first = w.copy_out(1, 0, 1)
        w.copy_in(0, first, w.per - 1)
        w.copy_in(1, last, 0)
        assert not w.check_sorted()


# ------------------------------------------------------- exchange / RCCL paths
def test_forced_exchange_at_p1(lsb_built, oracle_mod, digests):
    d = next(r for r in digests["rows"] if r["P"] == 1)
    with lsb_built.World(d["n"], ranks=1) as w:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == d["output"]


@pytest.mark.parametrize("slices", [1, 3, 7])
@pytest.mark.parametrize("n,P,bits", [(100_003, 2, 8), (100_003, 5, 16), (250_001, 8, 8),
                                      (9, 8, 16), (13, 3, 8)])
def test_exchange_slices(lsb_built, oracle_mod, slices, n, P, bits):
    """The all-to-all cut into slices, each placed while the next is in flight."""
    rng = np.random.default_rng(n + 7 * P + slices)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["key"][rng.random(n) < 0.3] = np.uint64(0x1234)  # heavy duplicates: uneven segments
    a["val"] = np.arange(n, dtype=np.uint64)
    with lsb_built.World(n, ranks=P, radix_bits=bits) as w:
        w.set_option(lsb_built.OPT_EXCHANGE_SLICES, slices)
        w.scatter_global(a)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))


# ------------------------------------------------ peer-store exchange (opt-in)
@pytest.mark.parametrize("row", range(5))
@pytest.mark.parametrize("bits", [8, 16])
def test_peer_exchange_golden_digests(lsb_built, oracle_mod, digests, row, bits):
    d = digests["rows"][row]
    with lsb_built.World(d["n"], ranks=d["P"], radix_bits=bits) as w:
        w.set_option(lsb_built.OPT_EXCHANGE_PEER, 1)
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == d["output"]
        assert w.verify() == (True, -1)


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "zipf", "small_range"])
@pytest.mark.parametrize("P,bits", [(3, 8), (8, 16)])
def test_peer_exchange_distributions(lsb_built, oracle_mod, name, P, bits):
    rng = np.random.default_rng(hash((name, P, bits)) & 0xFFFF)
    a = _dist(name, 100_003, rng)
    with lsb_built.World(a.size, ranks=P, radix_bits=bits) as w:
        w.set_option(lsb_built.OPT_EXCHANGE_PEER, 1)
        w.scatter_global(a)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))


@pytest.mark.parametrize("n,P", [(0, 3), (1, 4), (9, 8), (4096 * 3 + 1, 2)])
def test_peer_exchange_tiny(lsb_built, oracle_mod, n, P):
    a = _masked_keys(n, 0xF0F0F0F0F0F0F0F0, np.random.default_rng(n + P))
    with lsb_built.World(n, ranks=P) as w:
        w.set_option(lsb_built.OPT_EXCHANGE_PEER, 1)
        w.scatter_global(a)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))


def test_peer_exchange_rccl_world_of_one(lsb_built, oracle_mod, digests):
    d = next(r for r in digests["rows"] if r["P"] == 1)
    w = lsb_built.World.rank(d["n"], 1, 0, 0, lsb_built.get_unique_id(), radix_bits=16)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.set_option(lsb_built.OPT_EXCHANGE_PEER, 1)
        w.generate()
        w.my_sort()
        w.sync()
        assert oracle_mod.digest(w.copy_out(0)) == d["output"]
    finally:
        w.close()


def test_error_codes_on_a_context(lsb_built):
    """Bad arguments on a live context return LSB_ERR_INVALID and leave it usable."""
    import ctypes
    lib = lsb_built._lib()
    with lsb_built.World(1000, ranks=2) as w:
        h = w._h
        buf = np.zeros(600, dtype=DT)
        assert lib.lsb_copy_in(h, 2, 0, 1, buf.ctypes.data) == 1          # no rank 2
        assert lib.lsb_copy_in(h, 0, 400, 101, buf.ctypes.data) == 1      # past per = 500
        assert lib.lsb_copy_out(h, 0, -1, 1, buf.ctypes.data) == 1
        assert lib.lsb_copy_in(h, 0, 0, 1, None) == 1
        assert lib.lsb_pass(h, 8) == 1 and lib.lsb_pass(h, -1) == 1       # 8-bit: digits 0..7
        assert lib.lsb_set_option(h, 99, 1) == 1
        assert lib.lsb_generate_ex(h, 7, 0.0) == 1
        assert lib.lsb_generate_ex(h, lsb_built.DIST_ZIPF, 0.0) == 1
        assert lib.lsb_get_kernel_stats(h, len(lsb_built.KERNEL_NAMES), None, None) == 1
        first, num = ctypes.c_int(), ctypes.c_int()
        assert lib.lsb_local_ranks(h, ctypes.byref(first), ctypes.byref(num)) == 0
        assert (first.value, num.value) == (0, 2)
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)


def test_exchange_slices_option_range(lsb_built):
    with lsb_built.World(10, ranks=2) as w:
        for bad in (0, 65):
            with pytest.raises(lsb_built.LsbError):
                w.set_option(lsb_built.OPT_EXCHANGE_SLICES, bad)


@pytest.mark.parametrize("p2p", [0, 1])
def test_rccl_world_of_one(lsb_built, oracle_mod, digests, p2p):
    """ncclAllToAllv (default) and grouped ncclSend/ncclRecv."""
    d = next(r for r in digests["rows"] if r["P"] == 1)
    uid = lsb_built.get_unique_id()
    w = lsb_built.World.rank(d["n"], 1, 0, 0, uid)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.set_option(lsb_built.OPT_EXCHANGE_P2P, p2p)
        w.generate()
        w.barrier()
        w.my_sort()
        w.barrier()
        assert oracle_mod.digest(w.copy_out(0)) == d["output"]
        assert w.verify() == (True, -1)
        assert w.check_sorted()
    finally:
        w.close()


@pytest.mark.parametrize("lg,bits,slices", [(27, 16, 0), (28, 16, 0), (28, 8, 1), (28, 64, 1)])
def test_world_of_one_large_calls(lsb_built, lg, bits, slices):
    """The bench's x16 extra at smaller sizes: every record through
    ncclAllToAllv of a world-of-one RCCL communicator, with slices whose
    per-peer range reaches 1 GiB (2^27 records, first halving slice), 2 GiB
    (2^28) and, in one slice, 4 GiB.  RCCL moved ranges of 2 GiB or more
    wrongly (verify false at 2^28 in round 5); the runtime now cuts such a
    call into calls of at most 1 GiB per peer (coll_alltoallv_u64)."""
    n = 1 << lg
    w = lsb_built.World.rank(n, 1, 0, 0, lsb_built.get_unique_id(), radix_bits=bits)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.set_option(lsb_built.OPT_EXCHANGE_SELF, 1)
        if slices:
            w.set_option(lsb_built.OPT_EXCHANGE_SLICES, slices)
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        assert w.exchange_stats()["sent_bytes"][0] > 0
    finally:
        w.close()


@pytest.mark.parametrize("bits,slices", [(16, 4), (8, 3), (64, 5)])
def test_exchange_stats_world_of_one(lsb_built, oracle_mod, digests, bits, slices):
    """lsb_get_exchange_stats through real RCCL: a world of one with the
    exchange forced and the self segment sent through ncclAllToAllv, so every
    record crosses the collective once per exchange digit (16 B each), in
    `slices` calls; the wire, plan, placement and tail times are timed and
    the placement bytes follow the gathered-pass rule (the last exchange
    places, 32 B per record; the others count, 16 B).  The whole key: one
    exchange, one merge level (a single run is copied)."""
    d = next(r for r in digests["rows"] if r["P"] == 1)
    n = d["n"]
    w = lsb_built.World.rank(n, 1, 0, 0, lsb_built.get_unique_id(), radix_bits=bits)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.set_option(lsb_built.OPT_EXCHANGE_SELF, 1)
        w.set_option(lsb_built.OPT_EXCHANGE_SLICES, slices)
        w.generate()
        w.reset_kernel_stats()
        w.set_timing(True)
        w.my_sort()
        w.sync()
        x = w.exchange_stats()
        assert oracle_mod.digest(w.copy_out(0)) == d["output"]
        ex = 1 if bits == 64 else 64 // bits
        assert x["exchanges"] == ex and x["calls"] == ex * slices
        assert x["sent_bytes"] == [16 * n * ex] and x["recv_bytes"] == [16 * n * ex]
        assert x["wire_ms"] > 0 and x["plan_ms"] > 0 and x["place_ms"] > 0 and x["place_tail_ms"] >= 0
        if bits == 64:
            assert x["placed_records"] == n and x["place_bytes"] == 32 * n  # one level: the single run copied
        else:
            assert x["placed_records"] == n and x["counted_records"] == n * (ex - 1)
            assert x["place_bytes"] == 32 * n + 16 * n * (ex - 1)
            rows = w.pass_stats()
            xrows = [r for r in rows if r["exchange_bytes"]]
            assert len(xrows) == ex and all(r["exchange_bytes"] == 16 * n for r in xrows)
            assert all(r["ms_wire"] > 0 and r["ms_exchange"] >= r["ms_wire"] for r in xrows)
        w.reset_kernel_stats()
        assert w.exchange_stats()["sent_bytes"] == [0]
    finally:
        w.close()


@pytest.mark.parametrize("onesweep", [1, 0])
def test_kernel_stats(lsb_built, onesweep):
    with lsb_built.World(1 << 20, ranks=1) as w:
        w.set_option(lsb_built.OPT_ONESWEEP, onesweep)
        w.generate()
        w.set_timing(True)
        w.my_sort()
        st = w.kernel_stats()
        # single-read passes: one count read per sort, not one per pass
        counts = 1 if onesweep else 8
        assert st["scatter"][0] == 8 and st["upsweep"][0] == counts and st["sort"][0] == 1
        assert st["scatter"][1] > 0
        assert w.scatter_elems() == 8 << 20


@pytest.mark.parametrize("onesweep", [1, 0])
def test_pass_stats(lsb_built, onesweep):
    """lsb_get_pass_stats: one row per local pass, in order,
    whose scatter times add up to the kernel totals."""
    n = 1 << 20
    with lsb_built.World(n, ranks=1) as w:
        w.set_option(lsb_built.OPT_ONESWEEP, onesweep)
        w.generate()
        w.set_timing(True)
        for _ in range(2):
            w.my_sort()
        rows = w.pass_stats()
        st = w.kernel_stats()
        assert [r["pass"] for r in rows] == list(range(8))
        assert [r["shift"] for r in rows] == [8 * p for p in range(8)]
        assert all(r["launches"] == 2 and r["elems"] == 2 * n and r["ms_scatter"] > 0 for r in rows)
        assert sum(r["ms_scatter"] for r in rows) == pytest.approx(st["scatter"][1], rel=1e-9)
        assert sum(r["ms_count"] for r in rows) == pytest.approx(st["upsweep"][1] + st["scan"][1], rel=1e-9)
        # single-read passes: the one count read per sort is filed under pass 0
        assert (rows[0]["ms_count"] > 0) and all((r["ms_count"] > 0) == (not onesweep) for r in rows[1:])
        assert all(r["ms_exchange"] == 0 and r["ms_place"] == 0 for r in rows)
        w.reset_kernel_stats()
        assert w.pass_stats() == []


def test_pass_stats_exchange_and_skipped_digits(lsb_built, oracle_mod):
    """Exchanges are filed under the local pass before them; constant bytes
    are not passes (keys < 2^24: bytes 0-2 vary)."""
    rng = np.random.default_rng(3)
    a = _masked_keys(200_003, 0xFFFFFF, rng)
    with lsb_built.World(a.size, ranks=2, radix_bits=16) as w:
        w.scatter_global(a)
        w.set_timing(True)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))
        rows = w.pass_stats()
        assert [r["shift"] for r in rows] == [0, 8, 16]
        # 16-bit exchange digits: after byte 1 (digit 0) and byte 2 (digit 1)
        assert [r["ms_exchange"] > 0 for r in rows] == [False, True, True]
        assert [r["ms_place"] > 0 for r in rows] == [False, True, True]
        assert all(r["elems"] == a.size for r in rows)  # both ranks' records
    with pytest.raises(lsb_built.LsbError):
        lsb_built._check(lsb_built._lib().lsb_get_pass_stats(None, 0, None, None, None, None, None, None,
                                                             None), "null context")


def _rebalanced_hist(rng, P, nb, n, here, skew):
    """Random P x nb count matrix whose row r sums to here(n, P, r)."""
    if skew:
        p = rng.dirichlet(np.full(nb, 0.05))
    else:
        p = np.full(nb, 1.0 / nb)
    return np.stack([rng.multinomial(here[r], p) for r in range(P)]).astype(np.int64)


@pytest.mark.parametrize("P,nb,n,skew", [(1, 256, 10_000, False), (2, 256, 0, False),
                                          (3, 256, 7, True), (5, 65536, 1_000_003, False),
                                          (7, 256, 100_000, True), (8, 65536, 5_000_000, True),
                                          (64, 256, 1_000, False)])
def test_device_plan_equals_host_plan(lsb_built, P, nb, n, skew):
    """The runtime's device planner (k_plan_*) against the host planner."""
    rng = np.random.default_rng(P * 1000 + nb + n)
    here = [lsb_built.here(n, P, r) for r in range(P)]
    hist = _rebalanced_hist(rng, P, nb, n, here, skew)
    for me in range(P):
        h = lsb_built.plan_exchange(n, P, me, hist)
        d = lsb_built.plan_exchange(n, P, me, hist, device=0)
        for k in ("send_counts", "send_displs", "recv_counts", "recv_displs"):
            assert np.array_equal(h[k], d[k]), (me, k)
        # offsets matter only where a piece of (s, b) lands in my range
        gstart = np.concatenate([[0], np.cumsum(hist.sum(0))[:-1]])[None, :] + \
            np.concatenate([np.zeros((1, nb), np.int64), np.cumsum(hist, 0)[:-1]])
        per = -(-n // P) if n else 0
        lo, hi = me * per, me * per + here[me]
        live = (np.minimum(gstart + hist, hi) - np.maximum(gstart, lo)) > 0
        assert np.array_equal(h["place_off"][live], d["place_off"][live])


# ------------------------------------------------------------ larger sizes
@pytest.mark.parametrize("n,P", [(1 << 27, 1), ((1 << 26) + 12345, 2)])
def test_large_verify_on_device(lsb_built, n, P):
    with lsb_built.World(n, ranks=P) as w:
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        assert w.check_sorted()


@pytest.mark.parametrize("split", [0, 1, 2])
@pytest.mark.parametrize("n,P,bits", [((1 << 27) + 333, 1, 8), ((1 << 26) + 12345, 2, 16)])
def test_large_zipf_verify_on_device(lsb_built, n, P, bits, split):
    """Zipf keys at scale through every stage form (auto picks the split
    stage for them), at P = 1 and through the per-digit exchange."""
    with lsb_built.World(n, ranks=P, radix_bits=bits) as w:
        w.set_option(lsb_built.OPT_ONESWEEP_SPLIT, split)
        w.generate("zipf", 1.1)
        w.my_sort()
        assert w.verify() == (True, -1)
        assert w.check_sorted()


def test_beyond_32bit_indices(lsb_built):
    """2^32 + 12345 records on one rank (137 GB of A + B): every index,
    chunk offset and bucket start must be 64-bit (the reference's int MPI
    counts cap a rank below 2^31 records, mpi/mpi_lsbsort.cpp:257-325)."""
    n = (1 << 32) + 12345
    with lsb_built.World(n, ranks=1) as w:
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        tail = w.copy_out(0, n - 4, 4)
        assert np.all(np.diff(tail["key"].astype(np.float64)) >= 0)


# ------------------------------------------------------------- the harness
@pytest.mark.parametrize("corrupt", [False, True])
def test_harness_shmem_lines(lsb_built, ref_vectors, corrupt):
    """--shmem: the lines and exit status of shmem/shmem_lsbsort.cpp's main
    (:474-584): its banner (:498), verify on by default (:479), printed
    elements tagged with their rank (:149-177), checkSorted alone (:568-578)
    and exit status !sorted (:583).  The SHMEM program itself cannot be built
    here (no OpenSHMEM), so its print vectors are the MPI program's (same
    input, same sorted output, same element format, :36-41) with the tag."""
    case = next(c for c in ref_vectors["cases"] if c["n"] == 1000003 and c["P"] == 4)
    args = [lsb_built.HARNESS_PATH, "--n", "1000003", "--ranks", "4", "--print", "--shmem"]
    if corrupt:
        args += ["--test-corrupt", "400000"]  # a small key in rank 1's sorted middle
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    lines = r.stdout.splitlines()
    assert lines[0] == "Total number of shmem PEs: 4" and lines[1] == "Problem size: 1000003"
    assert "Verifying" not in lines
    per = 250001
    printed = [l for l in lines if l.startswith("A[")]
    assert printed == [f"A[{i}] = ({k},{v}) (rank {i // per})" for i, k, v in case["input"] + case["output"]]
    if corrupt:
        assert "Array is NOT sorted" in lines and r.returncode == 1
    else:
        assert "Array is sorted" in lines and r.returncode == 0


@pytest.mark.parametrize("extra", [[], ["--exchange", "peer"], ["--slices", "3", "--radix-bits", "16"],
                                   ["--radix-bits", "64"], ["--radix-bits", "64", "--hybrid", "1"],
                                   ["--radix-bits", "64", "--hybrid", "2"]])
def test_harness_matches_reference_lines(lsb_built, ref_vectors, extra):
    case = next(c for c in ref_vectors["cases"] if c["n"] == 1000003 and c["P"] == 4)
    exe = lsb_built.HARNESS_PATH
    out = subprocess.run([exe, "--n", "1000003", "--ranks", "4", "--print"] + extra, check=True,
                         capture_output=True, text=True, timeout=300).stdout
    lines = out.splitlines()
    assert lines[0] == "Total number of MPI ranks: 4"
    assert lines[1] == "Problem size: 1000003"
    assert "Verifying" in lines and "Array is sorted" in lines
    assert any(l.startswith("That's ") and l.endswith(" M elements sorted / s") for l in lines)
    printed = [l for l in lines if l.startswith("A[")]
    expect = [f"A[{i}] = ({k},{v})" for i, k, v in case["input"] + case["output"]]
    assert printed == expect


@pytest.mark.parametrize("extra", [[], ["--hybrid", "1"], ["--hybrid", "2"]])
def test_harness_one_gpu_process(lsb_built, extra):
    exe = lsb_built.HARNESS_PATH
    r = subprocess.run([exe, "--n", "300000", "--gpus", "1", "--verify", "--json"] + extra,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Array is sorted" in r.stdout


def test_harness_rejects_bad_hybrid(lsb_built):
    r = subprocess.run([lsb_built.HARNESS_PATH, "--n", "10", "--hybrid", "3"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 2


# ------------------------------------------------ 16-bit digits (config C5)
@pytest.mark.parametrize("row", range(5))
def test_radix16_golden_digests(lsb_built, oracle_mod, digests, row):
    """The reference's own radix (RADIX 16): 4 passes, 65536-bucket exchange."""
    d = digests["rows"][row]
    with lsb_built.World(d["n"], ranks=d["P"], radix_bits=16) as w:
        w.generate()
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == d["output"]
        assert w.verify() == (True, -1)


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "zipf", "small_range"])
@pytest.mark.parametrize("P", [1, 3, 8])
def test_radix16_distributions(lsb_built, oracle_mod, name, P):
    rng = np.random.default_rng(hash((name, P, 16)) & 0xFFFF)
    a = _dist(name, 120_007, rng)
    w = lsb_built.World(a.size, ranks=P, radix_bits=16)
    w.scatter_global(a)
    w.my_sort()
    assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))
    w.close()


def test_radix16_single_pass(lsb_built, oracle_mod):
    rng = np.random.default_rng(16)
    n = 70_001
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    with lsb_built.World(n, ranks=1, radix_bits=16) as w:
        w.copy_in(0, a)
        cur = a
        for d in (0, 2):
            w.global_shuffle(d)
            cur, _ = oracle_mod.local_pass(cur, 16, d)
            assert np.array_equal(w.copy_out(0), cur)


def test_radix16_forced_exchange_and_rccl(lsb_built, oracle_mod, digests):
    d = next(r for r in digests["rows"] if r["P"] == 1)
    with lsb_built.World(d["n"], ranks=1, radix_bits=16) as w:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == d["output"]
    w = lsb_built.World.rank(d["n"], 1, 0, 0, lsb_built.get_unique_id(), radix_bits=16)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()
        w.barrier()
        assert oracle_mod.digest(w.copy_out(0)) == d["output"]
    finally:
        w.close()


# ------------------------------------------------------ Zipf keys (config C4)
@pytest.mark.parametrize("P,bits", [(1, 8), (4, 8), (4, 16), (8, 16)])
def test_zipf_input_sorts_bit_exact(lsb_built, oracle_mod, P, bits):
    n = 1_000_003
    with lsb_built.World(n, ranks=P, radix_bits=bits) as w:
        w.generate("zipf", 1.1)
        inp = w.gather_global()
        assert np.array_equal(inp["val"], np.arange(n, dtype=np.uint64))
        # heavily skewed: many duplicates, one dominant key (~9% at s = 1.1)
        uniq, counts = np.unique(inp["key"], return_counts=True)
        assert uniq.size < n // 2 and counts.max() > n // 20
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(inp))
        assert w.verify() == (True, -1)
        assert w.check_sorted()


def test_zipf_verify_uses_zipf_keys(lsb_built):
    n = 50_000
    with lsb_built.World(n, ranks=2) as w:
        w.generate("zipf", 1.3)
        w.my_sort()
        assert w.verify() == (True, -1)
        w.generate()  # uniform again: verify must recompute uniform keys
        w.my_sort()
        assert w.verify() == (True, -1)


@pytest.mark.parametrize("mode", [["--ranks", "3"], ["--gpus", "1"], ["--gpus", "2", "--share-gpus", "1"],
                                  ["--gpus", "3", "--share-gpus", "1"]])
def test_harness_reports_every_mismatch(lsb_built, oracle_mod, mode):
    """A failed verify prints every bad index with Expected/Got, as the
    reference does (mpi/mpi_lsbsort.cpp:729-737), and exits like its failed
    assert (134).  With --gpus P the bad record sits on the last rank, whose
    process streams its records to the root (the reference's gather to rank 0,
    :715-719); only the root regenerates and sorts the input."""
    n, bad = 5000, 3766
    exe = lsb_built.HARNESS_PATH
    r = subprocess.run([exe, "--n", str(n), "--verify", "--test-corrupt", str(bad)] + mode,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 134, (r.returncode, r.stderr)
    P = int(mode[1])
    expect = oracle_mod.stable_sort(oracle_mod.generate(n, P))[bad]
    lines = r.stdout.splitlines()
    i = lines.index(f"Sorted element {bad} did not match")
    assert lines[i + 1] == f"Expected: ({int(expect['key']):016x},{int(expect['val'])})"
    assert lines[i + 2] == f"Got:      (0123456789abcdef,{n + 7})"
    assert sum(l.startswith("Sorted element ") for l in lines) == 1
    assert "Array is NOT sorted" in lines or "Array is sorted" in lines


@pytest.mark.parametrize("n,P,extra", [(1000003, 4, []), (1000000, 2, ["--radix-bits", "64"]),
                                       (17, 8, ["--exchange", "p2p"])])
def test_harness_rccl_ranks_share_gpu(lsb_built, ref_vectors, n, P, extra):
    """`hip_lsbsort --gpus P` forks P RCCL ranks itself; --share-gpus 1 puts
    them all on this GPU, each its own RCCL host (socket transport), so the
    harness's multi-process RCCL path prints the reference's own lines."""
    case = next(c for c in ref_vectors["cases"] if c["n"] == n and c["P"] == P)
    r = subprocess.run([lsb_built.HARNESS_PATH, "--n", str(n), "--gpus", str(P), "--share-gpus", "1",
                        "--print", "--verify"] + extra, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    # RCCL prints its own init banner (RCCL / HIP / ROCm versions, ...) to
    # stdout from rank 0 on some setups, before the harness's first line.
    lines = r.stdout.splitlines()
    head = f"Total number of MPI ranks: {P}"
    assert head in lines, r.stdout[:2000]
    lines = lines[lines.index(head):]
    assert lines[1] == f"Problem size: {n}"
    assert "Array is sorted" in lines
    printed = [l for l in lines if l.startswith("A[")]
    assert printed == [f"A[{i}] = ({k},{v})" for i, k, v in case["input"] + case["output"]]


# ------------------------------------- record buffers and the placement probe
@pytest.mark.parametrize("alloc", ["vmm", "malloc"])
def test_record_buffers_and_opt_in_probe(lsb_built, monkeypatch, alloc):
    """Record buffers of >= 1 GiB are built from 1 GiB VMM pieces
    (LSB_RECORD_ALLOC=malloc: hipMalloc) and no placement probe runs by
    default for buffers under 4 GiB (lsb_get_placement: 0 candidates).  LSB_PLACEMENT_CANDIDATES=8
    still picks A and B among 8 candidate buffers by a timed pass, and R
    among 3.  Every form sorts the same (verified on device), the local LSD
    passes, the hybrid (R) and the forced exchange (R)."""
    monkeypatch.delenv("LSB_PLACEMENT_CANDIDATES", raising=False)
    if alloc == "malloc":
        monkeypatch.setenv("LSB_RECORD_ALLOC", "malloc")
    n = (1 << 26) + 4097  # 1 GiB and a tile per buffer: two pieces, the second nearly empty
    with lsb_built.World(n, ranks=1) as w:
        assert w.placement()["candidates"] == 0
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        w.set_option(lsb_built.OPT_HYBRID, 1)
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
    with lsb_built.World(n, ranks=1, radix_bits=16) as w:  # R of the exchange path
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
    monkeypatch.setenv("LSB_PLACEMENT_CANDIDATES", "8")
    with lsb_built.World(n, ranks=1) as w:
        p = w.placement()
        assert p["candidates"] == 8, p
        # mean ms as a destination: the kept two, the first two, the slowest one
        assert 0 < p["chosen_ms"] <= p["worst_ms"] and p["first_pair_ms"] <= p["worst_ms"], p
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        # the third buffer (hybrid) is placed against A and B by reading them:
        # the input in A survives its probe
        w.set_option(lsb_built.OPT_HYBRID, 1)
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
    monkeypatch.setenv("LSB_PLACEMENT_PICK", "worst")  # the experiment hook keeps the slowest pair
    with lsb_built.World(n, ranks=1) as w:
        p = w.placement()
        assert p["candidates"] == 8 and 0 < p["chosen_ms"] <= p["worst_ms"], p
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
    monkeypatch.delenv("LSB_PLACEMENT_PICK")
    # P logical ranks on one device never probe (the advisor's shared-device case)
    with lsb_built.World(4 * n, ranks=4) as w:
        assert all(w.placement(r)["candidates"] == 0 for r in range(4))


def test_default_probe_on_large_buffers(lsb_built, monkeypatch):
    """Buffers of at least 4 GiB (2^28 records) take the placement probe by
    default: 4 candidates of VMM pieces, the pair fastest both ways kept
    (DESIGN.md §4), and the sorts that follow, LSD and hybrid (R placed
    among 3 against B), verify.  LSB_PLACEMENT_CANDIDATES=0 turns it off."""
    monkeypatch.delenv("LSB_PLACEMENT_CANDIDATES", raising=False)
    monkeypatch.delenv("LSB_RECORD_ALLOC", raising=False)
    n = 1 << 28
    with lsb_built.World(n, ranks=1) as w:
        p = w.placement()
        assert p["candidates"] == 4, p
        assert 0 < p["chosen_ms"] <= p["worst_ms"] and p["first_pair_ms"] <= p["worst_ms"], p
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        w.set_option(lsb_built.OPT_HYBRID, 1)
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
    monkeypatch.setenv("LSB_PLACEMENT_CANDIDATES", "0")
    with lsb_built.World(n, ranks=1) as w:
        assert w.placement()["candidates"] == 0


@pytest.mark.parametrize("P,bits,hybrid", [(1, 8, 0), (1, 8, 1), (2, 16, 0), (8, 8, 0), (8, 16, 0), (4, 64, 0)])
def test_small_vmm_pieces_golden(lsb_built, oracle_mod, digests, monkeypatch, P, bits, hybrid):
    """Every record buffer built from 2 MiB VMM pieces (LSB_VMM_CHUNK_MIB=2),
    so the small golden cases run the VMM allocator, with several pieces per
    buffer, through every form: LSD passes, the hybrid, the per-digit and
    whole-key exchanges between logical ranks (device copies between VMM
    buffers)."""
    monkeypatch.setenv("LSB_VMM_CHUNK_MIB", "2")
    row = next(r for r in digests["rows"] if r["P"] == P)
    with lsb_built.World(row["n"], ranks=P, radix_bits=bits) as w:
        w.set_option(lsb_built.OPT_HYBRID, hybrid)
        w.generate()
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == row["output"]
        assert w.verify() == (True, -1)
    with lsb_built.World(1 << 20, ranks=1) as w:  # small buffers: as allocated
        assert w.placement() == {"candidates": 0, "chosen_ms": 0.0, "first_pair_ms": 0.0, "worst_ms": 0.0}


def test_rccl_contexts_after_released_vmm_buffers(lsb_built):
    """Five world-of-one RCCL contexts one after the other in a fresh process
    (2^28 records, 8-bit digits, every record through ncclAllToAllv in one
    slice, the placement probe on): each verifies.  With VMM record buffers
    at addresses of an earlier RCCL context's released ones, records through
    RCCL came back as garbage from the third context on (LSB_RCCL_VMM=1
    restores that for reproduction); later RCCL contexts now take hipMalloc'd
    buffers (lsb_alloc.cpp, "RCCL and VMM address reuse"; the fault is in
    HIP's VMM, reproduced without RCCL by tools/rccl_vmm_reuse.cpp)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LP_QUICK="1")
    env.pop("LSB_RCCL_VMM", None)
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "tools", "r06", "large_call_probe.py"), "28", "8", "1",
                        "5"], capture_output=True, text=True, timeout=280, cwd=root, env=env)
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and len(rows) == 5, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    assert all(r["verified"] for r in rows), rows


def test_rccl_contexts_after_released_vmm_buffers_other_input(lsb_built):
    """As above with other random input in every context (LP_SEED=1: checked
    on the host -- keys with their values, values a permutation, stable
    order), so no context can pass on an earlier context's leftovers in a
    buffer: four contexts, the third and fourth being the ones that failed
    with VMM buffers at reused addresses (DESIGN.md §0,
    profiles/r06/large_call/r06_g28/)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LP_QUICK="1", LP_SEED="1")
    env.pop("LSB_RCCL_VMM", None)
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "tools", "r06", "large_call_probe.py"), "28", "8", "1",
                        "4"], capture_output=True, text=True, timeout=280, cwd=root, env=env)
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and len(rows) == 4, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    assert all(r["seeded"] for r in rows), rows
    assert all(r["verified"] for r in rows), rows
