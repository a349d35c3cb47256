"""Per-digit exchange with single-read local passes (sort_exchange_onesweep).

The per-digit exchange forms (radix_bits 8 / 16, P > 1: the reference's
globalShuffle per digit, mpi/mpi_lsbsort.cpp:481-585) run each local pass as
a k_onesweep.  Only the first byte's sub-array histogram is read (k_subhist,
once per sort); every later one is counted by what writes the records: the
previous local pass, or the exchange's k_place launches.  The high-byte pass
of a 16-bit digit also counts the digit's 65536 bins for the exchange.

Bit-exact against the oracle's stable sort and against the reduce-then-scan
form of the same exchange (LSB_OPT_ONESWEEP = 0) on the same input: P logical
ranks on one GPU (device-copy all-to-all), RCCL at world size 1 with every
record through the collective, and the peer-store exchange (whose placement
counts nothing, so the next pass reads its histogram).
"""
import numpy as np
import pytest

from test_gpu_sort import DT, _dist

pytestmark = pytest.mark.gpu

T = 4096


def _sort(lsbsort, a, P, bits, onesweep, slices=0, peer=0, skip=1, stats=False, split=0):
    with lsbsort.World(a.size, ranks=P, radix_bits=bits) as w:
        w.set_option(lsbsort.OPT_ONESWEEP, onesweep)
        w.set_option(lsbsort.OPT_ONESWEEP_SPLIT, split)
        w.set_option(lsbsort.OPT_SKIP_CONSTANT_DIGITS, skip)
        if slices:
            w.set_option(lsbsort.OPT_EXCHANGE_SLICES, slices)
        if peer:
            w.set_option(lsbsort.OPT_EXCHANGE_PEER, 1)
        w.scatter_global(a)
        w.set_timing(stats)
        w.my_sort()
        out = w.gather_global()
        return out, w.last_sort(), (w.kernel_stats() if stats else None)


def _uniform(n, seed):
    rng = np.random.default_rng(seed)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


@pytest.mark.parametrize("bits", [8, 16])
@pytest.mark.parametrize("n,P", [(1, 2), (17, 8), (2 * T - 1, 2), (16 * T + 3, 2), (8 * T * 3 + 5, 3),
                                 (100_003, 5), (300_001, 8), ((1 << 20) + 777, 4)])
def test_sizes_bit_exact(lsb_built, oracle_mod, n, P, bits):
    a = _uniform(n, n ^ P)
    out, last, _ = _sort(lsb_built, a, P, bits, 1)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    ref, last0, _ = _sort(lsb_built, a, P, bits, 0)
    assert np.array_equal(out, ref)
    if n > 1:  # one record: every digit is constant, and only digit 0 of
        # the reduce-then-scan form runs (its count kernel reads the span)
        assert last[1] == last0[1]  # same exchanges


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "high_bits_only",
                                  "zipf", "sorted", "reverse", "small_range"])
@pytest.mark.parametrize("P,bits", [(2, 16), (3, 8), (8, 16)])
def test_distributions_bit_exact(lsb_built, oracle_mod, name, P, bits):
    """Skewed bytes: a 16-bit digit's low byte constant over many tiles (the
    high-byte pass's running counts), tiles across low-byte boundaries (the
    staged-run walk), hot next-byte slots in the placement's histogram."""
    rng = np.random.default_rng(hash((name, P, bits)) & 0xFFFF)
    a = _dist(name, 150_001, rng)
    for skip in (1, 0):
        out, _, _ = _sort(lsb_built, a, P, bits, 1, skip=skip)
        assert np.array_equal(out, oracle_mod.stable_sort(a)), skip


@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("name", ["uniform", "zipf", "hot_bucket"])
@pytest.mark.parametrize("P,bits", [(2, 16), (3, 8)])
def test_split_stage(lsb_built, oracle_mod, name, P, bits, split):
    """Both k_onesweep stage forms in every rank's local passes (the 16-bit
    digit's high-byte pass, which counts the 65536 digits, keeps the whole
    stage)."""
    n = 200_003
    if name == "uniform":
        a = _uniform(n, 99 + split)
    else:
        a = _dist(name, n, np.random.default_rng(hash((name, P, split)) & 0xFFFF))
    out, _, _ = _sort(lsb_built, a, P, bits, 1, split=split)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


@pytest.mark.parametrize("slices", [1, 3, 8])
@pytest.mark.parametrize("P,bits", [(2, 8), (5, 16)])
def test_slices(lsb_built, oracle_mod, slices, P, bits):
    """Every (source, slice) k_place launch adds into one next-byte histogram."""
    a = _uniform(250_007, slices * 31 + P)
    out, _, _ = _sort(lsb_built, a, P, bits, 1, slices=slices)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


def test_low_byte_runs_cross_tiles(lsb_built, oracle_mod):
    """16-bit digits whose low byte takes few values: long single-low-byte
    stretches and many tiles whose runs span two low bytes."""
    n = 40 * T + 77
    rng = np.random.default_rng(5)
    a = np.zeros(n, dtype=DT)
    lo = rng.integers(0, 5, n, dtype=np.uint64)
    hi = rng.integers(0, 256, n, dtype=np.uint64)
    a["key"] = lo | (hi << np.uint64(8)) | (rng.integers(0, 4, n, dtype=np.uint64) << np.uint64(16))
    a["val"] = np.arange(n, dtype=np.uint64)
    for P in (1, 3):
        with lsb_built.World(n, ranks=P, radix_bits=16) as w:
            w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
            w.scatter_global(a)
            w.my_sort()
            assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a)), P


@pytest.mark.parametrize("bits", [8, 16])
def test_one_count_read_per_sort(lsb_built, bits):
    """k_subhist runs once per rank and sort; the local passes are k_onesweep."""
    P, n = 4, 1 << 20
    with lsb_built.World(n, ranks=P, radix_bits=bits) as w:
        w.generate()
        w.set_timing(True)
        w.my_sort()
        st = w.kernel_stats()
        assert w.last_sort()[:2] == (8, 64 // bits)
        assert st["upsweep"][0] == P, st
        assert st["scatter"][0] == 8 * P, st
        assert st["scan"][0] == 0, st
        assert w.scatter_elems() == 8 * n
        assert w.verify() == (True, -1)


def test_peer_exchange_reads_its_histogram(lsb_built, oracle_mod):
    """Peer stores place records without counting them: the pass after each
    exchange reads its histogram (one k_subhist per rank and exchange)."""
    P, n = 3, 200_003
    a = _uniform(n, 99)
    out, last, st = _sort(lsb_built, a, P, 16, 1, peer=1, stats=True)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert st["upsweep"][0] == P * last[1]


@pytest.mark.parametrize("self_coll", [0, 1])
@pytest.mark.parametrize("bits", [8, 16])
def test_rccl_world_of_one(lsb_built, oracle_mod, digests, bits, self_coll):
    """RCCL communicator of one rank with the exchange forced; with
    LSB_OPT_EXCHANGE_SELF every record goes through ncclAllToAllv and is
    placed (and counted) from the receive buffer."""
    d = next(r for r in digests["rows"] if r["P"] == 1)
    uid = lsb_built.get_unique_id()
    w = lsb_built.World.rank(d["n"], 1, 0, 0, uid, radix_bits=bits)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.set_option(lsb_built.OPT_EXCHANGE_SELF, self_coll)
        w.generate()
        w.my_sort()
        w.sync()
        assert oracle_mod.digest(w.copy_out(0)) == d["output"]
        assert w.verify() == (True, -1)
    finally:
        w.close()


def test_golden_digests_loopback(lsb_built, oracle_mod, digests):
    for d in digests["rows"]:
        if d["P"] == 1:
            continue
        for bits in (8, 16):
            with lsb_built.World(d["n"], ranks=d["P"], radix_bits=bits) as w:
                w.set_option(lsb_built.OPT_ONESWEEP, 1)
                w.generate()
                w.my_sort()
                assert oracle_mod.digest(w.gather_global()) == d["output"], (d["n"], d["P"], bits)


@pytest.mark.parametrize("n,P,bits", [(1 << 22, 2, 8), (1 << 22, 3, 16), (3 * T + 11, 2, 16),
                                      ((1 << 21) + 5, 8, 8), (600_011, 5, 16)])
def test_gathered_pass_matches_placed(lsb_built, oracle_mod, n, P, bits):
    """LSB_OPT_EXCHANGE_GATHER (the default): every exchange but the last only
    counts the next byte, and the next pass reads its tiles where the records
    arrived (receive buffer, the rank's own segment in A) through the plan's
    piece table.  Long pieces (8-bit digits: a few per tile, the tile
    descriptors) and short ones (16-bit digits at these sizes: the per-record
    search) both give the placed form's output (LSB_OPT_EXCHANGE_GATHER = 0),
    the oracle's stable sort, and the same k_place launches (count-only or
    placing)."""
    a = _uniform(n, n + P)
    outs, stats = [], []
    for g in (1, 0):
        with lsb_built.World(a.size, ranks=P, radix_bits=bits) as w:
            w.set_option(lsb_built.OPT_EXCHANGE_GATHER, g)
            w.scatter_global(a)
            w.set_timing(True)
            w.my_sort()
            outs.append(w.gather_global())
            stats.append(w.kernel_stats())
    assert np.array_equal(outs[0], oracle_mod.stable_sort(a))
    assert np.array_equal(outs[0], outs[1])
    assert stats[0]["place"][0] == stats[1]["place"][0]
    assert stats[0]["upsweep"][0] == stats[1]["upsweep"][0] == P  # one k_subhist per rank


@pytest.mark.parametrize("split", [0, 2])
def test_skewed_keys_gather(lsb_built, oracle_mod, split):
    """Zipf keys pick the split stage (auto, 0) or have it forced (2); their
    exchanges still only count the arriving records but the last, and the
    gathered passes take the whole stage (round 4):
    lsb_get_exchange_stats shows every record counted at 3 of the 4
    exchanges and placed at the last."""
    P, n = 2, 200_003
    a = _dist("zipf", n, np.random.default_rng(17 + split))
    with lsb_built.World(n, ranks=P, radix_bits=16) as w:
        w.set_option(lsb_built.OPT_ONESWEEP_SPLIT, split)
        w.scatter_global(a)
        w.reset_kernel_stats()
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))
        ex = w.last_sort()[1]
        x = w.exchange_stats()
        assert ex >= 2 and x["exchanges"] == ex
        assert x["placed_records"] == n and x["counted_records"] == n * (ex - 1), x
