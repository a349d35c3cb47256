"""Hybrid local sort (LSB_OPT_HYBRID): k stable k_onesweep passes on the
most significant varying bytes; every segment (run of records equal on
those bytes) is then ordered by the whole key: by the last pass itself,
inside each tile, plus k_segfix for the segments split between tiles
(mode 1, the default), or by a separate k_segsort pass (mode 2, and the
fallback of mode 1 when a run crossing a tile is too long).

The output must be the reference's: the stable sort by key
(mpi/mpi_lsbsort.cpp:580-585 produces it by LSD passes; the verify at
:722-737 checks exactly that), bit for bit against the oracle.  Sizes straddle
k_segsort's 4096-record tiles and the choice of k; distributions include the
skewed ones that take the LSD passes directly, and keys whose segments run
past the segment sorts' kSegMax (64 records), where the sort must redo the
kept input with the LSD passes (without trusting the fused pass's output).
"""
import numpy as np
import pytest

from test_gpu_sort import DT, _dist

pytestmark = pytest.mark.gpu

T = 4096


def _sort(lsbsort, a, skip=1, split=0, timing=False, mode=1):
    with lsbsort.World(a.size, ranks=1) as w:
        w.set_option(lsbsort.OPT_HYBRID, mode)
        w.set_option(lsbsort.OPT_SKIP_CONSTANT_DIGITS, skip)
        w.set_option(lsbsort.OPT_ONESWEEP_SPLIT, split)
        w.set_timing(timing)
        w.copy_in(0, a)
        w.my_sort()
        w.sync()
        return w.copy_out(0), w.last_sort(), (w.pass_stats() if timing else None)


def _uniform(n, seed):
    rng = np.random.default_rng(seed)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


@pytest.mark.parametrize("n", [1, 2, 100, 128, 129, 1000, T - 1, T, T + 1, 2 * T + 3, 10_000, 65_537,
                               1 << 20, (1 << 20) + 12_345, 1 << 22])
@pytest.mark.parametrize("mode", [1, 2])
def test_sizes_bit_exact(lsb_built, oracle_mod, n, mode):
    a = _uniform(n, n)
    out, (lp, ex, _), _ = _sort(lsb_built, a, mode=mode)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    # k MSD passes + one segmented sort: fewer passes than the 8 LSD ones
    # (tiny blocks look skewed to the 1/32 rule and take the LSD passes)
    assert ex == 0 and (lp <= 5 or n < 1000), lp


@pytest.mark.parametrize("n,k", [(256, 1), (257, 2), (1000, 2), (1 << 16, 2), (1 << 22, 3),
                                 ((1 << 24) + 1, 4)])
@pytest.mark.parametrize("mode", [1, 2])
def test_msd_byte_count(lsb_built, oracle_mod, n, k, mode):
    """k = the fewest top bytes whose varying bits reach ceil(log2 n);
    the per-pass stats show the k byte passes (top bytes, least significant
    first) and, in mode 2, the segmented sort (shift 64)."""
    a = _uniform(n, 7 * n)
    out, (lp, _, _), rows = _sort(lsb_built, a, timing=True, mode=mode)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    seg = [64] if mode == 2 else []
    assert lp == k + len(seg)
    assert [r["shift"] for r in rows] == [8 * (8 - k + i) for i in range(k)] + seg
    assert all(r["elems"] == n for r in rows)


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "high_bits_only",
                                  "zipf", "sorted", "reverse", "small_range"])
@pytest.mark.parametrize("n", [200_003, 1 << 21])
@pytest.mark.parametrize("mode", [1, 2])
def test_distributions_bit_exact(lsb_built, oracle_mod, name, n, mode):
    rng = np.random.default_rng(hash((name, n)) & 0xFFFF)
    a = _dist(name, n, rng)
    out, _, _ = _sort(lsb_built, a, mode=mode)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


@pytest.mark.parametrize("split", [1, 2])
def test_stage_split_forced(lsb_built, oracle_mod, split):
    a = _uniform(300_001, split)
    out, _, _ = _sort(lsb_built, a, split=split)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


def test_skip_constant_digits_off(lsb_built, oracle_mod):
    a = _uniform(500_009, 3)
    out, (lp, _, _), _ = _sort(lsb_built, a, skip=0)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert lp == 3  # 3 top bytes (guessed from n alone); the last one orders the segments


@pytest.mark.parametrize("mode", [1, 2])
def test_duplicate_keys_keep_input_order(lsb_built, oracle_mod, mode):
    """Equal keys share a segment, also across tiles (k_segfix keeps tile
    t's records first); they are ranked by input position."""
    rng = np.random.default_rng(11)
    n = 1 << 20
    a = np.zeros(n, dtype=DT)
    pool = rng.integers(0, 2**64 - 1, n // 8, dtype=np.uint64)
    a["key"] = pool[rng.integers(0, pool.size, n)]
    a["val"] = np.arange(n, dtype=np.uint64)
    out, _, _ = _sort(lsb_built, a, mode=mode)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


def test_long_runs_take_the_segment_sort(lsb_built, oracle_mod):
    """Runs of records equal on all but the last pass's byte hold ~2048
    records, past the kSegCap slots a tile reports for k_segfix: the fused
    pass flags it and a k_segsort pass orders the (small) segments."""
    rng = np.random.default_rng(5)
    n = 1 << 22
    mid = rng.integers(0, 1 << 16, 2048, dtype=np.uint64)  # bytes 5-6: 2048 values
    a = np.zeros(n, dtype=DT)
    a["key"] = ((rng.integers(0, 256, n, dtype=np.uint64) << np.uint64(56)) |
                (mid[rng.integers(0, mid.size, n)] << np.uint64(40)) |
                rng.integers(0, 1 << 40, n, dtype=np.uint64))
    a["val"] = np.arange(n, dtype=np.uint64)
    out, (lp, _, _), _ = _sort(lsb_built, a)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert lp == 3 + 1  # 3 byte passes + the segmented sort


@pytest.mark.parametrize("n", [1 << 23, (1 << 23) + 4_097])
def test_long_runs_take_the_large_segfix(lsb_built, oracle_mod, n):
    """2^23 records over 3 top bytes: runs of ~128 records per value of the
    two run bytes, so launch_segfix takes its 1024-record form; no k_segsort
    pass, output exact."""
    a = _uniform(n, 23)
    out, (lp, _, _), rows = _sort(lsb_built, a, timing=True)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert lp == 3 and [r["shift"] for r in rows] == [40, 48, 56]


@pytest.mark.parametrize("mids,run", [(28_000, 150), (20_000, 210)])
def test_crossing_runs_past_one_window(lsb_built, oracle_mod, mids, run):
    """Runs of ~150-210 records (equal on the two bytes below the top one):
    k_segfix's 64-record windows do not hold the crossing run, so it scans on
    (still under kSegCap): no k_segsort pass, output exact."""
    rng = np.random.default_rng(mids)
    n = 1 << 22
    mid = rng.choice(1 << 16, mids, replace=False).astype(np.uint64)
    a = np.zeros(n, dtype=DT)
    a["key"] = ((rng.integers(0, 256, n, dtype=np.uint64) << np.uint64(56)) |
                (mid[rng.integers(0, mid.size, n)] << np.uint64(40)) |
                rng.integers(0, 1 << 40, n, dtype=np.uint64))
    a["val"] = np.arange(n, dtype=np.uint64)
    assert abs(n / np.unique(a["key"] >> np.uint64(40) & np.uint64(0xFFFF)).size - run) < run / 5
    out, (lp, _, _), _ = _sort(lsb_built, a)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert lp == 3  # 3 byte passes, segments merged by k_segfix


@pytest.mark.parametrize("bases", [1024, 4096, 1 << 15])
def test_long_segments_fall_back_to_lsd(lsb_built, oracle_mod, bases):
    """n / bases records share each of `bases` random top parts: the first
    byte looks uniform (no skew), but segments hold ~128-4096 records, past
    the segment sorts' limit (kSegMax = 64), so the sort redoes the kept input
    by the LSD passes."""
    rng = np.random.default_rng(bases)
    n = 1 << 22
    top = rng.integers(0, 2**64 - 1, bases, dtype=np.uint64) & np.uint64(0xFFFFFFFFFF000000)
    a = np.zeros(n, dtype=DT)
    a["key"] = top[rng.integers(0, bases, n)] | rng.integers(0, 1 << 24, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    out, (lp, _, _), _ = _sort(lsb_built, a)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    # 3 byte passes, then (the fused pass found a segment past kSegMax inside
    # a tile: its output is no permutation) straight to the 8 LSD passes
    assert lp == 3 + 8
    out, (lp, _, _), _ = _sort(lsb_built, a, mode=2)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert lp == 3 + 1 + 8  # mode 2: the byte passes, the failed k_segsort, the LSD passes


def _stress_seed19_iter3258(n):
    """The input that made `tools/stress_mix.py --seed 19 --max-log2 29` fail
    at iteration 3258 (P = 2, whole key, hybrid 1; its rank 0 block alone
    fails the same way at P = 1), rebuilt from the draws its thinned_keys
    made (`tools/stress_replay.py`): uniform bytes 0-2 and 4, bytes 3 and 5
    constant, bytes 6 and 7 each from a pool of two values."""
    g = np.random.default_rng(10821365)
    full = 693_391
    k = g.integers(0, 2**64 - 1, full, dtype=np.uint64)
    for b, c in ((3, 174), (5, 227)):
        sh = np.uint64(8 * b)
        k = (k & ~(np.uint64(0xFF) << sh)) | (np.uint64(c) << sh)
    for b in (6, 7):
        sh = np.uint64(8 * b)
        pool = g.integers(0, 256, 2, dtype=np.uint64)
        k = (k & ~(np.uint64(0xFF) << sh)) | (pool[g.integers(0, pool.size, full)] << sh)
    a = np.zeros(full, dtype=DT)
    a["key"] = k
    a["val"] = np.arange(full, dtype=np.uint64)
    return a[:n].copy()


def test_fused_pass_with_long_segments_stress_seed19(lsb_built, oracle_mod):
    """Round 5's stress found it: the fused pass (mode 1) over
    segments of ~340 records computed their slots from walks cut at kSegMax,
    so records collided and stale ones filled the holes; k_segsort, run on
    that output, found the long segments cut short by the stale records and
    kept a wrong result.  Now such a pass sends the sort straight to the LSD
    passes over the kept input: 3 byte passes + 6 (bytes 3 and 5 constant)."""
    a = _stress_seed19_iter3258(346_696)
    out, (lp, _, _), _ = _sort(lsb_built, a)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert lp == 3 + 6


def test_constant_top_byte_takes_lsd(lsb_built, oracle_mod):
    """Digit skipping off: the hybrid guesses the top bytes of full 64-bit
    keys; keys below 2^32 make the first of them constant, and the sort takes
    the LSD passes at once (8 passes, no segment sort; advisor r03)."""
    a = _uniform(300_007, 5)
    a["key"] &= np.uint64(0xFFFFFFFF)
    out, (lp, _, _), _ = _sort(lsb_built, a, skip=0)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert lp == 8


def test_generated_input_verifies(lsb_built, digests, oracle_mod):
    for row in digests["rows"]:
        if row["P"] != 1:
            continue
        with lsb_built.World(row["n"], ranks=1) as w:
            w.set_option(lsb_built.OPT_HYBRID, 1)
            w.generate()
            w.my_sort()
            assert oracle_mod.digest(w.copy_out(0)) == row["output"]
            assert w.verify() == (True, -1)


def test_repeated_sorts_on_one_context(lsb_built, oracle_mod):
    """The hybrid rotates three buffers; the look-back status rows are
    shared with the LSD passes of the same context."""
    n = 300_007
    with lsb_built.World(n, ranks=1) as w:
        for i in range(6):
            w.set_option(lsb_built.OPT_HYBRID, i % 3)
            a = _uniform(n, 100 + i)
            w.copy_in(0, a)
            w.my_sort()
            assert np.array_equal(w.copy_out(0), oracle_mod.stable_sort(a))


@pytest.mark.parametrize("P", [2, 4, 8])
def test_whole_key_local_sorts(lsb_built, oracle_mod, digests, P):
    """Each rank's local sort of the whole-key exchange (radix_bits = 64)."""
    for row in digests["rows"]:
        if row["P"] != P:
            continue
        with lsb_built.World(row["n"], ranks=P, radix_bits=64) as w:
            w.set_option(lsb_built.OPT_HYBRID, 1)
            w.generate()
            w.my_sort()
            assert oracle_mod.digest(w.gather_global()) == row["output"]


def test_option_range(lsb_built):
    with lsb_built.World(10, ranks=1) as w:
        with pytest.raises(lsb_built.LsbError):
            w.set_option(lsb_built.OPT_HYBRID, 3)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("fail_at", [1, 2, 3])
def test_failed_launch_mid_hybrid_keeps_the_context(lsb_built, oracle_mod, mode, fail_at):
    """A k_onesweep launch that fails inside the hybrid (LSB_OPT_FAIL_ONESWEEP
    injects it: 300,007 records take k = 3 byte passes) returns the error and
    leaves the context whole (advisor r03): A again holds the input, A, B and
    R are three distinct buffers, so the next sort on the same context sorts
    that input exactly, later sorts too, and the context closes cleanly."""
    n = 300_007
    with lsb_built.World(n, ranks=1) as w:
        w.set_option(lsb_built.OPT_HYBRID, mode)
        w.generate()
        inp = w.gather_global()
        w.set_option(lsb_built.OPT_FAIL_ONESWEEP, fail_at)
        with pytest.raises(lsb_built.LsbError, match="injected"):
            w.my_sort()
        assert np.array_equal(w.gather_global(), inp)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(inp))
        assert w.verify() == (True, -1)
        for _ in range(2):  # the buffers keep rotating without aliasing
            w.generate()
            w.my_sort()
            assert w.verify() == (True, -1)


@pytest.mark.parametrize("fail_at", [2, 4])
def test_failed_launch_in_phased_local_sorts(lsb_built, oracle_mod, fail_at):
    """The whole-key exchange's local sorts run step by step across a loopback
    context's ranks (sort_local_ranks).  A launch that fails in rank 0's
    passes (2) or rank 1's (4: each rank's 150,004 records take k = 3 byte
    passes, queued rank after rank) leaves every rank's input in A, and the
    next sort on the context is exact."""
    n = 300_007
    with lsb_built.World(n, ranks=2, radix_bits=64) as w:
        w.set_option(lsb_built.OPT_HYBRID, 1)
        w.generate()
        inp = w.gather_global()
        w.set_option(lsb_built.OPT_FAIL_ONESWEEP, fail_at)
        with pytest.raises(lsb_built.LsbError, match="injected"):
            w.my_sort()
        assert np.array_equal(w.gather_global(), inp)
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(inp))
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
