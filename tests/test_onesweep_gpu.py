"""Single-read passes (k_subhist + k_onesweep, LSB_OPT_ONESWEEP, P == 1).

Bit-exact against the oracle's stable sort and against the reduce-then-scan
path of the same library (LSB_OPT_ONESWEEP = 0) on the same inputs.  Sizes
straddle the structure the kernel relies on: 4096-record tiles, 8
sub-arrays of floor(x * tiles / 8) tiles (empty sub-arrays below 8 tiles,
one-tile sub-arrays below 16), a partial last tile, runs that cross a
sub-array boundary, and the work-stealing tail.
"""
import numpy as np
import pytest

from test_gpu_sort import DT, _dist

pytestmark = pytest.mark.gpu

T = 4096


def _sort(lsbsort, a, onesweep, skip=1, split=0):
    with lsbsort.World(a.size, ranks=1) as w:
        w.set_option(lsbsort.OPT_ONESWEEP, onesweep)
        w.set_option(lsbsort.OPT_SKIP_CONSTANT_DIGITS, skip)
        w.set_option(lsbsort.OPT_ONESWEEP_SPLIT, split)
        w.copy_in(0, a)
        w.my_sort()
        w.sync()
        return w.copy_out(0), w.last_sort()


def _uniform(n, seed):
    rng = np.random.default_rng(seed)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


@pytest.mark.parametrize("n", [1, 2, 63, T - 1, T, T + 1, 3 * T + 5, 8 * T - 1, 8 * T, 8 * T + 1,
                               9 * T + 5, 15 * T + 1, 16 * T, 17 * T + 4095, 100_003,
                               (1 << 20) + 777])
def test_sizes_bit_exact(lsb_built, oracle_mod, n):
    a = _uniform(n, n)
    out, last = _sort(lsb_built, a, 1)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    ref, last0 = _sort(lsb_built, a, 0)
    assert np.array_equal(out, ref)
    # reduce-then-scan always runs digit 0 (its count kernel reads the span);
    # single-read passes skip it too when it is constant (n = 1: every digit)
    assert last == last0 or (n == 1 and last == (0, 0, 0) and last0 == (1, 0, 0))


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "high_bits_only",
                                  "zipf", "sorted", "reverse", "small_range"])
@pytest.mark.parametrize("n", [50_001, (1 << 21) + 3])
def test_distributions_bit_exact(lsb_built, oracle_mod, name, n):
    """Skewed digits: runs of one bucket span many tiles and sub-arrays."""
    rng = np.random.default_rng(hash((name, n)) & 0xFFFF)
    a = _dist(name, n, rng)
    for skip in (1, 0):
        out, _ = _sort(lsb_built, a, 1, skip)
        assert np.array_equal(out, oracle_mod.stable_sort(a)), skip


@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("n", [1, T // 2 - 1, T // 2, T // 2 + 1, T + T // 2, 8 * T + 1,
                               17 * T + 2049, 100_003])
def test_split_stage_sizes(lsb_built, oracle_mod, n, split):
    """LSB_OPT_ONESWEEP_SPLIT forced: the tile staged whole (1) or in two
    halves of its output order (2, 3 workgroups per CU), around half-tile
    boundaries and partial tiles."""
    a = _uniform(n, 7 * n + split)
    out, _ = _sort(lsb_built, a, 1, split=split)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


@pytest.mark.parametrize("split", [1, 2])
@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "zipf", "sorted",
                                  "reverse"])
def test_split_stage_distributions(lsb_built, oracle_mod, name, split):
    """Skewed keys through both stage forms (auto picks the split one for
    them); runs of one bucket cross the half-stage boundary."""
    n = 300_001
    rng = np.random.default_rng(hash((name, split)) & 0xFFFF)
    a = _dist(name, n, rng)
    out, _ = _sort(lsb_built, a, 1, split=split)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


def test_split_option_rejected(lsb_built):
    with lsb_built.World(1000, ranks=1) as w:
        with pytest.raises(lsb_built.LsbError):
            w.set_option(lsb_built.OPT_ONESWEEP_SPLIT, 3)


def test_one_bucket_per_subarray(lsb_built, oracle_mod):
    """Digit 0 = sub-array index, digit 1 = reversed: every run of the second
    pass is a whole sub-array crossing into the next one."""
    n = 64 * T + 123
    a = np.zeros(n, dtype=DT)
    i = np.arange(n, dtype=np.uint64)
    a["key"] = (i * np.uint64(8) // np.uint64(n)) | ((np.uint64(255) - i % np.uint64(7)) << np.uint64(8))
    a["val"] = i
    out, last = _sort(lsb_built, a, 1)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert last[0] == 2


def test_repeated_sorts_reuse_status(lsb_built, oracle_mod):
    """Status words are never cleared: each launch's epoch tells stale from fresh."""
    n = 300_007
    with lsb_built.World(n, ranks=1) as w:
        for seed in range(4):
            a = _uniform(n, 1000 + seed)
            if seed == 2:
                a["key"] &= np.uint64(0x00FF00FF00FF00FF)  # 4 of 8 passes
            w.copy_in(0, a)
            w.my_sort()
            w.sync()
            assert np.array_equal(w.copy_out(0), oracle_mod.stable_sort(a)), seed


def test_generated_input_verifies(lsb_built, digests, oracle_mod):
    for row in digests["rows"]:
        if row["P"] != 1:
            continue
        with lsb_built.World(row["n"], ranks=1) as w:
            w.generate()
            w.my_sort()
            assert oracle_mod.digest(w.gather_global()) == row["output"]
            assert w.verify() == (True, -1)
