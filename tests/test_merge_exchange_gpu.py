"""Whole-key exchange (radix_bits = 64): local sort, one all-to-all, merge.

Same bar as every other exchange form: bit-exact against the reference's
golden digests (`mpirun -n P mpi_lsbsort`) and against the oracle's stable
sort on adversarial keys.  Multi-rank cases run P logical ranks on one GPU
(lsb_create): the splitter search, plan and merge tree are the per-rank
code of the RCCL contexts; the all-gathers and the all-to-all are device
copies.  The multi-process form (gloo collectives, one process per rank) is
in test_dist_ops_gpu.py.
"""
import numpy as np
import pytest

from test_gpu_sort import DT, _dist

pytestmark = pytest.mark.gpu


def _sort(lsbsort, a, P, **opts):
    with lsbsort.World(a.size, ranks=P, radix_bits=64) as w:
        for k, v in opts.items():
            w.set_option(getattr(lsbsort, k), v)
        w.scatter_global(a)
        w.my_sort()
        out = w.gather_global()
        meta = w.last_sort()
        sorted_ = w.check_sorted()
    return out, meta, sorted_


@pytest.mark.parametrize("row", range(5))
def test_golden_digests(lsb_built, oracle_mod, digests, row):
    d = digests["rows"][row]
    with lsb_built.World(d["n"], ranks=d["P"], radix_bits=64) as w:
        w.generate()
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == d["output"]
        assert w.verify() == (True, -1)
        assert w.check_sorted()
        passes, exchanges = w.last_sort()[:2]
        assert passes == 8 and exchanges == (1 if d["P"] > 1 else 0)


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "high_bits_only",
                                  "zipf", "sorted", "reverse", "small_range"])
@pytest.mark.parametrize("P", [2, 3, 8])
def test_distributions_bit_exact(lsb_built, oracle_mod, name, P):
    rng = np.random.default_rng(hash((name, P, 64)) & 0xFFFF)
    a = _dist(name, 200_003, rng)
    out, _, ok = _sort(lsb_built, a, P)
    assert np.array_equal(out, oracle_mod.stable_sort(a)) and ok


@pytest.mark.parametrize("n,P", [(0, 3), (1, 4), (2, 8), (5, 8), (9, 8), (13, 3),
                                 (4095, 2), (4096, 2), (4097, 2), (8193, 2),
                                 (4096 * 3 + 1, 2), (4096 * 64 + 5, 5), (4096 * 513 + 7, 7)])
def test_ragged_and_tiny(lsb_built, oracle_mod, n, P):
    rng = np.random.default_rng(n * 31 + P)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64) & np.uint64(0xF0F0F0F0F0F0F0F0)
    a["val"] = np.arange(n, dtype=np.uint64)
    out, _, _ = _sort(lsb_built, a, P)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


@pytest.mark.parametrize("slices", [1, 3, 16, 64])
@pytest.mark.parametrize("P", [2, 7, 8])
def test_slices(lsb_built, oracle_mod, slices, P):
    """Owner blocks cut into S sub-blocks (default 8), each merged while the next
    is on the wire; P * S beyond kMergeMaxCuts = 512 is capped."""
    rng = np.random.default_rng(slices * 13 + P)
    a = _dist("zipf" if slices % 2 else "hot_bucket", 150_007, rng)
    out, _, ok = _sort(lsb_built, a, P, OPT_EXCHANGE_SLICES=slices)
    assert np.array_equal(out, oracle_mod.stable_sort(a)) and ok


def test_one_source_owns_everything(lsb_built, oracle_mod):
    """Rank 0 holds all the small keys: every other owner receives one run."""
    n, P = 40_000, 4
    a = np.zeros(n, dtype=DT)
    a["key"] = np.arange(n, dtype=np.uint64)[::-1] * np.uint64(3)
    a["val"] = np.arange(n, dtype=np.uint64)
    out, _, ok = _sort(lsb_built, a, P)
    assert np.array_equal(out, oracle_mod.stable_sort(a)) and ok


@pytest.mark.parametrize("P", [2, 5])
def test_reduce_scan_local_sort(lsb_built, oracle_mod, digests, P):
    """The local sort by count + scan + scatter (LSB_OPT_ONESWEEP = 0)."""
    rng = np.random.default_rng(P)
    a = _dist("zipf", 150_001, rng)
    out, meta, _ = _sort(lsb_built, a, P, OPT_ONESWEEP=0)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


@pytest.mark.parametrize("mask,passes", [(0x00000000FFFFFFFF, 4), (0xFF000000000000FF, 2), (0, 0)])
def test_constant_digits_skipped_locally(lsb_built, oracle_mod, mask, passes):
    n, P = 100_003, 3
    rng = np.random.default_rng(mask & 0xFFFF)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64) & np.uint64(mask)
    a["val"] = np.arange(n, dtype=np.uint64)
    out, meta, _ = _sort(lsb_built, a, P)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert meta[0] == passes and meta[1] == 1


def test_global_shuffle_is_the_sort(lsb_built, oracle_mod, digests):
    """globalShuffle of the one 64-bit digit == mySort."""
    d = next(r for r in digests["rows"] if r["P"] == 4)
    with lsb_built.World(d["n"], ranks=4, radix_bits=64) as w:
        w.generate()
        w.global_shuffle(0)
        assert oracle_mod.digest(w.gather_global()) == d["output"]
        with pytest.raises(lsb_built.LsbError):
            w.global_shuffle(1)


def test_forced_exchange_at_p1(lsb_built, oracle_mod, digests):
    d = next(r for r in digests["rows"] if r["P"] == 1)
    with lsb_built.World(d["n"], ranks=1, radix_bits=64) as w:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.my_sort()
        assert oracle_mod.digest(w.gather_global()) == d["output"]
        assert w.last_sort()[:2] == (8, 1)


def test_rccl_world_of_one(lsb_built, oracle_mod, digests):
    d = next(r for r in digests["rows"] if r["P"] == 1)
    w = lsb_built.World.rank(d["n"], 1, 0, 0, lsb_built.get_unique_id(), radix_bits=64)
    try:
        w.set_option(lsb_built.OPT_FORCE_EXCHANGE, 1)
        w.generate()
        w.barrier()
        w.my_sort()
        w.barrier()
        assert oracle_mod.digest(w.copy_out(0)) == d["output"]
        assert w.verify() == (True, -1)
    finally:
        w.close()


def test_repeated_sorts_on_one_context(lsb_built, oracle_mod, digests):
    d = next(r for r in digests["rows"] if r["P"] == 8 and r["n"] < 2_000_000)
    with lsb_built.World(d["n"], ranks=8, radix_bits=64) as w:
        for _ in range(3):
            w.generate()
            w.my_sort()
            assert oracle_mod.digest(w.gather_global()) == d["output"]


@pytest.mark.parametrize("n,P", [((1 << 26) + 12345, 4), ((1 << 25) + 3, 3)])
def test_large_verify_on_device(lsb_built, n, P):
    """Merge tree over runs of millions of records, checked by lsb_verify."""
    with lsb_built.World(n, ranks=P, radix_bits=64) as w:
        w.generate()
        w.my_sort()
        assert w.verify() == (True, -1)
        assert w.check_sorted()


def test_large_zipf(lsb_built):
    n, P = (1 << 24) + 77, 8
    with lsb_built.World(n, ranks=P, radix_bits=64) as w:
        w.generate("zipf", 1.1)
        w.my_sort()
        assert w.verify() == (True, -1)
