"""CPU model of the hybrid local sort's mode 1 (LSB_OPT_HYBRID = 1), at small
tile sizes so that every boundary case shows up in a few thousand records.

It restates the data flow of distributed-lsb_amd/csrc (k_onesweep with SEG,
then k_segfix) with numpy and checks it against the stable sort by key, the
reference's output (mpi/mpi_lsbsort.cpp:580-585, verified at :722-737):

  1. stable passes on the k top bytes but the last;
  2. the last pass, tile by tile: each tile's bucket-d block goes to the
     bucket's next slots (the look-back), and inside the block every segment
     (records equal on the k bytes) is ordered by the whole key;
  3. k_segfix, per tile boundary b: the run of records equal on the k - 1
     run bytes that crosses b is found in the last pass's input as
     [b - a, b + c); for every bucket present on both sides, its records are
     re-placed, stably, at P - (left count) + rank, where P is the end of
     tile t's bucket block (look-back value + bucket base);
  4. a run longer than the cap on one side, or one spanning a whole tile,
     is reported (the runtime then runs k_segsort).

The GPU tests (tests/test_hybrid_gpu.py) check the kernels; this checks the
algorithm they implement, including the cases the GPU sizes rarely reach.
"""
import numpy as np
import pytest

DT = np.dtype([("key", "<u8"), ("val", "<u8")])


def _byte(keys, b):
    return ((keys >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.int64)


def hybrid_model(a, msd, T, cap):
    """Mode 1 of the hybrid on records a (msd: the top bytes, least
    significant first).  Returns (output, ok); ok False = k_segfix's error."""
    x = a
    for b in msd[:-1]:
        x = x[np.argsort(_byte(x["key"], b), kind="stable")]
    last = msd[-1]
    pmask = np.uint64(sum(0xFF << (8 * b) for b in msd))
    rmask = pmask & ~np.uint64(0xFF << (8 * last))
    m = x.size
    d = _byte(x["key"], last)
    # The plain last pass: slot of each input record (stable by digit).
    order = np.argsort(d, kind="stable")
    slot = np.empty(m, dtype=np.int64)
    slot[order] = np.arange(m)
    out = np.empty_like(x)
    # SEG: inside each tile's bucket block, segments ordered by the key.
    for t0 in range(0, m, T):
        idx = np.arange(t0, min(t0 + T, m))
        for dd in np.unique(d[idx]):
            blk = idx[d[idx] == dd]  # input order = the block's slot order
            s = slot[blk]
            seg = x["key"][blk] & pmask
            # stable by (segment, key): segments stay where they are, since
            # the block is already ordered by its segment (run key sorted)
            o = np.lexsort((x["key"][blk], seg))
            out[s] = x[blk[o]]
    # k_segfix
    ok = True
    rk = x["key"] & rmask
    for b in range(T, m, T):
        lo, hi = b - T, min(b + T, m)
        v = rk[b - 1]
        if rk[b] != v:
            continue
        a_ = 0
        while b - 1 - a_ >= lo and rk[b - 1 - a_] == v:
            a_ += 1
        c_ = 0
        while b + c_ < hi and rk[b + c_] == v:
            c_ += 1
        if a_ > cap or c_ > cap or (b - a_ == lo and lo > 0 and rk[lo - 1] == v) or \
                (b + c_ == hi and hi < m and rk[hi] == v):
            ok = False
            continue
        run = np.arange(b - a_, b + c_)
        left = run < b
        for dd in np.unique(d[run]):
            L, R = run[left & (d[run] == dd)], run[~left & (d[run] == dd)]
            if L.size == 0 or R.size == 0:
                continue
            # P: the end of tile t's bucket-dd block = the slot after its last record
            tile_blk = np.arange(lo, b)[d[lo:b] == dd]
            P = slot[tile_blk].max() + 1
            both = np.concatenate([L, R])  # input order: left first
            o = np.argsort(x["key"][both], kind="stable")
            out[P - L.size + np.arange(both.size)] = x[both[o]]
    return out, ok


def _keys(rng, n, run_values=None):
    a = np.zeros(n, dtype=DT)
    k = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    if run_values is not None:  # few values of the two run bytes: long runs
        pool = rng.choice(1 << 16, run_values, replace=False).astype(np.uint64)
        k = (k & ~np.uint64(0xFFFF << 40)) | (pool[rng.integers(0, run_values, n)] << np.uint64(40))
    a["key"] = k
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


@pytest.mark.parametrize("n,T,run_values", [(3000, 64, 150), (5000, 128, 100), (4096, 64, None),
                                            (2047, 32, 400), (6000, 256, 60)])
def test_model_matches_stable_sort(n, T, run_values):
    """Runs of ~10-100 records (a few to ~half a tile) and uniform keys; most
    draws stay under the cap, and every one that does is exact."""
    done = 0
    for seed in range(6):
        rng = np.random.default_rng(seed * 1000 + n)
        a = _keys(rng, n, run_values)
        want = a[np.argsort(a["key"], kind="stable")]
        out, ok = hybrid_model(a, [5, 6, 7], T, cap=T // 2)
        if ok:
            assert np.array_equal(out, want), seed
            done += 1
    assert done >= 4


def test_model_duplicates_across_tiles():
    """Equal keys split between tiles: the left tile's records come first."""
    rng = np.random.default_rng(3)
    n = 4000
    a = np.zeros(n, dtype=DT)
    pool = rng.integers(0, 2**64 - 1, 300, dtype=np.uint64)
    a["key"] = pool[rng.integers(0, pool.size, n)]
    a["val"] = np.arange(n, dtype=np.uint64)
    out, ok = hybrid_model(a, [5, 6, 7], 128, cap=64)
    assert ok
    assert np.array_equal(out, a[np.argsort(a["key"], kind="stable")])


def test_model_reports_runs_past_the_cap():
    """A run of one run-key value over the cap on a side is reported, never
    silently mis-sorted."""
    rng = np.random.default_rng(4)
    a = _keys(rng, 4096, run_values=2)  # ~2048-record runs
    _, ok = hybrid_model(a, [5, 6, 7], 64, cap=32)
    assert not ok
