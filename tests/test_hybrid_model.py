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


# ---- the fused pass's segment walk and the error dispatch
# The model above orders every in-tile segment exactly.  The kernel does not:
# each record walks its segment in the stage at most kSegMax records each way
# (k_onesweep SEG, csrc/lsb_kernels.hip, the write-out's walk), and a segment
# longer than that inside a tile gets slots from cut walks, which can collide:
# the pass then sets error bit 2 and its output is no permutation (duplicates,
# and holes keeping whatever the buffer held).  k_segfix sets bit 1 for a
# crossing run it leaves alone, whose output IS a permutation.  The runtime's
# dispatch (LocalSort::finish, csrc/lsb_passes.cpp): no bit -> done; bit 1
# alone -> k_segsort over the pass's output; bit 2 -> the LSD passes over the
# kept input.  Before d4f7b64 every error took k_segsort, which is how stress
# seed 19 kept a wrong sort.


def fused_pass_model(x, last, pmask, T, seg_max, stale):
    """k_onesweep SEG on x (stably sorted by the lower top bytes) into a
    buffer holding `stale`: returns (out, bit2)."""
    m = x.size
    d = _byte(x["key"], last)
    counts = np.bincount(d, minlength=256)
    base = np.concatenate([[0], np.cumsum(counts)[:-1]])
    seen = np.zeros(256, dtype=np.int64)  # records of each bucket in earlier tiles
    out = stale.copy()
    bit2 = False
    keys = x["key"]
    for t0 in range(0, m, T):
        idx = np.arange(t0, min(t0 + T, m))
        stage = idx[np.argsort(d[idx], kind="stable")]  # the tile, bucket-ordered
        sk = keys[stage]
        sd = d[stage]
        nvalid = stage.size
        lstart = {dd: int(np.argmax(sd == dd)) for dd in np.unique(sd)}
        for j in range(nvalid):
            v = sk[j]
            pk = v & pmask
            pos = j
            sp = j > 0 and (sk[j - 1] & pmask) == pk
            sn = j + 1 < nvalid and (sk[j + 1] & pmask) == pk
            if sp or sn:
                less = eqb = 0
                k = j - 1
                klo = max(j - seg_max, 0)
                while k >= klo:
                    kk = sk[k]
                    if (kk & pmask) != pk:
                        break
                    less += kk < v
                    eqb += kk == v
                    k -= 1
                sfirst = k + 1
                too_long = k < klo and klo > 0
                khi = min(j + 1 + seg_max, nvalid)
                k = j + 1
                while k < khi:
                    kk = sk[k]
                    if (kk & pmask) != pk:
                        break
                    less += kk < v
                    k += 1
                too_long |= k == khi and khi < nvalid
                bit2 |= too_long
                pos = sfirst + less + eqb
            dd = int(sd[j])
            slot = base[dd] + seen[dd] + (pos - lstart[dd])
            if 0 <= slot < m:  # the kernel clamps into the buffer
                out[slot] = x[stage[j]]
        seen += np.bincount(sd, minlength=256)
    return out, bit2


def segfix_bit1(x, msd, T, cap):
    """k_segfix's verdict only (bit 1): a crossing run too long to merge."""
    last = msd[-1]
    rmask = np.uint64(sum(0xFF << (8 * b) for b in msd)) & ~np.uint64(0xFF << (8 * last))
    rk = x["key"] & rmask
    m = x.size
    for b in range(T, m, T):
        lo, hi = b - T, min(b + T, m)
        v = rk[b - 1]
        if rk[b] != v:
            continue
        a_ = c_ = 0
        while b - 1 - a_ >= lo and rk[b - 1 - a_] == v:
            a_ += 1
        while b + c_ < hi and rk[b + c_] == v:
            c_ += 1
        if a_ > cap or c_ > cap or (b - a_ == lo and lo > 0 and rk[lo - 1] == v) or \
                (b + c_ == hi and hi < m and rk[hi] == v):
            return True
    return False


def segsort_model(y, pmask, seg_max):
    """k_segsort over y (taken as sorted by pmask): every maximal run of equal
    pmask ordered by the whole key; (out, err) with err for a run over seg_max."""
    out = y.copy()
    p = y["key"] & pmask
    i = 0
    while i < y.size:
        j = i + 1
        while j < y.size and p[j] == p[i]:
            j += 1
        if j - i > seg_max:
            return y, True
        out[i:j] = y[i:j][np.argsort(y["key"][i:j], kind="stable")]
        i = j
    return out, False


def hybrid_mode1(a, msd, T, seg_max, cap, stale, dispatch):
    """The hybrid's mode 1 end to end on a (one rank): passes on msd[:-1], the
    fused SEG pass, k_segfix, then the error dispatch ("shipped": bit 2 goes
    to the LSD passes; "pre_d4f7b64": every error takes k_segsort)."""
    x = a
    for b in msd[:-1]:
        x = x[np.argsort(_byte(x["key"], b), kind="stable")]
    pmask = np.uint64(sum(0xFF << (8 * b) for b in msd))
    fused, bit2 = fused_pass_model(x, msd[-1], pmask, T, seg_max, stale)
    if not bit2:  # k_segfix as the first model does it (the fused output is then exact in-tile)
        fused, ok = hybrid_model(a, msd, T, cap)
        bit1 = not ok
    else:
        bit1 = segfix_bit1(x, msd, T, cap)
    err = (1 if bit1 else 0) | (2 if bit2 else 0)
    if err == 0:
        return fused, "fused"
    lsd = a[np.argsort(a["key"], kind="stable")]  # the LSD passes over the kept input
    if dispatch == "shipped" and err & 2:
        return lsd, "lsd"
    out, serr = segsort_model(fused, pmask, seg_max)
    return (lsd, "lsd") if serr else (out, "segsort")


def _seed19_like(rng, n, v4=64):
    """Stress seed 19's shape: bytes 3 and 5 constant, bytes 6
    and 7 two values each, so the hybrid's top bytes are 4, 6, 7; byte 4 takes
    v4 values here, so a segment (records equal on them) holds ~n / (4 v4)
    records: several times the walk's cut, as ~340 records were against
    kSegMax = 64 in the stress input."""
    k = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    k = (k & ~np.uint64(0xFF << 24)) | np.uint64(0x5A << 24)
    k = (k & ~np.uint64(0xFF << 40)) | np.uint64(0x11 << 40)
    k = (k & ~np.uint64(0xFF << 32)) | (rng.integers(0, v4, n, dtype=np.uint64) << np.uint64(32))
    b6 = rng.choice(np.array([0x20, 0x9C], dtype=np.uint64), n)
    b7 = rng.choice(np.array([0x03, 0xE1], dtype=np.uint64), n)
    k = (k & ~np.uint64(0xFFFF << 48)) | (b6 << np.uint64(48)) | (b7 << np.uint64(56))
    a = np.zeros(n, dtype=DT)
    a["key"] = k
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


def test_pre_fix_dispatch_keeps_a_wrong_sort_shipped_does_not():
    """Segments of ~250 records, ~128 of them inside a 256-record tile, with
    the walk cut at 16: the fused pass's slots collide (bit 2).  The
    pre-d4f7b64 dispatch hands that output to k_segsort, whose runs the stale
    records in the holes cut short, and keeps a wrong sort for some inputs;
    the shipped dispatch re-sorts the kept input exactly every time."""
    msd = [4, 6, 7]
    wrong_pre = 0
    for seed in range(6):
        rng = np.random.default_rng(1900 + seed)
        a = _seed19_like(rng, 8000, v4=8)
        want = a[np.argsort(a["key"], kind="stable")]
        stale = _keys(np.random.default_rng(seed), a.size)  # what the pass's buffer held
        stale["val"] += np.uint64(10**9)
        out, route = hybrid_mode1(a, msd, 256, 16, 128, stale, "shipped")
        assert route == "lsd" and np.array_equal(out, want), seed
        out, route = hybrid_mode1(a, msd, 256, 16, 128, stale, "pre_d4f7b64")
        if not np.array_equal(out, want):
            assert route == "segsort"  # the wrong answer came through k_segsort
            assert np.unique(out["val"]).size < out.size or out["val"].max() >= 10**9  # no permutation
            wrong_pre += 1
    assert wrong_pre >= 2  # the round-5 bug, reproduced by the model (3 of these 6 inputs)


def test_dispatch_exact_across_the_cap():
    """Small tiles (32-256 records) and segments on both sides of the walk's
    cut (16): bytes 5 and 6 from a pool (runs of ~seg_len records), byte 7
    from two values (a segment holds ~seg_len / 2 records) or uniform (short
    segments, long crossing runs for k_segfix).  Every route of
    the shipped dispatch -- the fused output, k_segsort after bit 1, the LSD
    passes after bit 2 -- ends in the stable sort, bit for bit, and the grid
    reaches all three."""
    msd = [5, 6, 7]
    routes = {}
    for T in (32, 64, 128, 256):
        for seg_len in (8, 24, 48, 96, 192):
            for seed, two in ((0, True), (1, False)):
                rng = np.random.default_rng(seed * 7919 + T + seg_len)
                n = 3000 + seed * 333
                a = _keys(rng, n, run_values=max(1, n // seg_len))
                if two:
                    a["key"] = (a["key"] & ~np.uint64(0xFF << 56)) | \
                        (rng.choice(np.array([0x11, 0xEE], dtype=np.uint64), n) << np.uint64(56))
                want = a[np.argsort(a["key"], kind="stable")]
                stale = _keys(np.random.default_rng(seed + 99), n)
                out, route = hybrid_mode1(a, msd, T, 16, T // 2, stale, "shipped")
                routes.setdefault(route, []).append((T, seg_len))
                assert np.array_equal(out, want), (T, seg_len, seed, route)
    assert set(routes) == {"fused", "segsort", "lsd"}, {k: len(v) for k, v in routes.items()}
