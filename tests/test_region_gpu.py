"""The regional first pass (LSB_OPT_REGION_FIRST) against the
oracle and against the usual start (a histogram read before the first pass).

A P == 1 LSD sort of at least 2^27 records (LSB_REGION_MIN lowers that for
these tests) starts with a pass that needs no histogram: the records of each
(digit-0 bucket, sub-array) class go to a slot range of their own, and the
second pass reads that layout back to a dense one.  The output must be the
stable sort bit for bit whichever way a sort starts:
  * uniform keys take the regional pass (lsb_get_first_pass says so);
  * skewed or structured keys, which a 2^20-record sample catches, take the
    histogram read;
  * keys that overflow a region where the sample does not look make the sort
    start over from its input (LSB_FIRST_REGIONAL_REDONE);
  * several sorts on one context, in both forms, keep the look-back tracks
    of the two tile counts apart.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = np.dtype([("key", "<u8"), ("val", "<u8")])


def _stable(a):
    return a[np.argsort(a["key"], kind="stable")]


def _uniform(n, seed):
    rng = np.random.default_rng(seed)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


def _sort(L, a, region=1):
    w = L.World(a.size, ranks=1)
    try:
        w.set_option(L.OPT_REGION_FIRST, region)
        w.scatter_global(a)
        w.my_sort()
        out = w.gather_global()
        return out, w.first_pass(), w.last_sort()
    finally:
        w.close()


@pytest.fixture
def small_regions(monkeypatch):
    """Regional first pass from 2^16 records on (contexts created after this)."""
    monkeypatch.setenv("LSB_REGION_MIN", str(1 << 16))


@pytest.mark.parametrize("n", [1 << 16, 1_000_003, (1 << 22) + 77])
def test_uniform_takes_the_regional_pass(lsb_built, oracle_mod, small_regions, n):
    a = _uniform(n, n)
    out, first, (passes, _, _) = _sort(lsb_built, a)
    assert first == lsb_built.FIRST_REGIONAL
    assert passes == 8
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    out0, first0, _ = _sort(lsb_built, a, region=0)
    assert first0 == lsb_built.FIRST_COUNT
    assert np.array_equal(out, out0)


def test_golden_row_through_the_regional_pass(lsb_built, oracle_mod, digests, small_regions):
    d = [r for r in digests["rows"] if r["P"] == 1][0]
    with lsb_built.World(d["n"], ranks=1) as w:
        w.generate()
        assert oracle_mod.digest(w.gather_global()) == d["input"]
        w.my_sort()
        assert w.first_pass() == lsb_built.FIRST_REGIONAL
        assert oracle_mod.digest(w.gather_global()) == d["output"]
        ok, bad = w.verify()
        assert ok and bad == -1


@pytest.mark.parametrize("name", ["all_equal", "two_keys", "hot_bucket", "high_bits_only", "zipf",
                                  "small_range", "low_byte_even", "sorted", "reverse"])
def test_keys_the_sample_sends_elsewhere(lsb_built, oracle_mod, small_regions, name):
    """Skewed or structured keys take the histogram read; sorted and reversed
    uniform keys take the regional pass.  Bit-exact either way."""
    n = 1 << 20
    rng = np.random.default_rng(len(name))
    a = _uniform(n, 7)
    k = a["key"]
    if name == "all_equal":
        k[:] = np.uint64(0xDEADBEEF12345678)
    elif name == "two_keys":
        k[:] = np.where(rng.random(n) < 0.5, 7, 0xFFFFFFFFFFFFFFFF).astype(np.uint64)
    elif name == "hot_bucket":
        hot = rng.random(n) < 0.9
        k[hot] = (k[hot] & ~np.uint64(0xFF00FF)) | np.uint64(0x2A002A)
    elif name == "high_bits_only":
        k[:] = rng.integers(0, 256, n, dtype=np.uint64) << np.uint64(56)
    elif name == "zipf":
        k[:] = np.minimum(rng.zipf(1.1, n), 2**20).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    elif name == "small_range":
        k[:] = rng.integers(0, 3, n, dtype=np.uint64)
    elif name == "low_byte_even":  # every byte varies, half the digit-0 buckets empty
        k[:] = k & ~np.uint64(1)
    elif name == "sorted":
        k[:] = np.sort(k)
    elif name == "reverse":
        k[:] = np.sort(k)[::-1]
    out, first, _ = _sort(lsb_built, a)
    want = lsb_built.FIRST_REGIONAL if name in ("sorted", "reverse") else lsb_built.FIRST_COUNT
    assert first == want
    assert np.array_equal(out, oracle_mod.stable_sort(a))


@pytest.mark.parametrize("extra", [4700, 3000])
def test_overflow_the_sample_misses_starts_over(lsb_built, small_regions, extra):
    """2^24 records: the sample reads every 16th tile; `extra` more records of
    digit-0 bucket 7 in sub-array 3, all in unsampled tiles.  Region (7, 3)
    holds 3 tiles (12288 slots) over a mean of 8192: +4700 overflows it (the
    sort starts over), +3000 fills its third tile most of the way."""
    n = 1 << 24
    a = _uniform(n, 24)
    k = a["key"]
    tile = np.arange(n) // 4096
    lo = 3 * n // 8
    cand = np.flatnonzero((np.arange(n) >= lo) & (np.arange(n) < lo + n // 8) & (tile % 16 != 0)
                          & ((k & np.uint64(0xFF)) != 7))
    pick = cand[:: max(1, cand.size // extra)][:extra]
    k[pick] = (k[pick] & ~np.uint64(0xFF)) | np.uint64(7)
    out, first, _ = _sort(lsb_built, a)
    want = lsb_built.FIRST_REGIONAL_REDONE if extra > 4096 else lsb_built.FIRST_REGIONAL
    assert first == want
    assert np.array_equal(out, _stable(a))


def test_many_sorts_on_one_context(lsb_built, small_regions):
    """Regional, usual and restarted sorts in turn on one context: each
    verified (the look-back rows of the two tile counts on separate tracks)."""
    n = (1 << 22) + 4097
    L = lsb_built
    with L.World(n, ranks=1) as w:
        forms = []
        for i in range(7):
            if i in (2, 5):
                a = _uniform(n, i)
                a["key"][:] = a["key"] & ~np.uint64(0xFF00)  # digit 1 constant: the usual start
                w.scatter_global(a)
                w.my_sort()
                assert np.array_equal(w.gather_global(), _stable(a))
            else:
                w.set_option(L.OPT_REGION_FIRST, 0 if i == 4 else 1)
                w.generate()
                w.my_sort()
                ok, bad = w.verify()
                assert ok and bad == -1
            forms.append(w.first_pass())
        assert forms == [1, 1, 0, 1, 0, 0, 1]


@pytest.mark.parametrize("n", [1 << 27, (1 << 27) + 12345])
def test_default_threshold_verifies(lsb_built, n):
    """The default form at 2^27 records: regional, verified on device."""
    with lsb_built.World(n, ranks=1) as w:
        for _ in range(2):
            w.generate()
            w.my_sort()
            assert w.first_pass() == lsb_built.FIRST_REGIONAL
            ok, bad = w.verify()
            assert ok and bad == -1


def test_below_threshold_takes_the_count(lsb_built, monkeypatch):
    monkeypatch.delenv("LSB_REGION_MIN", raising=False)
    with lsb_built.World((1 << 27) - 1, ranks=1) as w:
        w.generate()
        w.my_sort()
        assert w.first_pass() == lsb_built.FIRST_COUNT
        ok, _ = w.verify()
        assert ok


def test_hybrid_and_regional_sorts_share_a_context(lsb_built, small_regions):
    """The hybrid permutes A, B and R; the regional first pass writes its
    layout into whichever buffer is B by then, so R holds as many records as
    A and B.  Hybrid and LSD sorts in turn on one context, each verified."""
    L = lsb_built
    n = (1 << 22) + 333
    with L.World(n, ranks=1) as w:
        for hybrid in (1, 0, 1, 0, 2, 0, 0):
            w.set_option(L.OPT_HYBRID, hybrid)
            w.generate()
            w.my_sort()
            ok, bad = w.verify()
            assert ok and bad == -1, hybrid
            if hybrid == 0:
                assert w.first_pass() == L.FIRST_REGIONAL


@pytest.mark.parametrize("hybrid", [1, 2])
def test_hybrid_starts_with_the_regional_pass(lsb_built, oracle_mod, small_regions, hybrid):
    """The hybrid's first byte pass (the lowest of its top bytes) into the
    regional layout, its second reading it; bit-exact, then an overflow the
    sample misses (the kept input sorted the usual way)."""
    L = lsb_built
    n = (1 << 22) + 4097
    a = _uniform(n, 22 + hybrid)
    with L.World(n, ranks=1) as w:
        w.set_option(L.OPT_HYBRID, hybrid)
        w.scatter_global(a)
        w.my_sort()
        assert w.first_pass() == L.FIRST_REGIONAL
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a))
        # 2^22 records: k = 3 top bytes (5, 6, 7); crowd byte 5 = 0x21 in
        # sub-array 6's tiles that the sample (tile g * TT / 256 for g < 256)
        # does not read.
        b = _uniform(n, 5)
        k = b["key"]
        tile = np.arange(n) // 4096
        TT = (n + 4095) // 4096
        sampled = np.array(sorted({g * TT // 256 for g in range(256)}))
        lo, hi = 6 * TT // 8 * 4096, 7 * TT // 8 * 4096
        sel = np.flatnonzero((np.arange(n) >= lo) & (np.arange(n) < hi) & ~np.isin(tile, sampled))[:9000]
        k[sel] = (k[sel] & ~np.uint64(0xFF << 40)) | np.uint64(0x21 << 40)
        w.scatter_global(b)
        w.my_sort()
        assert w.first_pass() == L.FIRST_REGIONAL_REDONE
        assert np.array_equal(w.gather_global(), _stable(b))
