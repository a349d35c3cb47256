"""Host-side checks of the C ABI (no GPU needed).

* the library loads and exports every function include/lsb.h declares;
* block-partition helpers equal DistributedArray::create's
  (mpi/mpi_lsbsort.cpp:144-149);
* the exchange planner (lsb_plan_exchange) against an independent Python
  derivation of the reference's digit-major, rank-minor destination rule
  (mpi/mpi_lsbsort.cpp:350, 378, 401, 546-560), and end to end: P ranks
  simulated with the oracle's local pass + numpy copies, using the planner
  as the runtime does, reproduce the reference's golden digests.
"""
import os
import re

import numpy as np
import pytest

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "lsb.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lsb_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol(lsb_built):
    import ctypes
    lib = ctypes.CDLL(lsb_built.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_exchange_stats_struct_layout(lsb_built, tmp_path):
    """lsbsort.ExchangeStats (ctypes) has lsb_exchange_stats_t's layout:
    every field's offset and the size, as the C compiler lays them out."""
    import ctypes
    import subprocess
    fields = [f for f, _ in lsb_built.ExchangeStats._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "lsb.h"\nint main(void) {\n' +
                   "".join(f'  printf("%zu\\n", offsetof(lsb_exchange_stats_t, {f}));\n' for f in fields) +
                   '  printf("%zu\\n", sizeof(lsb_exchange_stats_t));\n  return 0;\n}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [getattr(lsb_built.ExchangeStats, f).offset for f in fields] + [ctypes.sizeof(lsb_built.ExchangeStats)]
    assert got == want
    assert lsb_built.MAX_RANKS == 64 and len(lsb_built.KERNEL_NAMES) == 9


def test_partition_helpers(lsb_built, oracle_mod):
    for n in (0, 1, 2, 7, 20, 1000003, 1 << 33):
        for P in (1, 2, 3, 4, 5, 8, 13):
            assert lsb_built.per_rank(n, P) == oracle_mod.per_rank(n, P)
            for r in range(P):
                assert lsb_built.here(n, P, r) == oracle_mod.here(n, P, r)


def test_library_built_from_this_tree(lsb_built):
    """The compiled-in source digest (lsb_build_info) equals the tree's."""
    info = lsb_built.build_info()
    assert info["sha256"] == lsb_built.source_digest(), info


def test_strerror(lsb_built):
    lib = lsb_built._lib()
    assert lib.lsb_strerror(0) == b"ok"
    assert lib.lsb_strerror(5) == b"verification failed"


def py_plan(n, P, me, hist):
    """Independent derivation: explicit per-element destinations."""
    nb = hist.shape[1]
    per = -(-n // P)
    total = hist.sum(axis=0)
    base = np.concatenate([[0], np.cumsum(total)[:-1]])
    gstart = base[None, :] + np.concatenate([np.zeros((1, nb), np.int64),
                                              np.cumsum(hist, axis=0)[:-1]])  # [s][b]
    dests = {}
    for s in range(P):
        d = np.concatenate([gstart[s, b] + np.arange(hist[s, b]) for b in range(nb)]) \
            if hist[s].sum() else np.zeros(0, np.int64)
        bk = np.repeat(np.arange(nb), hist[s])
        dests[s] = (d.astype(np.int64), bk)
    d_me, _ = dests[me]
    owners = d_me // per if per else d_me
    send_counts = np.bincount(owners, minlength=P)[:P] if d_me.size else np.zeros(P, np.int64)
    recv = []
    for s in range(P):
        d, bk = dests[s]
        sel = (d // per == me) if per else np.zeros(d.size, bool)
        recv.append((d[sel] - me * per, bk[sel]))
    return send_counts, recv


@pytest.mark.parametrize("seed", range(12))
def test_planner_matches_independent_derivation(lsb_built, seed):
    rng = np.random.default_rng(seed)
    P = int(rng.integers(1, 9))
    nb = int(rng.choice([1, 2, 5, 256]))
    hist = rng.integers(0, 6, (P, nb)).astype(np.int64)
    if seed % 3 == 0:
        hist[:, rng.integers(0, nb)] = 0
    n = int(hist.sum())
    # each rank's count must equal here(n, P, r): rebalance rows to the partition
    here = np.array([lsb_built.here(n, P, r) for r in range(P)])
    flat = np.repeat(np.tile(np.arange(nb), P), hist.reshape(-1))
    rng.shuffle(flat)
    hist = np.zeros((P, nb), np.int64)
    pos = 0
    for r in range(P):
        np.add.at(hist[r], flat[pos:pos + here[r]], 1)
        pos += here[r]
    for me in range(P):
        plan = lsb_built.plan_exchange(n, P, me, hist)
        sc, recv = py_plan(n, P, me, hist)
        assert np.array_equal(plan["send_counts"], sc)
        assert np.array_equal(plan["send_displs"], np.concatenate([[0], np.cumsum(sc)[:-1]]))
        rc = np.array([r[0].size for r in recv])
        assert np.array_equal(plan["recv_counts"], rc)
        # place_off maps every received element to its slot
        k = 0
        for s in range(P):
            slots, bk = recv[s]
            for j in range(slots.size):
                assert plan["place_off"][s, bk[j]] + k == slots[j]
                k += 1


def simulate(lsbsort, oracle, n, P):
    """The runtime's P > 1 pass loop with numpy for the device work."""
    per = -(-n // P)
    slots = oracle.generate_slots(n, P)
    A = [slots[r * per: r * per + lsbsort.here(n, P, r)].copy() for r in range(P)]
    for d in range(8):
        B, hist = [], np.zeros((P, 256), np.int64)
        for r in range(P):
            b, h = oracle.local_pass(A[r], 8, d)
            B.append(b)
            hist[r] = h
        plans = [lsbsort.plan_exchange(n, P, r, hist) for r in range(P)]
        for q in range(P):
            R = np.empty(lsbsort.here(n, P, q), dtype=oracle.ELEM_DTYPE)
            for s in range(P):
                c = plans[s]["send_counts"][q]
                assert c == plans[q]["recv_counts"][s]
                so, ro = plans[s]["send_displs"][q], plans[q]["recv_displs"][s]
                R[ro:ro + c] = B[s][so:so + c]
            ends = np.cumsum(plans[q]["recv_counts"])
            src = np.searchsorted(ends, np.arange(R.size), side="right")
            dig = ((R["key"] >> np.uint64(8 * d)) & np.uint64(255)).astype(np.int64)
            dst = plans[q]["place_off"][src, dig] + np.arange(R.size)
            out = np.empty_like(R)
            out[dst] = R
            assert np.array_equal(np.sort(dst), np.arange(R.size))
            A[q] = out
    return np.concatenate(A) if A else np.empty(0, oracle.ELEM_DTYPE)


@pytest.mark.parametrize("row", [0, 1, 3])
def test_simulated_exchange_reproduces_golden(lsb_built, oracle_mod, digests, row):
    d = digests["rows"][row]
    out = simulate(lsb_built, oracle_mod, d["n"], d["P"])
    assert oracle_mod.digest(out) == d["output"]


@pytest.mark.parametrize("n,P", [(0, 3), (1, 4), (5, 8), (17, 8), (1001, 7)])
def test_simulated_exchange_small(lsb_built, oracle_mod, n, P):
    out = simulate(lsb_built, oracle_mod, n, P)
    assert np.array_equal(out, oracle_mod.mpi_sort(n, P))


def simulate16(lsbsort, oracle, n, P):
    """P > 1 pass loop with 16-bit exchange digits (two 8-bit local sub-passes)."""
    per = -(-n // P)
    slots = oracle.generate_slots(n, P)
    A = [slots[r * per: r * per + lsbsort.here(n, P, r)].copy() for r in range(P)]
    for d in range(4):
        hist = np.zeros((P, 65536), np.int64)
        for r in range(P):
            x, _ = oracle.local_pass(A[r], 8, 2 * d)
            x, _ = oracle.local_pass(x, 8, 2 * d + 1)
            A[r] = x
            dig = ((x["key"] >> np.uint64(16 * d)) & np.uint64(0xFFFF)).astype(np.int64)
            hist[r] = np.bincount(dig, minlength=65536)
        plans = [lsbsort.plan_exchange(n, P, r, hist) for r in range(P)]
        out = []
        for q in range(P):
            R = np.concatenate([A[s][plans[s]["send_displs"][q]:plans[s]["send_displs"][q] + plans[s]["send_counts"][q]]
                                for s in range(P)])
            ends = np.cumsum(plans[q]["recv_counts"])
            src = np.searchsorted(ends, np.arange(R.size), side="right")
            dig = ((R["key"] >> np.uint64(16 * d)) & np.uint64(0xFFFF)).astype(np.int64)
            dst = plans[q]["place_off"][src, dig] + np.arange(R.size)
            o = np.empty_like(R)
            o[dst] = R
            out.append(o)
        A = out
    return np.concatenate(A)


@pytest.mark.parametrize("n,P", [(50_003, 3), (1000, 8)])
def test_simulated_exchange_radix16(lsb_built, oracle_mod, n, P):
    out = simulate16(lsb_built, oracle_mod, n, P)
    assert np.array_equal(out, oracle_mod.mpi_sort(n, P))


# ------------------------------------------------------------ error paths
# Checks that return before any device call, so they run without a GPU.
def test_error_codes_without_device(lsb_built):
    import ctypes
    lib = lsb_built._lib()
    ctx = ctypes.c_void_p()
    # lsb_create: null out, bad P, bad n, unsupported radix
    assert lib.lsb_create(None, 10, 1, None, 8) == 1
    assert lib.lsb_create(ctypes.byref(ctx), 10, 0, None, 8) == 1
    assert lib.lsb_create(ctypes.byref(ctx), 10, 65, None, 8) == 1
    assert lib.lsb_create(ctypes.byref(ctx), -1, 1, None, 8) == 1
    assert lib.lsb_create(ctypes.byref(ctx), 10, 1, None, 12) == 6
    assert not ctx.value
    uid = bytes(128)
    assert lib.lsb_create_rank(ctypes.byref(ctx), 10, 2, 2, 0, 8, uid) == 1   # rank >= P
    assert lib.lsb_create_rank(ctypes.byref(ctx), 10, 2, 0, 0, 8, None) == 1  # no id
    assert lib.lsb_create_rank(ctypes.byref(ctx), 10, 2, 0, 0, 32, uid) == 6
    # every context call rejects a null context
    n = ctypes.c_int64()
    assert lib.lsb_sort(None) == 1
    assert lib.lsb_pass(None, 0) == 1
    assert lib.lsb_sync(None) == 1
    assert lib.lsb_generate(None) == 1
    assert lib.lsb_set_option(None, 0, 1) == 1
    assert lib.lsb_verify(None, ctypes.byref(n)) == 1
    assert lib.lsb_get_kernel_stats(None, 0, None, None) == 1
    assert lib.lsb_get_last_sort(None, None, None, None) == 1
    lib.lsb_destroy(None)  # no-op
    for code in range(8):
        assert lib.lsb_strerror(code)


def test_planner_rejects_bad_input(lsb_built):
    import ctypes
    lib = lsb_built._lib()
    P, nb = 2, 256
    hist = np.zeros((P, nb), dtype=np.int64)
    outs = [np.zeros(P, dtype=np.int64) for _ in range(4)] + [np.zeros(P * nb, dtype=np.int64)]
    ptrs = [o.ctypes.data for o in outs]
    assert lib.lsb_plan_exchange(0, P, 0, nb, hist.ctypes.data, *ptrs) == 0
    assert lib.lsb_plan_exchange(0, P, 2, nb, hist.ctypes.data, *ptrs) == 1    # rank >= P
    hist[0, 3] = -1
    assert lib.lsb_plan_exchange(10, P, 0, nb, hist.ctypes.data, *ptrs) == 1   # negative count
    hist[0, 3] = 11
    assert lib.lsb_plan_exchange(10, P, 0, nb, hist.ctypes.data, *ptrs) == 1   # counts exceed n


# ------------------------------------------------- whole-key exchange plan
def simulate_merge(lsbsort, inp_parts, n, P):
    """radix_bits = 64 on the CPU: every rank sorts its block (stable, by key),
    the cuts come from lsb_plan_merge given each rank's counts below / up to
    the key at global position q * per (derived here independently, from the
    globally sorted keys), one all-to-all of contiguous ranges, then each
    owner merges its P runs in rank order."""
    per = -(-n // P) if P else 0
    A = [x[np.argsort(x["key"], kind="stable")] for x in inp_parts]
    allkeys = np.sort(np.concatenate([x["key"] for x in A])) if n else np.zeros(0, np.uint64)
    below = np.zeros((P, max(P - 1, 0)), np.int64)
    upto = np.zeros_like(below)
    for q in range(1, P):
        T = q * per
        if T >= n:
            continue
        k = allkeys[T]
        for s in range(P):
            below[s, q - 1] = np.searchsorted(A[s]["key"], k, side="left")
            upto[s, q - 1] = np.searchsorted(A[s]["key"], k, side="right")
    plans = [lsbsort.plan_merge(n, P, r, below, upto) for r in range(P)]
    out = []
    for q in range(P):
        runs = []
        for s in range(P):
            c = plans[s]["send_counts"][q]
            assert c == plans[q]["recv_counts"][s]
            so = plans[s]["send_displs"][q]
            runs.append(A[s][so:so + c])
        R = np.concatenate(runs)
        assert R.size == lsbsort.here(n, P, q)
        out.append(R[np.argsort(R["key"], kind="stable")])  # stable merge, rank order
    return np.concatenate(out) if out else np.empty(0, inp_parts[0].dtype)


def _parts(oracle, n, P, keymap=None):
    per = -(-n // P)
    slots = oracle.generate_slots(n, P)
    parts = [slots[r * per: r * per + (max(0, min(per, n - r * per)))].copy() for r in range(P)]
    if keymap is not None:
        for x in parts:
            x["key"] = keymap(x["key"])
    return parts


@pytest.mark.parametrize("row", [0, 1, 3, 4])
def test_simulated_merge_exchange_reproduces_golden(lsb_built, oracle_mod, digests, row):
    d = digests["rows"][row]
    out = simulate_merge(lsb_built, _parts(oracle_mod, d["n"], d["P"]), d["n"], d["P"])
    assert oracle_mod.digest(out) == d["output"]


@pytest.mark.parametrize("n,P", [(0, 3), (1, 4), (5, 8), (17, 8), (1001, 7), (4096, 64)])
def test_simulated_merge_exchange_small(lsb_built, oracle_mod, n, P):
    out = simulate_merge(lsb_built, _parts(oracle_mod, n, P), n, P)
    assert np.array_equal(out, oracle_mod.mpi_sort(n, P))


@pytest.mark.parametrize("name,keymap", [
    ("three_values", lambda k: k % np.uint64(3)),
    ("all_equal", lambda k: np.zeros_like(k)),
    ("hot_key", lambda k: np.where(k % np.uint64(4) == 0, np.uint64(7), k)),
])
@pytest.mark.parametrize("n,P", [(10_007, 2), (20_000, 5), (3_333, 8)])
def test_simulated_merge_exchange_duplicates(lsb_built, oracle_mod, name, keymap, n, P):
    """Equal keys straddling owner boundaries: cuts follow rank order."""
    parts = _parts(oracle_mod, n, P, keymap)
    out = simulate_merge(lsb_built, parts, n, P)
    inp = np.concatenate(parts)
    assert np.array_equal(out, inp[np.argsort(inp["key"], kind="stable")])


def test_plan_merge_rejects_bad_counts(lsb_built):
    n, P = 100, 2
    ok = lsb_built.plan_merge(n, P, 0, np.array([[40], [9]]), np.array([[41], [10]]))
    assert list(ok["send_counts"]) == [41, 9] and list(ok["recv_counts"]) == [41, 9]
    with pytest.raises(lsb_built.LsbError):      # target 50 not bracketed
        lsb_built.plan_merge(n, P, 0, np.array([[10], [10]]), np.array([[20], [20]]))
    with pytest.raises(lsb_built.LsbError):      # below > upto
        lsb_built.plan_merge(n, P, 0, np.array([[30], [30]]), np.array([[20], [40]]))
    with pytest.raises(lsb_built.LsbError):      # more than the rank holds
        lsb_built.plan_merge(n, P, 0, np.array([[40], [9]]), np.array([[60], [10]]))


def test_rank_footprint_model(lsb_built, monkeypatch):
    """lsb_rank_footprint (host arithmetic): record buffers rounded up to whole
    1 GiB VMM pieces (hipMalloc'd ones are not), R only with an exchange or
    the hybrid, 4 B of look-back row per bucket per 4096-record tile, and the
    placement probe's one extra candidate live at a time (by default 4
    candidates for buffers of at least 4 GiB; LSB_PLACEMENT_CANDIDATES = K
    sets K; round 6: K passes, losers freed at once)."""
    L = lsb_built
    gib = 1 << 30
    monkeypatch.delenv("LSB_PLACEMENT_CANDIDATES", raising=False)
    monkeypatch.delenv("LSB_RECORD_ALLOC", raising=False)
    monkeypatch.delenv("LSB_VMM_CHUNK_MIB", raising=False)
    monkeypatch.delenv("LSB_REGION_MIN", raising=False)
    n = 1 << 30
    rows = (n // 4096) * 256 * 4
    # P == 1 blocks of >= 2^27 records: A and B hold the regional first pass's
    # slots (2048 regions of 130 tiles at 2^30: 17 pieces each) and its pass
    # over them has look-back rows of its own.
    slots = 2048 * 130 * 4096
    f = L.rank_footprint(n, 1, 8)
    assert 0 <= f["bytes"] - 34 * gib - rows - (slots // 4096) * 256 * 4 < 64 << 20
    assert f["probe_bytes"] == 17 * gib  # the default probe: one candidate of 17 pieces beside A and B
    monkeypatch.setenv("LSB_REGION_MIN", str(1 << 40))  # no regional slots from here on
    f = L.rank_footprint(n, 1, 8)
    assert f["probe_bytes"] == 16 * gib and 0 <= f["bytes"] - 32 * gib - rows < 64 << 20
    assert L.rank_footprint(n // 8, 1, 8)["probe_bytes"] == 0  # 2 GiB buffers: no default probe
    extra = L.rank_footprint(n, 1, 8, with_recv=True)["bytes"] - f["bytes"]
    assert 16 * gib <= extra < 16 * gib + (64 << 20)  # R, and the gathered passes' tile descriptors
    ragged = L.rank_footprint(n + 12345, 1, 8)["bytes"]
    assert ragged - f["bytes"] >= 2 * gib  # A and B each take a 17th piece
    monkeypatch.setenv("LSB_RECORD_ALLOC", "malloc")
    assert L.rank_footprint(n + 12345, 1, 8)["bytes"] - f["bytes"] < 1 << 20
    monkeypatch.delenv("LSB_RECORD_ALLOC")
    monkeypatch.setenv("LSB_PLACEMENT_CANDIDATES", "0")
    assert L.rank_footprint(n, 1, 8)["probe_bytes"] == 0
    monkeypatch.setenv("LSB_PLACEMENT_CANDIDATES", "8")
    assert L.rank_footprint(n, 1, 8)["probe_bytes"] == 16 * gib  # 8 candidates, still one at a time
    assert L.rank_footprint(1 << 20, 1, 8)["probe_bytes"] == 0  # buffers under 1 GiB: no probe
    # P ranks: per = ceil(n / P) records each
    assert L.rank_footprint(8 * n, 8, 16, with_recv=True)["bytes"] > 48 * gib
    with pytest.raises(L.LsbError):
        L.rank_footprint(n, 0, 8)
