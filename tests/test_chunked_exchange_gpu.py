"""The per-digit exchange in chunks (LSB_OPT_EXCHANGE_CHUNKS; VERDICT r05
missing item 1).

For a 16-bit exchange digit, one read after the low-byte pass counts the
digit and every chunk's high-byte histogram (launch_count16_chunks); the plan
puts a source's pieces in R in chunk order; then chunk k's high-byte pass runs
while chunk k - 1's records are on the wire, and chunk k is counted (or, in
the last exchange, placed) once it has arrived.  The output must be the
reference's (mpi/mpi_lsbsort.cpp:481-585) bit for bit: the oracle's stable
sort, the golden digests of the reference binary, and the unchunked exchange
on the same input.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from test_gpu_sort import DT

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _uniform(n, seed):
    rng = np.random.default_rng(seed)
    a = np.zeros(n, dtype=DT)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


def _sort(L, a, P, chunks, gather=1, force=0, stats=False):
    with L.World(a.size, ranks=P, radix_bits=16) as w:
        w.set_option(L.OPT_EXCHANGE_CHUNKS, chunks)
        w.set_option(L.OPT_EXCHANGE_GATHER, gather)
        if force:
            w.set_option(L.OPT_FORCE_EXCHANGE, 1)
        w.scatter_global(a)
        w.set_timing(stats)
        w.my_sort()
        out = w.gather_global()
        assert w.check_sorted()
        return out, w.last_sort(), (w.kernel_stats() if stats else None)


@pytest.mark.parametrize("chunks", [2, 4, 8])
@pytest.mark.parametrize("n,P", [(8 * 65536 + 12345, 8), (3 * 70001, 3), ((1 << 20) + 777, 2)])
def test_loopback_bit_exact(lsb_built, oracle_mod, n, P, chunks):
    a = _uniform(n, n ^ P ^ chunks)
    out, last, _ = _sort(lsb_built, a, P, chunks)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    ref, last0, _ = _sort(lsb_built, a, P, 0)
    assert np.array_equal(out, ref)
    assert last == last0  # 8 local passes, 4 exchanges either way


@pytest.mark.parametrize("gather", [0, 1])
def test_every_exchange_placed_or_gathered(lsb_built, oracle_mod, gather):
    """LSB_OPT_EXCHANGE_GATHER = 0: every exchange places (into the low-byte
    pass's buffer, once every chunk pass has read it)."""
    n, P = 4 * (1 << 18) + 99, 4
    a = _uniform(n, 7 + gather)
    out, _, _ = _sort(lsb_built, a, P, 8, gather=gather)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


def test_golden_digests(lsb_built, oracle_mod, digests):
    """The reference binary's own output for (n, P) at every golden row whose
    blocks are large enough to be cut (per >= 2^16)."""
    done = 0
    for d in digests["rows"]:
        if d["P"] == 1 or -(-d["n"] // d["P"]) < (1 << 16):
            continue
        with lsb_built.World(d["n"], ranks=d["P"], radix_bits=16) as w:
            w.set_option(lsb_built.OPT_EXCHANGE_CHUNKS, 8)
            w.generate()
            w.my_sort()
            assert oracle_mod.digest(w.gather_global()) == d["output"], d
        done += 1
    assert done >= 2


@pytest.mark.parametrize("P", [2, 8])
def test_zipf_chunks_of_any_size(lsb_built, oracle_mod, P):
    """Skewed keys: chunks (low-byte ranges) of very different sizes, hot
    digits in one chunk; stable order of the duplicates across ranks."""
    from test_gpu_sort import _dist
    n = P * (1 << 17) + 5
    a = _dist("zipf", n, np.random.default_rng(11 * P))
    out, _, _ = _sort(lsb_built, a, P, 8)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


def test_constant_bytes_fall_back(lsb_built, oracle_mod):
    """A digit with a constant byte takes the unchunked exchange; the others
    are cut.  Bit-exact either way."""
    n, P = 4 * (1 << 17), 4
    a = _uniform(n, 3)
    a["key"] &= ~np.uint64(0x00FF0000FF000000)  # byte 3 (digit 1's high) and byte 6 (digit 3's low) constant
    out, last, _ = _sort(lsb_built, a, P, 4)
    assert np.array_equal(out, oracle_mod.stable_sort(a))


def test_world_of_one_rccl_every_record_through_the_collective(lsb_built, oracle_mod):
    """The x16 extra's form: one RCCL rank, the exchange forced, the self
    segment through ncclAllToAllv chunk by chunk (LSB_OPT_EXCHANGE_SELF)."""
    L = lsb_built
    n = (1 << 20) + 3
    for self_coll in (0, 1):
        w = L.World.rank(n, 1, 0, 0, L.get_unique_id(), radix_bits=16)
        try:
            w.set_option(L.OPT_FORCE_EXCHANGE, 1)
            w.set_option(L.OPT_EXCHANGE_SELF, self_coll)
            w.set_option(L.OPT_EXCHANGE_CHUNKS, 8)
            w.generate()
            inp = w.copy_out(0)
            w.my_sort()
            w.sync()
            assert np.array_equal(w.copy_out(0), oracle_mod.stable_sort(inp))
            assert w.verify() == (True, -1)
            calls, nbytes, _ = w.exchange_bytes()
            if self_coll:
                assert nbytes == 4 * n * 16  # every record, every exchange
        finally:
            w.close()


@pytest.mark.parametrize("world,extra,exchange", [(2, {}, "alltoallv"), (4, {}, "alltoallv"), (8, {}, "alltoallv"),
                                                  (2, {"LSB_RCCL_CALL_U64": "4096"}, "alltoallv"),
                                                  (4, {}, "p2p")])
def test_real_rccl_ranks(lsb_built, world, extra, exchange):
    """Real RCCL ranks (one process each, socket transport on the one GPU,
    tools/rccl_two_ranks.py) with LSB_EXCHANGE_CHUNKS=8: the golden digest
    and every rank verified; with a small call bound the chunks' calls are
    cut too; grouped ncclSend / ncclRecv (LSB_OPT_EXCHANGE_P2P) on the wire
    stream as well."""
    import json
    n = {2: 1_000_000, 4: 1_000_003, 8: 1_048_576}[world]
    env = dict(os.environ, LSB_EXCHANGE_CHUNKS="8", **extra)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "rccl_two_ranks.py"), "16", str(n),
                        str(world), exchange, "0"], capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=env)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert lines, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}"
    r = json.loads(lines[-1])
    assert r["status"] == "ok" and r["golden_match"] is True, r
    assert all(r["verify"]) and all(r["check_sorted"]), r
    assert p.returncode == 0


def test_stats_file_the_chunk_passes_under_the_high_byte(lsb_built, oracle_mod):
    """Per-pass stats: the chunk passes are the high-byte pass's launches (C
    each), and the count read is the digit's upsweep."""
    n, P = 2 * (1 << 18), 2
    a = _uniform(n, 5)
    out, _, ks = _sort(lsb_built, a, P, 4, stats=True)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    assert ks["scatter"][0] == P * 4 * (1 + 4)  # per digit: the low pass + 4 chunk passes, on each rank


def test_skewed_split_stage_chunks(lsb_built, oracle_mod):
    """Keys whose low bytes are skewed take the split stage (3 workgroups per
    CU) in the chunk passes too; hot digits make one chunk hold most of the
    block.  Bit-exact, forced split and auto."""
    from test_gpu_sort import _dist
    n, P = 4 * (1 << 17) + 3, 4
    a = _dist("hot_bucket", n, np.random.default_rng(99))
    for split in (0, 2):
        with lsb_built.World(n, ranks=P, radix_bits=16) as w:
            w.set_option(lsb_built.OPT_EXCHANGE_CHUNKS, 8)
            w.set_option(lsb_built.OPT_ONESWEEP_SPLIT, split)
            w.scatter_global(a)
            w.my_sort()
            assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(a)), split


def test_failed_chunk_pass_then_sort(lsb_built, oracle_mod):
    """A chunk pass that fails to launch (LSB_OPT_FAIL_ONESWEEP) after earlier
    chunks' transfers were queued on the wire streams: lsb_sort waits for
    every rank's streams before it reports the error (quiesce), A still holds
    a permutation of the records (the low-byte pass's output), and the next
    sort on the same context sorts it exactly."""
    L = lsb_built
    n, P = 4 * (1 << 17) + 3, 4
    with L.World(n, ranks=P, radix_bits=16) as w:
        w.set_option(L.OPT_EXCHANGE_CHUNKS, 8)
        w.generate()
        inp = w.gather_global()
        # 4 low-byte passes (one per rank), then chunk passes rank by rank:
        # the 14th launch is chunk 2 of rank 1, after chunks 0 and 1 went out.
        w.set_option(L.OPT_FAIL_ONESWEEP, 14)
        with pytest.raises(L.LsbError):
            w.my_sort()
        w.set_option(L.OPT_FAIL_ONESWEEP, 0)
        held = w.gather_global()
        assert np.array_equal(np.sort(held, order=["key", "val"]), np.sort(inp, order=["key", "val"]))
        w.my_sort()
        assert np.array_equal(w.gather_global(), oracle_mod.stable_sort(held))
        assert w.verify() == (True, -1)
        assert w.check_sorted()


@pytest.mark.parametrize("n,P,chunks", [(4 * 65536, 4, 8),          # per = 2^16 exactly: chunked
                                        (4 * 65536 - 4, 4, 8),      # per just below: unchunked
                                        (3 * 65536 + 1, 3, 4),      # ragged: the last rank is 2 short
                                        (8 * 70000 + 7, 8, 2)])
def test_block_sizes_at_the_threshold(lsb_built, oracle_mod, n, P, chunks):
    """Blocks at the chunking threshold (kChunkMinPer = 2^16 records per
    rank) and ragged last ranks: bit-exact either way, same local passes and
    exchanges as the unchunked sort."""
    a = _uniform(n, n + P)
    out, last, _ = _sort(lsb_built, a, P, chunks)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    _, last0, _ = _sort(lsb_built, a, P, 0)
    assert last == last0


@pytest.mark.parametrize("form", ["first", "ends", "middle"])
def test_empty_chunks(lsb_built, oracle_mod, form):
    """The low byte of every digit limited so that at C = 8 (32 values per
    chunk) most chunks are empty on every rank (no pass, empty transfers):
    only chunk 0 ("first"), chunks 0 and 7 ("ends"), chunks 2 and 3
    ("middle")."""
    n, P = 4 * (1 << 17) + 11, 4
    a = _uniform(n, 40 + len(form))
    rng = np.random.default_rng(len(form))
    pool = {"first": np.arange(0, 32), "ends": np.array([0, 1, 254, 255]), "middle": np.arange(64, 128)}[form]
    for d in range(4):
        sh = np.uint64(16 * d)
        lo = pool[rng.integers(0, pool.size, n)].astype(np.uint64)
        a["key"] = (a["key"] & ~(np.uint64(0xFF) << sh)) | (lo << sh)
    out, _, _ = _sort(lsb_built, a, P, 8)
    assert np.array_equal(out, oracle_mod.stable_sort(a))
