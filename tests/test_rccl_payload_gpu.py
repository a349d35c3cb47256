"""The element exchange carried by RCCL itself, on the one GPU we have.

A world of one normally exchanges nothing: the rank's own segment is placed
straight out of A, so every ncclAllToAllv of the suite would move zero bytes.
LSB_OPT_EXCHANGE_SELF sends that segment through the collective too
(ncclAllToAllv, or grouped ncclSend/ncclRecv to itself) with the production
slice displacements, and places it from the receive buffer like any other
source.  So these tests execute the reference's payload exchange
(mpi/mpi_lsbsort.cpp:316-324, :563) through RCCL with every record on the
wire: the per-digit forms (8- and 16-bit exchange digits, one all-to-all per
digit) and the whole-key form (8 splitter-search all-gathers, one sliced
all-to-all, merge).  The library counts the payload it hands to the
collective (lsb_get_exchange_bytes); the output must match the reference's
golden digest for (n = 2^20, P = 1) and the on-device verify.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _world(lsb, n, bits, p2p, slices):
    w = lsb.World.rank(n, 1, 0, 0, lsb.get_unique_id(), radix_bits=bits)
    w.set_option(lsb.OPT_FORCE_EXCHANGE, 1)
    w.set_option(lsb.OPT_EXCHANGE_SELF, 1)
    w.set_option(lsb.OPT_EXCHANGE_P2P, p2p)
    w.set_option(lsb.OPT_EXCHANGE_SLICES, slices)
    return w


@pytest.mark.parametrize("slices", [1, 8])
@pytest.mark.parametrize("p2p", [0, 1])
@pytest.mark.parametrize("bits", [8, 16, 64])
def test_payload_through_rccl_golden(lsb_built, oracle_mod, digests, bits, p2p, slices):
    d = next(r for r in digests["rows"] if r["P"] == 1)  # n = 2^20, P = 1
    n = d["n"]
    w = _world(lsb_built, n, bits, p2p, slices)
    try:
        w.generate()
        w.barrier()
        calls0, bytes0, _ = w.exchange_bytes()
        w.my_sort()
        w.barrier()
        calls, nbytes, biggest = w.exchange_bytes()
        _, exchanges, _ = w.last_sort()
        assert exchanges == (1 if bits == 64 else 64 // bits)
        # every record crosses the collective once per exchange, in `slices` calls
        assert calls - calls0 == exchanges * slices
        assert nbytes - bytes0 == exchanges * n * 16
        assert biggest >= MIB
        assert oracle_mod.digest(w.copy_out(0)) == d["output"]
        assert w.verify() == (True, -1)
        assert w.check_sorted()
    finally:
        w.close()


@pytest.mark.parametrize("bits", [16, 64])
def test_payload_through_rccl_large(lsb_built, bits):
    """2^27 records (2 GiB per all-to-all), all of them through RCCL."""
    n = 1 << 27
    w = _world(lsb_built, n, bits, 0, 4 if bits == 16 else 8)
    try:
        w.generate()
        w.barrier()
        w.my_sort()
        w.barrier()
        calls, nbytes, biggest = w.exchange_bytes()
        _, exchanges, _ = w.last_sort()
        assert nbytes == exchanges * n * 16
        assert biggest >= 256 * MIB
        assert w.verify() == (True, -1)
        assert w.check_sorted()
    finally:
        w.close()


def test_payload_through_rccl_skewed_keys(lsb_built, oracle_mod):
    """Tied keys through the whole-key form with the self range on the wire:
    the splitter cut among equal keys must keep rank (input) order."""
    n = 300_007
    rng = np.random.default_rng(5)
    a = np.zeros(n, dtype=lsb_built.ELEM_DTYPE)
    a["key"] = rng.integers(0, 7, n, dtype=np.uint64) << np.uint64(40)
    a["val"] = np.arange(n, dtype=np.uint64)
    for bits in (16, 64):
        w = _world(lsb_built, n, bits, 1, 3)
        try:
            w.copy_in(0, a)
            w.my_sort()
            w.barrier()
            assert np.array_equal(w.copy_out(0), oracle_mod.stable_sort(a))
            assert w.exchange_bytes()[1] > 0
        finally:
            w.close()


def test_loaded_library_matches_tree(lsb_built):
    """The library this run loaded was built from the sources in this tree
    (its compiled-in digest equals the digest of the files here)."""
    info = lsb_built.build_info()
    assert info["sha256"] == lsb_built.source_digest(), info
