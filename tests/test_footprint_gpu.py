"""lsb_rank_footprint against the device's own count of free memory.

The model (csrc/lsb_abi.cpp) restates init_rank's and the sort's
allocations; this test creates a context, runs one sort (which allocates the
look-back rows, and R for an exchange or the hybrid), and compares the drop
in hipMemGetInfo's free bytes with the model.  Allocation granularity and the
runtime's own bookkeeping make the two differ by a few MiB, not more."""
import pytest

MiB = 1 << 20


@pytest.mark.gpu
@pytest.mark.parametrize("n,P,bits,hybrid", [(1 << 28, 1, 8, 0), (1 << 28, 1, 8, 1), (3 << 27, 2, 16, 0),
                                             ((1 << 30) + 12345, 1, 8, 0)])
def test_footprint_matches_free_memory(lsb_built, n, P, bits, hybrid):
    lsbsort = lsb_built
    free0, total = lsbsort.device_memory(0)
    w = lsbsort.World(n, ranks=P, radix_bits=bits)
    try:
        w.set_option(lsbsort.OPT_HYBRID, hybrid)
        w.generate()
        w.my_sort()
        w.sync()
        free1, _ = lsbsort.device_memory(0)
    finally:
        w.close()
    used = free0 - free1
    model = P * lsbsort.rank_footprint(n, P, bits, with_recv=P > 1 or hybrid == 1)["bytes"]
    assert abs(used - model) <= 64 * MiB + 0.002 * model, (used, model)
    free2, _ = lsbsort.device_memory(0)
    assert free0 - free2 <= 64 * MiB  # everything given back at close
