"""The one-rank-per-process runtime with real processes on the GPU.

lsb_create_rank_ops runs exactly the per-rank code of the RCCL contexts
(lsb_create_rank): the device plan, the sliced all-to-all with placement
overlapped on a second stream, the key-span all-gather and digit skipping,
the cross-rank verify and checkSorted.  Only the collectives differ: here
they are gloo calls from host callbacks instead of RCCL calls.  RCCL itself
refuses two ranks on one GPU, so this is how the multi-process protocol is
tested on a one-GPU box: P processes share the GPU, each owns one rank.
The gathered output must match the reference's golden digest
(`mpirun -n P mpi_lsbsort --n N`) or the oracle's stable sort.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case, result_dir):
    for p in (ROOT, os.path.join(ROOT, "distributed-lsb_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import lsbsort
    from bench import GlooComm  # lsb_comm_ops_t over gloo (bench.py --transport gloo)

    os.environ.update(case.get("env", {}))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, bits, slices, mask = case["n"], case["bits"], case["slices"], case["mask"]
    w = lsbsort.World.rank_ops(n, world, rank, 0, GlooComm(dist, world, rank), radix_bits=bits)
    w.set_option(lsbsort.OPT_EXCHANGE_SLICES, slices)
    w.set_option(lsbsort.OPT_EXCHANGE_PEER, int(case.get("peer", 0)))
    if mask is None:
        w.generate()  # pcg64(rank), as mpi_lsbsort.cpp:650-656
    else:
        a = np.load(os.path.join(result_dir, "input.npy"))
        per, here = lsbsort.per_rank(n, world), lsbsort.here(n, world, rank)
        w.copy_in(rank, a[rank * per: rank * per + here], 0)
    w.barrier()
    w.my_sort()
    w.barrier()
    out = w.copy_out(rank)
    ok, bad = w.verify() if mask is None else (None, None)
    sorted_ = w.check_sorted()
    np.save(os.path.join(result_dir, f"rank{rank}.npy"), out)
    np.save(os.path.join(result_dir, f"meta{rank}.npy"),
            np.array([ok is not False, bad if bad is not None else -1, sorted_,
                      *w.last_sort()[:2]], dtype=np.int64))
    w.close()
    dist.destroy_process_group()


def _run(tmp_path, world, case):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    out = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    meta = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    return out, meta


@pytest.mark.parametrize("world,bits,slices", [(2, 8, 4), (2, 16, 3), (4, 16, 1), (4, 8, 7),
                                               (2, 64, 1), (4, 64, 1), (4, 64, 8)])
def test_processes_reproduce_reference_digest(tmp_path, digests, oracle_mod, world, bits, slices):
    row = next(r for r in digests["rows"] if r["P"] == world)
    case = dict(n=row["n"], bits=bits, slices=slices, mask=None)
    out, meta = _run(tmp_path, world, case)
    assert oracle_mod.digest(out) == row["output"]
    for m in meta:
        assert m[0] == 1 and m[1] == -1 and m[2] == 1  # verify ok on every rank, checkSorted
        assert m[4] == 64 // bits                       # one exchange per digit


@pytest.mark.parametrize("world,bits,vmm_mib", [(2, 8, 0), (4, 16, 0), (2, 16, 2), (4, 8, 2)])
def test_processes_peer_store_exchange(tmp_path, digests, oracle_mod, world, bits, vmm_mib):
    """Peer stores through IPC-mapped buffers of the other processes.  With
    vmm_mib, the record buffers start as VMM pieces of that many MiB, which
    IPC handles cannot name: the exchange's setup moves them into hipMalloc
    buffers first (peer_setup), records and all."""
    row = next(r for r in digests["rows"] if r["P"] == world)
    env = {"LSB_VMM_CHUNK_MIB": str(vmm_mib)} if vmm_mib else {}
    out, meta = _run(tmp_path, world, dict(n=row["n"], bits=bits, slices=4, mask=None, peer=1, env=env))
    assert oracle_mod.digest(out) == row["output"]
    for m in meta:
        assert m[0] == 1 and m[1] == -1 and m[2] == 1


@pytest.mark.parametrize("world,bits,mask,passes,exchanges", [
    (2, 8, 0x00000000FFFFFFFF, 4, 4),
    (3, 16, 0x00FF0000000000FF, 2, 2),   # digits 0 and 3, each its low byte only; 1, 2 skipped
    (3, 64, 0x00FF0000000000FF, 2, 1),   # whole-key exchange: local passes on bytes 0 and 6
])
def test_processes_skip_constant_digits(tmp_path, oracle_mod, world, bits, mask, passes, exchanges):
    n = 300_007
    rng = np.random.default_rng(world * 100 + bits)
    a = np.zeros(n, dtype=oracle_mod.ELEM_DTYPE)
    a["key"] = rng.integers(0, 2**64 - 1, n, dtype=np.uint64) & np.uint64(mask)
    a["val"] = np.arange(n, dtype=np.uint64)
    np.save(tmp_path / "input.npy", a)
    out, meta = _run(tmp_path, world, dict(n=n, bits=bits, slices=4, mask=mask))
    assert np.array_equal(out, oracle_mod.stable_sort(a))
    for m in meta:
        assert m[2] == 1 and (m[3], m[4]) == (passes, exchanges)
