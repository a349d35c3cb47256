"""The N > 1 path with real processes on CPU (world size 2, gloo).

Each rank runs the runtime's per-pass protocol (lsb_runtime.cpp
exchange_rccl) with gloo standing in for RCCL and the oracle's local pass
standing in for the device kernels:
  local stable pass -> all-gather of bucket counts -> lsb_plan_exchange
  (the product's host planner) -> point-to-point send/recv of 16-byte
  records (RCCL grouped ncclSend/ncclRecv) -> placement by place_off.
The gathered result must equal the reference's golden digest for
`mpirun -n 2 mpi_lsbsort --n 1000000`.  bench.py's rank helper (unique-id
broadcast, max-reduction of step times) is exercised in the same processes.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, result_dir):
    for p in (ROOT, os.path.join(ROOT, "distributed-lsb_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist
    import lsbsort
    import oracle
    import bench

    d = bench.Dist()  # init_process_group("gloo") from the environment, as bench.py does
    assert d.world == world and d.rank == rank
    uid = d.bcast_bytes(b"x" * 128 if rank == 0 else None)
    assert uid == b"x" * 128
    assert d.max(float(rank + 1)) == float(world)

    per = lsbsort.per_rank(n, world)
    here = lsbsort.here(n, world, rank)
    slots = oracle.generate_slots(n, world)
    A = slots[rank * per: rank * per + here].copy()  # == lsb_generate on this rank
    for digit in range(8):
        B, h = oracle.local_pass(A, 8, digit)  # stands in for k_upsweep/k_scan/k_scatter
        gathered = [torch.zeros(256, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(h.astype(np.int64)))  # ncclAllGather
        hist = torch.stack(gathered).numpy()
        plan = lsbsort.plan_exchange(n, world, rank, hist)
        R = np.empty(here, dtype=oracle.ELEM_DTYPE)
        reqs = []
        for q in range(world):
            sc, so = int(plan["send_counts"][q]), int(plan["send_displs"][q])
            rc, ro = int(plan["recv_counts"][q]), int(plan["recv_displs"][q])
            if q == rank:
                assert sc == rc
                R[ro:ro + rc] = B[so:so + sc]
                continue
            if sc:
                buf = torch.from_numpy(B[so:so + sc].view(np.uint64).copy())
                reqs.append(dist.isend(buf, q))
            if rc:
                rbuf = torch.empty(2 * rc, dtype=torch.uint64)
                reqs.append((dist.irecv(rbuf, q), rbuf, ro, rc))
        for r in reqs:
            if isinstance(r, tuple):
                r[0].wait()
                R[r[2]:r[2] + r[3]] = r[1].numpy().view(oracle.ELEM_DTYPE)
            else:
                r.wait()
        # k_place: recv index k from source s (first s with k < rend[s]) -> place_off[s][digit] + k
        rend = np.cumsum(plan["recv_counts"])
        src = np.searchsorted(rend, np.arange(here), side="right")
        dig = ((R["key"] >> np.uint64(8 * digit)) & np.uint64(255)).astype(np.int64)
        dst = plan["place_off"][src, dig] + np.arange(here)
        A = np.empty_like(R)
        A[dst] = R
    np.save(os.path.join(result_dir, f"rank{rank}.npy"), A)
    d.close()


def test_world_size_2_reproduces_reference_digest(tmp_path, digests, oracle_mod):
    import torch.multiprocessing as mp
    row = next(r for r in digests["rows"] if r["P"] == 2)
    n, world = row["n"], 2
    mp.start_processes(_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    out = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    assert oracle_mod.digest(out) == row["output"]
