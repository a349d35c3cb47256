#!/usr/bin/env python3
"""Randomised stress of every sort form on one GPU: each iteration draws a
size (1 .. 2^27 records, log-uniform, ragged), a rank count (P logical ranks,
device-copy exchange), an exchange digit width (8, 16 or 64) and whether its
exchanges gather (LSB_OPT_EXCHANGE_GATHER), a key
distribution, a stage form and a local-sort form (LSD or the hybrid's two
modes), sorts, and checks lsb_verify and checkSorted.  One iteration in
three instead sorts host-made keys (up to 2^22 records) whose bytes are
thinned out at random -- constant bytes, few distinct values in the middle
bytes, duplicates -- the inputs that take the hybrid's fallbacks and
k_segfix's long crossing runs; those are checked against numpy's stable
argsort.  Record buffers come from VMM pieces of a drawn size (2 MiB,
64 MiB or the default 1 GiB), so small sorts run the VMM allocator too.  The
regional first pass (LSB_OPT_REGION_FIRST) starts at a drawn size (2^16
records or the default 2^27), and some host-made keys crowd one digit-0
bucket of one sub-array (the regions the sample may miss, so some sorts
overflow one and start over); each line names how the sort began.  One
draw in three sets LSB_PLACEMENT_CANDIDATES=4 (the placement probe for the
P = 1 buffers of >= 1 GiB, built from the drawn pieces), the others 0; and
three draws in five send 16-bit exchanges in 2, 4 or 8 chunks
(LSB_OPT_EXCHANGE_CHUNKS, blocks of >= 2^16 records).  --rccl-share runs a
share of the iterations as world-of-one RCCL contexts instead (every record
through ncclAllToAllv; the context kind where RCCL over reused VMM addresses
went wrong).  Runs until --seconds have passed; one line per
iteration.

    python tools/stress_mix.py --seconds 240 --seed 1
"""
import argparse
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-lsb_amd"))
import lsbsort  # noqa: E402
import numpy as np  # noqa: E402

DT = np.dtype([("key", "<u8"), ("val", "<u8")])


def thinned_keys(rng, n):
    """Uniform keys with random structure: each byte kept, made constant, or
    drawn from a small pool; sometimes whole keys from a small pool."""
    g = np.random.default_rng(rng.randrange(1 << 30))
    k = g.integers(0, 2**64 - 1, n, dtype=np.uint64)
    for b in range(8):
        r = rng.random()
        sh = np.uint64(8 * b)
        if r < 0.25:  # constant byte
            k = (k & ~(np.uint64(0xFF) << sh)) | (np.uint64(rng.randrange(256)) << sh)
        elif r < 0.45:  # few values
            pool = g.integers(0, 256, rng.choice((2, 4, 16)), dtype=np.uint64)
            k = (k & ~(np.uint64(0xFF) << sh)) | (pool[g.integers(0, pool.size, n)] << sh)
    if rng.random() < 0.2:  # duplicates: ~2 .. ~1024 copies of each key
        k = k[g.integers(0, max(1, n // rng.choice((2, 8, 64, 256, 1024))), n)]
    a = np.zeros(n, dtype=DT)
    a["key"] = k
    a["val"] = np.arange(n, dtype=np.uint64)
    return a


def crowded_keys(rng, n):
    """Uniform keys, except that a random share (up to 1/4) of one sub-array's
    records get one digit-0 value: a region of the regional first pass that
    can overflow where the sample does not look."""
    g = np.random.default_rng(rng.randrange(1 << 30))
    a = np.zeros(n, dtype=DT)
    a["key"] = g.integers(0, 2**64 - 1, n, dtype=np.uint64)
    a["val"] = np.arange(n, dtype=np.uint64)
    x = rng.randrange(8)
    lo, hi = x * n // 8, (x + 1) * n // 8
    pick = lo + np.flatnonzero(g.random(hi - lo) < rng.uniform(0, 0.25))
    a["key"][pick] = (a["key"][pick] & ~np.uint64(0xFF)) | np.uint64(rng.randrange(256))
    return a


def draw(rng, max_log2, draws="current", host_share=1 / 3, force_hybrid=None):
    """One iteration's configuration, drawn in a fixed order (tools/stress_replay.py
    replays the sequence without sorting).  draws: "current", or an earlier
    round's sequence -- "r05v12" (round 5's run v12: no probe and no chunk
    draws), "r05" (no chunk draw).  Host-made keys are drawn afterwards by
    host_keys, from the same rng."""
    n = int(2 ** rng.uniform(0, max_log2)) + rng.randrange(0, 4096)
    P = rng.choice((1, 1, 2, 3, 8))
    bits = rng.choice((8, 16, 64))
    dist = rng.choice(("uniform", "zipf"))
    split = rng.choice((0, 1, 2))
    hybrid = rng.choice((0, 1, 1, 2))
    gather = rng.choice((0, 1, 1))  # LSB_OPT_EXCHANGE_GATHER (per-digit exchange forms)
    if force_hybrid is not None:
        hybrid = force_hybrid
    host = rng.random() < host_share
    if host:
        n = min(n, 1 << 22)
        dist = "crowded" if rng.random() < 0.25 else "thinned"
    region_min = rng.choice((1 << 16, 1 << 27))
    # record buffers from VMM pieces of 2 / 64 MiB (several pieces per
    # buffer at these sizes), or the default 1 GiB (hipMalloc below it)
    vmm = rng.choice((2, 64, 1024, 1024))
    # the placement probe: off, or 4 candidates (K set: buffers of >= 1 GiB)
    probe = rng.choice((0, 0, 4)) if draws != "r05v12" else 0
    # the exchange in chunks (LSB_OPT_EXCHANGE_CHUNKS; 16-bit exchanges of
    # blocks of >= 2^16 records)
    chunks = rng.choice((0, 0, 2, 4, 8)) if draws == "current" else 0
    return dict(n=n, P=P, bits=bits, dist=dist, split=split, hybrid=hybrid, gather=gather, host=host,
                region_min=region_min, vmm=vmm, probe=probe, chunks=chunks)


def host_keys(rng, cfg):
    """The host-made keys of a configuration with cfg["host"]."""
    return crowded_keys(rng, cfg["n"]) if cfg["dist"] == "crowded" else thinned_keys(rng, cfg["n"])


def set_env(cfg):
    """The configuration's environment knobs, read at context creation."""
    os.environ["LSB_REGION_MIN"] = str(cfg["region_min"])
    os.environ["LSB_VMM_CHUNK_MIB"] = str(cfg["vmm"])
    os.environ["LSB_PLACEMENT_CANDIDATES"] = str(cfg["probe"])


def set_options(w, cfg):
    w.set_option(lsbsort.OPT_ONESWEEP_SPLIT, cfg["split"])
    w.set_option(lsbsort.OPT_HYBRID, cfg["hybrid"])
    w.set_option(lsbsort.OPT_EXCHANGE_GATHER, cfg["gather"])
    w.set_option(lsbsort.OPT_EXCHANGE_CHUNKS, cfg["chunks"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-log2", type=int, default=27)
    ap.add_argument("--trace", action="store_true", help="print each configuration before its sort")
    ap.add_argument("--stop-on-error", action="store_true", help="end at the first wrong sort or error")
    ap.add_argument("--host-share", type=float, default=1 / 3,
                    help="share of iterations that sort host-made (thinned / crowded) keys")
    ap.add_argument("--hybrid", type=int, choices=(0, 1, 2), default=None,
                    help="force LSB_OPT_HYBRID instead of drawing it (the draw still happens)")
    ap.add_argument("--draws", choices=("current", "r05", "r05v12"), default="current",
                    help="an earlier round's draws (as tools/stress_replay.py): r05v12 without the probe and "
                         "chunk draws, r05 without the chunk draw")
    ap.add_argument("--iters", type=int, default=0, help="stop after this many sorts (0: --seconds only)")
    ap.add_argument("--rccl-share", type=float, default=0.0,
                    help="share of iterations run as a world-of-one RCCL context (P = 1, exchange forced, every "
                         "record through ncclAllToAllv), drawn from a second generator so the other draws stay "
                         "those of --seed")
    a = ap.parse_args()
    rng = random.Random(a.seed)
    rng_rccl = random.Random(a.seed ^ 0x5EED5EED)
    t_end = time.time() + a.seconds
    it = bad = 0
    while time.time() < t_end and (a.iters <= 0 or it < a.iters):
        cfg = draw(rng, a.max_log2, a.draws, a.host_share, a.hybrid)
        set_env(cfg)
        rccl = rng_rccl.random() < a.rccl_share
        if rccl:
            cfg["P"] = 1
        n, P, bits, dist = cfg["n"], cfg["P"], cfg["bits"], cfg["dist"]
        desc = (f"iter {it}: n={n} P={P} bits={bits} dist={dist} split={cfg['split']} hybrid={cfg['hybrid']} "
                f"gather={cfg['gather']} vmm={cfg['vmm']} region_min={cfg['region_min']} probe={cfg['probe']} "
                f"chunks={cfg['chunks']}" + (" rccl=1" if rccl else ""))
        t0 = time.time()
        if a.trace:  # the configuration before the sort: a fault kills the process mid-sort
            print(f"begin {desc}", flush=True)
        try:
            if rccl:
                w = lsbsort.World.rank(n, 1, 0, 0, lsbsort.get_unique_id(), radix_bits=bits)
                w.set_option(lsbsort.OPT_FORCE_EXCHANGE, 1)
                w.set_option(lsbsort.OPT_EXCHANGE_SELF, 1)
            else:
                w = lsbsort.World(n, ranks=P, radix_bits=bits)
            with w:
                set_options(w, cfg)
                if cfg["host"]:
                    arr = host_keys(rng, cfg)
                    w.scatter_global(arr)
                    w.my_sort()
                    got = w.gather_global()
                    want = arr[np.argsort(arr["key"], kind="stable")]
                    diff = np.nonzero(got != want)[0]
                    ok, first = diff.size == 0, (int(diff[0]) if diff.size else -1)
                else:
                    w.generate(dist)
                    w.my_sort()
                    ok, first = w.verify()
                srt = w.check_sorted()
                form = w.first_pass()
        except lsbsort.LsbError as e:
            ok, first, srt, form = False, str(e), False, -1
        if not (ok and srt):
            bad += 1
            if a.stop_on_error:
                print(f"{desc} first_pass={form} verify={ok} first_bad={first} sorted={srt}", flush=True)
                print(f"done: {bad} of {it + 1} sorts wrong (stopped at the first)", flush=True)
                sys.exit(1)
        print(f"{desc} first_pass={form} verify={ok} first_bad={first} sorted={srt} "
              f"ms={(time.time() - t0) * 1e3:.0f}", flush=True)
        it += 1
    print(f"done: {bad} of {it} sorts wrong", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
