"""The peer-store exchange's release / acquire, read from the shipped code object.

The reference's one-sided exchange completes its puts before the barrier
(`shmem_putmem` then `shmem_barrier_all`, /root/reference/shmem/
shmem_lsbsort.cpp:441-456; `MPI_Put` between fences,
/root/reference/mpi/mpi_lsbsort_onesided.cpp:487-509).  Here that is
`k_peer_scatter`'s end (csrc/lsb_kernels.hip) and `k_system_acquire`: a
one-GPU box cannot show a missing cross-device fence by running, so this test
disassembles the gfx950 code object inside build/liblsb.so (CPU only) and
checks the order of the instructions that provide it:

* k_peer_scatter: after its last global store, every wave waits for its
  stores (s_waitcnt vmcnt(0)) before the workgroup barrier; after the
  barrier comes a system-scope L2 writeback (buffer_wbl2 sc0 sc1), and
  nothing after it but the kernel's end (and a wait, if the compiler keeps
  one there);
* k_system_acquire: a system-scope L2 invalidate (buffer_inv sc0 sc1).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed-lsb_amd", "build", "liblsb.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


@pytest.fixture(scope="module")
def disasm(lsb_built, tmp_path_factory):
    tools = {t: _tool(t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")}
    missing = [t for t, p in tools.items() if not p]
    if missing:
        pytest.skip(f"LLVM tools absent: {missing}")
    d = tmp_path_factory.mktemp("peer_fence")
    fb = d / "fatbin.bin"
    subprocess.run([tools["llvm-objcopy"], f"--dump-section=.hip_fatbin={fb}", LIB], check=True)
    blob = fb.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    assert starts, "no offload bundle in liblsb.so's .hip_fatbin"
    text = []
    for k, s in enumerate(starts):  # one bundle per .hip translation unit
        e = starts[k + 1] if k + 1 < len(starts) else len(blob)
        part = d / f"bundle{k}.bin"
        part.write_bytes(blob[s:e])
        co = d / f"bundle{k}.co"
        subprocess.run([tools["clang-offload-bundler"], "--unbundle", "--type=o", f"--input={part}",
                        f"--targets={TARGET}", f"--output={co}"], check=True)
        out = subprocess.run([tools["llvm-objdump"], "-d", "--no-show-raw-insn", str(co)], check=True,
                             capture_output=True, text=True).stdout
        text.append(out)
    return "\n".join(text)


def _functions(disasm, needle):
    """Instruction lists (comments stripped) of every function whose symbol contains needle."""
    funcs, cur = [], None
    for line in disasm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = [] if needle in m.group(1) else None
            if cur is not None:
                funcs.append(cur)
            continue
        if not line.startswith("\t"):  # instructions are indented; anything else ends a function
            cur = None
        if cur is not None:
            ins = line.split("//")[0].strip()
            if ins and ins != "...":
                cur.append(ins)
    return funcs


def test_peer_scatter_waits_for_every_wave_then_writes_back(disasm):
    funcs = _functions(disasm, "k_peer_scatter")
    assert len(funcs) == 2, "both k_peer_scatter instances (offset row in LDS or not)"
    for ins in funcs:
        last_store = max(i for i, x in enumerate(ins) if re.match(r"(global|flat|buffer)_store", x))
        barriers = [i for i, x in enumerate(ins) if x == "s_barrier" and i > last_store]
        assert barriers, "a workgroup barrier after the last store"
        bar = barriers[-1]
        waits = [i for i in range(last_store + 1, bar) if ins[i] == "s_waitcnt vmcnt(0)"]
        assert waits, "every wave waits for its own stores (vmcnt(0)) before the barrier:\n" + \
            "\n".join(ins[last_store:bar + 1])
        tail = ins[bar + 1:]
        wb = [i for i, x in enumerate(tail) if x == "buffer_wbl2 sc0 sc1"]
        assert wb, "a system-scope L2 writeback after the barrier"
        after = tail[wb[0] + 1:]
        # Nothing but a wait may follow the writeback: the compiler drops a
        # wait directly before s_endpgm, since the kernel's completion waits
        # for the wave's outstanding memory operations anyway.
        assert after and after[-1] == "s_endpgm" and set(after[:-1]) <= {"s_waitcnt vmcnt(0)"}, \
            "the writeback ends the kernel: " + "\n".join(after)


def test_system_acquire_invalidates(disasm):
    funcs = _functions(disasm, "k_system_acquire")
    assert len(funcs) == 1
    assert "buffer_inv sc0 sc1" in funcs[0]
