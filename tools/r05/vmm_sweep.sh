#!/bin/bash
# allocator modes of tools/kbench/vmmbw.hip, each in fresh
# processes (output: gpurun_out/r05_vmm/).
set -e
out=gpurun_out/r05_vmm
mkdir -p $out
run() {  # name mode chunk_mib
  timeout -k 10 120 tools/kbench/vmmbw $2 4 30 5 $3 > $out/$1.log 2>&1
  grep SUMMARY $out/$1.log
}
for i in 1 2 3; do run m0_$i 0 0; done
for i in 1 2 3; do run m1_$i 1 0; done
for i in 1 2; do run m2_1g_$i 2 1024; done
for i in 1 2; do run m3_rec_$i 3 0; done
for i in 1 2; do run m5_rec_$i 5 0; done
run m4_rec_1 4 0
run m3_64m_1 3 64
