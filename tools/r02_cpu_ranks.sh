#!/bin/bash
# The reference MPI sort on the GPU box at several rank counts, n = 2^26:
# the job's CPU share (cgroup quota) against all physical cores.  Shows why
# bench.py's CPU baseline uses one rank per core of the job's share.
set -o pipefail
O=gpurun_out/cpuranks
mkdir -p $O
M=$(command -v mpirun || echo /opt/conda/bin/mpirun)
{ echo "nproc=$(nproc) physical=$(lscpu -p=CORE,SOCKET | grep -v '^#' | sort -u | wc -l) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null) OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > $O/log
for r in 8 16 32 128; do
  echo "== ranks $r" >> $O/log
  timeout -k 10 150 $M -n $r oracle/_ref/mpi_lsbsort --n 67108864 --no-verify >> $O/log 2>&1 || echo "ranks $r: rc=$?" >> $O/log
done
grep -E 'nproc|==|sorted / s|rc=' $O/log
