#!/bin/bash
# C2 LDS-search probes: staging only (ab/sl_p1.so), search without staging
# (ab/sl_p2.so), and the in-tree kernel, each under a kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r06/c2probe; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in in sl_p1 sl_p2; do
  if [ $v = in ]; then L=$R/p2p-dhts_amd/chordx/libchordx.so; else L=$R/ab/$v.so; fi
  CHORDX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $R/benches/bench_c2.py 4 --rounds 2 > $O/$v.log 2>&1 || exit 1
  echo "$v: $(find $O/$v -name '*kernel_stats.csv' -exec grep successor_lds {} \; | cut -d, -f1-4)"
done
