#!/bin/bash
# C2 LDS search with streaming key loads / owner stores (ab/sl_nt.so) against
# the in-tree kernel: kernel traces, two alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r06/c2nt; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for i in 1 2; do
  for v in in sl_nt; do
    L=$R/ab/$v.so; [ $v = in ] && L=$R/p2p-dhts_amd/chordx/libchordx.so
    CHORDX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_$i -o run --output-format csv -- python3 $R/benches/bench_c2.py 4 --rounds 2 > $O/${v}_$i.log 2>&1 || exit 1
  done
done
