#!/bin/bash
# C2 LDS search launch shapes (kernel trace each, two alternating rounds):
# in-tree (256 blocks of 1024 lanes x 4 keys), ab/sl_half.so (128 blocks, two
# trips), ab/sl_b512.so (512-lane blocks x 8 keys).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r06/c2shape; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for i in 1 2; do
  for v in in sl_half sl_b512; do
    L=$R/ab/$v.so; [ $v = in ] && L=$R/p2p-dhts_amd/chordx/libchordx.so
    CHORDX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_$i -o run --output-format csv -- python3 $R/benches/bench_c2.py 4 --rounds 2 > $O/${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(find $O/${v}_$i -name '*kernel_stats.csv' -exec grep successor_lds {} \; | cut -d, -f3-6) $(grep -o '"identical": [a-z]*' $O/${v}_$i.log)"
  done
done
