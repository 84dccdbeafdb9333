#!/bin/bash
# C2 LDS search with int16 offset deviations and b = log2 n - 3 (in-tree)
# against the uint32 offsets at b = log2 n - 4 (ab/c2_b12.so): successor /
# predecessor tests, then kernel traces in two alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r06/c2d16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "successor or predecessor" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for i in 1 2; do
  for v in in c2_b12; do
    L=$R/ab/$v.so; [ $v = in ] && L=$R/p2p-dhts_amd/chordx/libchordx.so
    CHORDX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_$i -o run --output-format csv -- python3 $R/benches/bench_c2.py 4 --rounds 2 > $O/${v}_$i.log 2>&1 || exit 1
  done
done
