#!/bin/bash
# C2 successor kernel A/B (round 5): kernel-only times of the in-tree library
# and the ab/ variants under rocprofv3 --kernel-trace --stats, alternating.
#   bash tools/r05_c2_ab.sh <tag> lib1.so lib2.so ...
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/${1:-r05_c2_ab}
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/A_$round -o run --output-format csv \
    -- python3 $R/benches/bench_c2.py > $O/A_$round.json 2> $O/A_$round.err
  for L in "$@"; do
    b=$(basename $L .so)
    CHORDX_LIB=$R/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${b}_$round -o run \
      --output-format csv -- python3 $R/benches/bench_c2.py > $O/${b}_$round.json 2> $O/${b}_$round.err
  done
done
for f in $(find $O -name "run_kernel_stats.csv" | sort); do
  echo "$f $(grep -E 'k_successor' $f | cut -d, -f1-4 | head -2 | tr '\n' ' ')"
done
