#!/bin/bash
# Route-table build A/B (round 5): in-tree library (A: non-temporal plane
# gathers) against ab/libchordx_ab_planecached.so (B: ordinary plane gathers),
# ABBA order, bench_czbuild (2^24, table_build 0, 3 builds each), then one
# FETCH_SIZE and one WRITE_SIZE pass of k_cz_build_roots2 for each library.
#   bash tools/r05_build_ab.sh <tag>
# (Recorded in profiles/r05/build_ab/ before the switch: cached gathers won and
# are the default since; B is then built with -DCX_AB_PLANE_CACHED=1, a no-op.)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/${1:-r05_build_ab}
mkdir -p $O
B=$R/ab/libchordx_ab_planecached.so
run() {  # tag lib
  if [ "$2" = A ]; then
    timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 3 > $O/$1.json 2> $O/$1.err
  else
    CHORDX_LIB=$B timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 3 > $O/$1.json 2> $O/$1.err
  fi
}
run A1 A; run B1 B; run B2 B; run A2 A
cd /tmp && export TMPDIR=/tmp
for L in A B; do
  for P in FETCH_SIZE WRITE_SIZE; do
    if [ $L = A ]; then
      timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "k_cz_build_roots2" \
        -d $O/pmc_${L}_$P -o run --output-format csv -- python3 $R/benches/bench_czbuild.py 24 0 1 > $O/pmc_${L}_$P.log 2>&1
    else
      CHORDX_LIB=$B timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "k_cz_build_roots2" \
        -d $O/pmc_${L}_$P -o run --output-format csv -- python3 $R/benches/bench_czbuild.py 24 0 1 > $O/pmc_${L}_$P.log 2>&1
    fi
  done
done
for f in $O/*.json; do echo $f; cat $f; echo; done
