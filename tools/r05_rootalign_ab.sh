#!/bin/bash
# Route-table build dispatch order A/B: in-tree library (A: root-aligned chunk
# order) against $1 (B: the previous row-aligned order), ABBA, bench_czbuild
# (2^24, 5 builds each, same table hash), then one FETCH_SIZE and one
# WRITE_SIZE pass of k_cz_build_roots2 per library.
#   bash tools/r05_rootalign_ab.sh ab/libchordx_base.so <tag>
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
B=$R/$1
O=$R/gpurun_out/${2:-r05_rootalign_ab}
mkdir -p $O
run() {  # tag lib
  if [ "$2" = A ]; then
    timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 5 > $O/$1.json 2> $O/$1.err
  else
    CHORDX_LIB=$B timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 5 > $O/$1.json 2> $O/$1.err
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
