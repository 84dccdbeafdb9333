#!/bin/bash
# Route-table build profile (round 4): kernel trace of the two root-centric
# builds (table_build 0 = blocks sized by distinct roots, 4 = 256-row blocks),
# then PMC passes of the build kernels, each pass its own process.  CSV
# output straight under gpurun_out/r04_prof/ (small: the builds only).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/r04_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  --kernel-include-regex "cz_build|fingers" -- python3 $R/benches/bench_czbuild.py 24 0,4 2 > $O/trace.json 2> $O/trace.err
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_BUSY_max" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "cz_build" \
    -d $O/pmc$i -o run --output-format csv -- python3 $R/benches/bench_czbuild.py 24 0,4 1 > $O/pmc$i.json 2> $O/pmc$i.err
done
