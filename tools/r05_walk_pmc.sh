#!/bin/bash
# Route walk PMC (round 5): SQ / TA counters of the default walk (k_walk<false>)
# on the C4 batch (benches/bench_walk.py), one rocprofv3 pass per counter group.
#   bash tools/r05_walk_pmc.sh <tag> [kernel-regex]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/${1:-r05_walk_pmc}
RX=${2:-k_walk<false, false, false>}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/benches/bench_walk.py 2 1"
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TA_BUSY_avr TA_BUSY_max" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$RX" \
    -d $O/pmc$i -o run --output-format csv -- $B > $O/pmc$i.log 2>&1
done
find $O -name "*counter_collection.csv" | sort
