#!/bin/bash
# Route walk PMC (round 4): SQ counters of k_route_tree<false, true> on the
# bench ring (headline only), one pass per counter group.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/${1:-r04_route_pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-arc --no-churn --no-c5"
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
         "TA_BUSY_avr TA_BUSY_max" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "k_route_tree" \
    -d $O/pmc$i -o run --output-format csv -- $B > $O/pmc$i.log 2>&1
done
