#!/bin/bash
# C5 scan profile (round 4): kernel trace of benches/bench_c5.py, then PMC
# passes of k_misplaced (the fused maintenance pass), each pass its own
# process.  CSV output under gpurun_out/${1:-r04_c5}/.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/${1:-r04_c5}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/benches/bench_c5.py --steps 3 --warmup 1 --oracle-sample 4096"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  --kernel-include-regex "misplaced|nsucc" -- $B > $O/trace.json 2> $O/trace.err
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU" \
         "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_BUSY_max" \
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "k_misplaced" \
    -d $O/pmc$i -o run --output-format csv -- $B > $O/pmc$i.json 2> $O/pmc$i.err
done
