# IDA PMC passes (one counter group per rocprofv3 run), kernel-filtered.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/ida_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/benches/prof_ida.py"
RX="k_ida_encode|k_ida_decode"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-include-regex "$RX" -d "$OUT/sq" -o run --output-format csv -- $B > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d "$OUT/fetch" -o run --output-format csv -- $B > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d "$OUT/write" -o run --output-format csv -- $B > "$OUT/write.log" 2>&1
echo pmc done
