#!/bin/bash
# Round 6 batch 4: build-variant positions, GPU suite, C2 PMC passes, bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b4; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step czb 300 python -u tools/diag_cz_build_r5.py
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
P=1
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  step c2pmc$P 90 rocprofv3 --pmc $c -d $O/c2pmc$P -o c2 --output-format csv -- python3 benches/bench_c2.py
  P=$((P+1))
done
step bench 900 python -u bench.py
