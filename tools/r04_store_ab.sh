#!/bin/bash
# Route-table build A/B (round 4): streaming against write-back table stores,
# alternating processes.  First run (r04_storeab): streaming was the default and
# CX_CZ2_MODE=32 selected write-back; write-back is now the default and 32
# selects streaming (files nt_* / wb_* keep their meaning).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/${1:-r04_storeab}
mkdir -p $O
for r in 1 2 3; do
  CX_CZ2_MODE=32 timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 3 > $O/nt_$r.json 2> $O/nt_$r.err
  timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 3 > $O/wb_$r.json 2> $O/wb_$r.err
done
