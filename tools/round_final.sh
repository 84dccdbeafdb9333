#!/bin/bash
# Round-end evidence in one call: GPU suite + smoke + default bench + kernel
# trace (gpu_final.sh), PMC traffic passes (profiles/run_profile.sh), per-row
# bench with CPU legs.  Each step has its own limit; && chained.
set -eo pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_final.sh "$TAG"
cd "$GRAFT_REPO_ROOT"
bash profiles/run_profile.sh "${TAG}_pmc"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u benches/bench_rows.py > "gpurun_out/$TAG/rows.json" 2> "gpurun_out/$TAG/rows.err"
echo rows done
