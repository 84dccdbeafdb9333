#!/bin/bash
# Same-box A/B: run a JSON-printing python script once per ab_libs/*.so
# (CHORDX_LIB), two passes in alternating order.  bash tools/lib_ab_json.sh <script> [args]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
for pass in 1 2; do
  for lib in ab_libs/*.so; do
    CHORDX_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python -u "$@" 2>/dev/null | tail -1
  done
done
