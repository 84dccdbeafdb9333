#!/bin/bash
# Tail effect of the static per-wave chunks: route kernel time at 2^24, 2^25,
# 2^26 lookups on the 2^24 ring (kernel ms from the bench's HIP events).
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-tail}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
for k in 24 25 26; do
  timeout -k 10 300 python -u bench.py --keys-log2 $k --steps 5 --warmup 2 --no-cpu > "$OUT/bench_k$k.log" 2>&1
  python3 -c "
import json; d=json.loads(open('$OUT/bench_k$k.log').read().strip().splitlines()[-1])
print($k, d['roofline']['kernel_ms'], d['ms_per_step'], d['value'])"
done
