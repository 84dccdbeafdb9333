#!/bin/bash
# Same-box A/B of the finger build: bench_fingers.py child (2^24) per ab_libs/*.so
# under rocprofv3 kernel stats.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-fingers_ab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for pass in 1 2; do
for lib in "$GRAFT_REPO_ROOT"/ab_libs/*.so; do
  name=$(basename "$lib" .so)_$pass
  CHORDX_LIB=$lib CX_BENCH_FINGERS_CHILD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d "$OUT/$name" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benches/bench_fingers.py" 24 \
    > "$OUT/$name.log" 2>&1
  python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:30], r['Calls'], float(r['AverageNs'])/1e6) for r in csv.DictReader(open(sys.argv[1])) if 'fingers' in r['Name']]" "$OUT/$name/run_kernel_stats.csv" "$name"
  tail -1 "$OUT/$name.log"
done
done
