#!/bin/bash
# Arc protocols on one GPU: arc GPU tests, then the G-rank simulation
# (soa vs record key-first) at 2^25 total keys and at C4's 2^28 (2^25 / rank).
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-arc_soa}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_arc.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_arc.log" 2>&1
tail -2 "$OUT/pytest_arc.log"
timeout -k 10 400 python -u benches/bench_arc_sim.py --groups ${2:-8} --modes soa,key_first \
  --reps 2 > "$OUT/arc_sim_q25.json" 2> "$OUT/arc_sim_q25.err"
timeout -k 10 500 python -u benches/bench_arc_sim.py --groups ${2:-8} --modes soa \
  --keys-log2 28 --reps 2 > "$OUT/arc_sim_q28.json" 2> "$OUT/arc_sim_q28.err"
python3 - "$OUT" <<'PY'
import json, sys
for f in ("arc_sim_q25.json", "arc_sim_q28.json"):
    d = json.load(open(f"{sys.argv[1]}/{f}"))
    print(f, "replicated_ms", round(d["replicated_route_ms"], 3))
    for a in d["arc"]:
        print(a["G"], a["mode"], round(a["per_gpu_compute_ms"], 3),
              round(a["per_gpu_xgmi_ms_model"], 3), "%.3g" % a["projected_lookups_per_s_per_gpu"],
              a.get("equals_replicated"), a.get("partition_ms_max"), a.get("route_ms_max"),
              a.get("deliver_ms_max"))
PY
