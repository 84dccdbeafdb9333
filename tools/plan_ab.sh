# (Experiment record: the CX_CZ_PLAN knob was measured slower and removed; see DESIGN.md.)
# cz walk plan-budget A/B: route parity tests at budget 2, then the bench per budget.
set -eo pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/plan_ab
mkdir -p $OUT
CX_CZ_PLAN=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_b2.log 2>&1
tail -1 $OUT/pytest_b2.log
for b in 0 2 3 4 6; do
  CX_CZ_PLAN=$b timeout -k 10 300 python -u bench.py --no-cpu --steps 20 > $OUT/bench_b$b.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_b$b.log').read().strip().splitlines()[-1]); print('budget $b', round(d['value']/1e9,3), 'G/s kernel', round(d['roofline']['kernel_ms'],3), 'ms bad', d['bad_status'], 'mean_hops', round(d['mean_hops'],4))"
done
