#!/bin/bash
# Round 6 batch 17: where the non-kernel time of a warm churn -> route-ready
# epoch goes (kernel + HIP API trace of benches/bench_ready.py, 2^24, 4 epochs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b17; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step ready 300 python3 benches/bench_ready.py 24 4
tail -2 $O/ready.log
step ready_trace 300 rocprofv3 --kernel-trace --hip-trace -d $O/trace -o ready --output-format csv -- python3 benches/bench_ready.py 24 4
ls -la $O/trace/*/ 2>/dev/null | head; find $O/trace -name "*.csv" -size +20M -exec gzip {} \;
