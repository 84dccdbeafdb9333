#!/bin/bash
# Round-5 GPU check: the -m gpu suite, then the default bench line.
#   bash tools/r05_check.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r05_check}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc2=$?
echo "bench rc=$rc2 bytes=$(wc -c < $O/bench.json)"
tail -c 600 $O/bench.err
exit $rc2
