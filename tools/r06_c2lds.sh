cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06/${TAG:-c2lds}; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "successor or predecessor"
tail -2 $O/tests.log
step ab 300 python -u benches/bench_c2.py 1 5 4 --rounds 6
cat $O/ab.log
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benches/bench_c2.py 1 5 --rounds 2
find $O/prof -name "*kernel_stats.csv" -exec grep -E "Name|successor" {} \;
