#!/bin/bash
# C2 LDS search A/B: successor/predecessor tests of the in-tree library, then
# bench_c2.py (variants 4 and 5) alternating in-tree (A) and $1 (B), and a
# kernel trace of each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; B=$R/$1; O=$R/gpurun_out/r06/${2:-c2ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "successor or predecessor" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 120 python3 benches/bench_c2.py 4 5 --rounds 4 > $O/A_$i.json 2> $O/A_$i.err || exit 1
  CHORDX_LIB=$B timeout -k 10 120 python3 benches/bench_c2.py 4 5 --rounds 4 > $O/B_$i.json 2> $O/B_$i.err || exit 1
done
cd /tmp
for v in A B; do
  L=$R/p2p-dhts_amd/chordx/libchordx.so; [ $v = B ] && L=$B
  CHORDX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $R/benches/bench_c2.py 4 --rounds 2 > $O/prof_$v.log 2>&1 || exit 1
done
cd $R
python3 - $O <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
for v in "AB":
    for i in (1, 2):
        d = json.load(open(f"{o}/{v}_{i}.json"))
        print(v, i, {k: round(min(x), 2) for k, x in d["us_per_call_by_variant"].items()}, d["identical"])
    for f in glob.glob(f"{o}/prof_{v}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "successor" in r["Name"]:
                print(v, r["Name"][:32], r["Calls"], r["AverageNs"], r["MinNs"])
PY
