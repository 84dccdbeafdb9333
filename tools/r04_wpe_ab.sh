set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/r04_wpe
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 3 > $O/w7_$r.json 2> $O/w7_$r.err
  CX_CZ2_WPE=8 timeout -k 10 200 python3 benches/bench_czbuild.py 24 0 3 > $O/w8_$r.json 2> $O/w8_$r.err
done
