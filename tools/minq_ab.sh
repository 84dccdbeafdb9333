set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/minq; mkdir -p $O
for lq in 16 18 20 22; do
  for L in base 64 128 256; do
    if [ $L = base ]; then timeout -k 10 120 python3 benches/bench_walk.py 10 3 24 $lq > $O/${L}_$lq.json 2>/dev/null
    else CHORDX_LIB=$PWD/ab/libchordx_minq$L.so timeout -k 10 120 python3 benches/bench_walk.py 10 3 24 $lq > $O/${L}_$lq.json 2>/dev/null; fi
  done
done
