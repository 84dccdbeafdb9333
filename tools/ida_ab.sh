# IDA A/B on the GPU box: parity tests, then bench_ida.py per kernel variant.
set -eo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ida_ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_ida.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ida_ab/pytest.log 2>&1
tail -2 gpurun_out/ida_ab/pytest.log
run() { timeout -k 10 120 env "$@" python -u benches/bench_ida.py > gpurun_out/ida_ab/$1.json 2>gpurun_out/ida_ab/$1.err; echo "$1 $(cat gpurun_out/ida_ab/$1.json)"; }
run CX_IDA_GENERIC=1
run CX_IDA_DEC_D=1
run CX_IDA_DEC_D=2
