#!/bin/bash
# Round 6 diagnostics 1: u128 shift tests, pre-0a5da05 build repeat, RCCL sizes.
# Stops at the first step that aborts, faults or times out (rc not 0/1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/diag1; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step u128 240 python -u -m pytest tests/test_gpu_u128.py -x -v --timeout 200 --timeout-method thread
step r5enc_old_a 120 env CHORDX_LIB=$PWD/ab/libchordx_r5enc.so python -u tools/diag_r5enc_repeat.py 3
step r5enc_old_b 120 env CHORDX_LIB=$PWD/ab/libchordx_r5enc.so python -u tools/diag_r5enc_repeat.py 3
step r5enc_head 120 python -u tools/diag_r5enc_repeat.py 3
step rccl 400 python -u tools/diag_rccl_a2a.py AB
