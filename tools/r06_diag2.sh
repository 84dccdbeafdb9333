#!/bin/bash
# Round 6 diagnostics 2: pre-0a5da05 package repeat (old table builds), RCCL
# self-exchange size threshold and the 9ac284c placement path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/diag2; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step r5enc_old_a 120 env CHORDX_PKG=$PWD/ab/old_r5enc/p2p-dhts_amd python -u tools/diag_r5enc_repeat.py 3
step r5enc_old_b 120 env CHORDX_PKG=$PWD/ab/old_r5enc/p2p-dhts_amd python -u tools/diag_r5enc_repeat.py 3
step rccl 400 python -u tools/diag_rccl_a2a.py SB
step selfx 600 python -u -m pytest tests/test_gpu_arc.py -x -v --timeout 500 --timeout-method thread -k "self_exchange or rccl_world1"
