#!/bin/bash
# Alternating A/B of two builds of libchordx.so on one box: A = the in-tree
# library, B = the library named by $1 (CHORDX_LIB), each round runs
# `python3 <script> <args>` once per build.  Outputs: gpurun_out/$2/{A,B}_<round>.json
#   bash tools/ab_lib.sh ab/libchordx_base.so TAG ROUNDS script.py args...
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
BLIB=$R/$1; TAG=$2; N=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $N); do
  timeout -k 10 300 python3 "$@" > $O/A_$i.json 2> $O/A_$i.err
  CHORDX_LIB=$BLIB timeout -k 10 300 python3 "$@" > $O/B_$i.json 2> $O/B_$i.err
done
