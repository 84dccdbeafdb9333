# Gather ceiling vs table size (64-B quad entries up to 64 GiB, the cz table's
# size) and FETCH_SIZE calibration for the same access pattern.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/gather
mkdir -p "$OUT"
P=$GRAFT_REPO_ROOT/p2p-dhts_amd/csrc/tools/gather_probe
timeout -k 10 300 $P $((80 << 30)) coop_sweep > "$OUT/coop_sweep.json" 2>&1
cat "$OUT/coop_sweep.json"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_chase_coop" -d "$OUT/pmc_fetch" -o run --output-format csv -- $P $((64 << 30)) calib > "$OUT/calib.json" 2>&1
cat "$OUT/calib.json"
