#!/usr/bin/env bash
# rocprofv3 of the Pippenger MSM alone (tools/pip_probe.py: 2^20 config-3 points, window 12)
#   tools/profile_pip.sh <tag>  -> gpurun_out/prof_<tag>_pip/
# Kernel trace + stats of 12 MSMs over 2 streams; then PMC passes, each its own run with
# --kernel-trace only (FETCH_SIZE and WRITE_SIZE do not share a TCC pass on gfx950), over 3 MSMs
# on one stream (counters are per dispatch; the profiler serialises dispatches).
set -euo pipefail
TAG=${1:-r03}
OUT=gpurun_out/prof_${TAG}_pip
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 tools/pip_probe.py 20 12 12 2 > "$OUT/probe.txt" 2> "$OUT/trace.err"
P="python3 tools/pip_probe.py 20 12 3 1"
pmc() {   # pmc <name> <counters...>
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/pmc_$name" -o run -- $P > "$OUT/probe_$name.txt" 2> "$OUT/$name.err"
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc valu SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS
pmc cyc SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc busy VALUBusy VALUUtilization
pmc tcc TCC_HIT_sum TCC_MISS_sum
ls -R "$OUT" > "$OUT/listing.txt"
