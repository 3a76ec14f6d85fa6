#!/usr/bin/env bash
# Kernel timeline of warm one-proof cuda_range_proof_verify calls (tools/oneshot_probe.py) on the GPU box.
#   tools/profile_oneshot.sh <tag>  -> gpurun_out/prof_<tag>_oneshot/{trace/, timeline.txt}
set -euo pipefail
TAG=${1:-r04}
OUT=gpurun_out/prof_${TAG}_oneshot
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/oneshot_probe.py ${ITERS:-10} ${SIZES:-16,64} > "$OUT/probe.txt" 2> "$OUT/trace.log"
python3 - "$OUT" > "$OUT/timeline.txt" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
prev = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s - t0) / 1e3:12.1f} gap {(s - prev) / 1e3:8.1f} dur {(e - s) / 1e3:8.1f} us  q{r.get("Queue_Id", "?")} '
          f'grid {r.get("Grid_Size_X", r.get("Grid_Size", "?"))}  {r["Kernel_Name"].split("(")[0][-50:]}')
    prev = e
PY
