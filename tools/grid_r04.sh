#!/bin/bash
# SURVEY.md §8d's measurement grid: DeepFM at B = 1,024 ... 131,072 (the launch
# batch; the cliff check 32,768 ... 131,072), xDeepFM at 1,024 / 4,096 / 16,384, and the secondary Zipf(1.1)
# id distribution -- each line with the parity check of 512 (64) predicted rows against the fp64 oracle.
# Usage: bash tools/grid_r04.sh OUTDIR [deepfm|xdeepfm|zipf ...]
set -u
O=${1:-gpurun_out/grid}; shift || true
PARTS=${*:-"deepfm xdeepfm zipf"}
mkdir -p "$O"
line() {  # line <tag> <bench args...>
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-companion --parity-only "$@" > "$O/$tag.json" 2> "$O/$tag.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -3 "$O/$tag.err"; exit $rc; fi
  python3 - "$O/$tag.json" "$tag" <<'EOF' | tee -a "$O/summary.txt"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pc = (d.get("cpu_baseline") or {}).get("parity_check") or {}
st = " ".join("%s=%.4f" % (k, v["avg_ms"]) for k, v in d.get("stages", {}).items())
print("%-16s B=%-6d %9.3f M/s  %.4f ms/step  parity %.2e (%s)  %s" % (
    sys.argv[2], d["config"]["global_batch"], d["value"] / 1e6, d["ms_per_step"], pc.get("max_abs_diff", -1),
    "ok" if pc.get("ok") else "FAIL", st))
EOF
}
for part in $PARTS; do
  case $part in
    deepfm)
      for B in 1024 4096 8192 16384 32768 49152 65536 98304 131072; do
        steps=100; [ $B -le 16384 ] && steps=400
        line deepfm_b$B --batch $B --steps $steps --warmup 20
      done ;;
    xdeepfm)
      for B in 1024 4096 16384; do
        line xdeepfm_b$B --workload xdeepfm --batch $B --steps 30 --warmup 5
      done ;;
    zipf)
      line deepfm_zipf1.1_b65536 --zipf 1.1 --steps 100 --warmup 10 ;;
  esac
done
