#!/bin/bash
# A/B timing on the GPU box: bench.py (no CPU baseline, no companions) once per library variant, twice,
# interleaved; prints value and per-stage ms.  Usage: bash tools/ab_run.sh OUTDIR "bench args" lib1 lib2 ...
# (lib "default" = the in-tree librmx.so; "set:k=v,k=v" = the in-tree library with those knobs)
set -u
OUT=$1; ARGS=$2; shift 2
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    tag=$(basename "$(dirname "$lib")")
    [ "$lib" = default ] && tag=default
    case $lib in set:*) tag=${lib#set:}; tag=${tag//,/_};; esac
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion $ARGS > "$OUT/$tag.$rep.json" 2> "$OUT/$tag.$rep.err"
    elif [ "${lib#set:}" != "$lib" ]; then  # set:k=v,k=v -- knobs on the in-tree library
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion --set "${lib#set:}" $ARGS > "$OUT/$tag.$rep.json" 2> "$OUT/$tag.$rep.err"
    else
      RMX_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-companion $ARGS > "$OUT/$tag.$rep.json" 2> "$OUT/$tag.$rep.err"
    fi
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag rep $rep rc=$rc"; tail -3 "$OUT/$tag.$rep.err"; exit $rc; fi
    python3 - "$OUT/$tag.$rep.json" "$tag" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = " ".join("%s=%.4f" % (k, v["avg_ms"]) for k, v in d.get("stages", {}).items())
print("%-14s %8.2f M/s  %s" % (sys.argv[2], d["value"] / 1e6, st))
EOF
  done
done
