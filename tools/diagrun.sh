set -u
mkdir -p gpurun_out/diag
for d in base 1 2 3 4 32; do
  if [ $d = base ]; then L=recommendation-models_amd/csrc/librmx.so; else L=build/diag$d/librmx.so; fi
  RMX_LIB=$L timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-companion --no-cpu-baseline --settle-ms 300 > gpurun_out/diag/$d.json 2> gpurun_out/diag/$d.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/diag/$d.json')); print('$d', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
done
