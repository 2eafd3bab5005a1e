set -u
O=gpurun_out/pf; mkdir -p $O
for L in base pf6 pf13; do
  if [ $L = base ]; then LIB=recommendation-models_amd/csrc/librmx.so; else LIB=build/$L/librmx.so; fi
  for v in 4 6; do
    RMX_LIB=$LIB timeout -k 10 120 python bench.py --workload dcn_bf16 --steps 100 --warmup 10 --no-cpu-baseline --set tower_variant=$v > $O/${L}_$v.json || exit 1
    python3 -c "
import json; d=json.load(open('$O/${L}_$v.json')); print('$L var=$v', round(d['value']/1e6,1), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})"
  done
done
