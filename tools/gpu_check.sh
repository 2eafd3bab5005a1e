#!/bin/bash
# One GPU session on the gpurun box: parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / abort / timeout ends the script.
# Usage (from the repo root): bash tools/gpu_check.sh [tag] [steps...]
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-"tests bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # run <name> <seconds> <cmd...>; stop on anything but success / plain test failure
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    t:*) files=${s#t:}; files=${files//,/ }   # t:tests/a.py,tests/b.py
         run pytest_sel 900 python -u -m pytest $files -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py ;;
    benchd) run bench_driver 400 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    sqx:*) wl=${s#sqx:}
         run pmc_${wl}_sq 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_$wl/sq" -o sq -- \
            python3 bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --no-companion --no-encoder-record --settle-ms 0 &&
         run pmc_${wl}_grbm 400 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_$wl/grbm" -o grbm -- \
            python3 bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --no-companion --no-encoder-record --settle-ms 0 ;;
    benchx) run bench_xdeepfm 400 python bench.py --workload xdeepfm --no-cpu-baseline ;;
    benchs) run bench_sharded 400 python bench.py --workload deepfm_sharded --no-cpu-baseline ;;
    benchb) run bench_dcn_bf16 400 python bench.py --workload dcn_bf16 --no-cpu-baseline &&
            run bench_pnn_bf16 400 python bench.py --workload pnn_bf16 --no-cpu-baseline ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o deepfm -- \
            python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --settle-ms 0 ;;
    profx) run profx 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profx" -o xdeepfm -- \
            python3 bench.py --workload xdeepfm --steps 5 --warmup 2 --no-cpu-baseline --settle-ms 0 ;;
    sq) run pmc_sq 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_sq" -o sq -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --settle-ms 0 &&
        run pmc_grbm 400 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_grbm" -o grbm -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --settle-ms 0 ;;
    pmc) run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o fetch -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --settle-ms 0 &&
         run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o write -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --settle-ms 0 ;;
    pmc:*) wl=${s#pmc:}
         run pmc_${wl}_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$wl/fetch" -o fetch -- \
            python3 bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --no-companion --no-encoder-record --settle-ms 0 &&
         run pmc_${wl}_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$wl/write" -o write -- \
            python3 bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --no-companion --no-encoder-record --settle-ms 0 ;;
    prof:*) wl=${s#prof:}
         run prof_$wl 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$wl" -o $wl -- \
            python3 bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-companion --no-encoder-record ;;
    settle) for ms in 0 100 400 1000; do
              run settle_$ms 200 python bench.py --steps 20 --warmup 5 --no-companion --no-cpu-baseline --settle-ms $ms
            done ;;
    pmcenc:*) spec=${s#pmcenc:}; V=${spec%%:*}; tab=${spec#*:}   # pmcenc:<vocab>:<row|line>
         d="$OUT/pmc_enc_${V}_$tab"
         for pass in fetch write tcc sq grbm; do
           case $pass in
             fetch) ctr="FETCH_SIZE" ;; write) ctr="WRITE_SIZE" ;; tcc) ctr="TCC_HIT_sum TCC_MISS_sum" ;;
             sq) ctr="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU" ;;
             grbm) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
           esac
           run pmcenc_${V}_${tab}_$pass 300 rocprofv3 --pmc $ctr --output-format csv -d "$d/$pass" -o $pass -- \
              python3 bench.py --workload encoder --vocab $V --enc-table $tab --steps 20 --warmup 3 || exit $?
         done ;;
    pmcwl:*) wl=${s#pmcwl:}   # fetch / write / sq / grbm passes of one bench workload's forward
         d="$OUT/pmc_$wl"
         for pass in fetch write tcc sq sq2 grbm; do
           case $pass in
             fetch) ctr="FETCH_SIZE" ;; write) ctr="WRITE_SIZE" ;; tcc) ctr="TCC_HIT_sum TCC_MISS_sum" ;;
             sq) ctr="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" ;;
             sq2) ctr="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM" ;;
             grbm) ctr="GRBM_GUI_ACTIVE GRBM_COUNT" ;;
           esac
           run pmcwl_${wl}_$pass 400 rocprofv3 --pmc $ctr --output-format csv -d "$d/$pass" -o $pass -- \
              python3 bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline --no-companion --no-encoder-record --no-la-record --settle-ms 0 || exit $?
         done ;;
    profdrv) run profdrv 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profdrv" -o deepfm -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    abenc) for round in 1 2; do   # encoder line table: encoder_line8_kernel (1, 2) vs encoder_k16v2_kernel (0)
             for V in 100000000 1000000; do
               for l8 in 0 1 2; do
                 run abenc_${V}_${l8}_$round 200 python bench.py --workload encoder --vocab $V --enc-table line --steps 100 --warmup 10 --set enc_line8=$l8 || exit $?
                 python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/abenc_${V}_${l8}_$round.log') if l.startswith('{')][-1]); e=d['encoder']['line_table']; print('V=$V enc_line8=$l8 round $round', e['avg_ms'], 'ms', e['line_frac'], d['encoder']['parity_check']['bitwise_equal'])" | tee -a $OUT/abenc.txt
               done
             done
           done ;;
    ab:*) spec=${s#ab:}; wl=${spec%%:*}; libs=${spec#*:}; libs=${libs//,/ }   # ab:<workload>:tree,<vbuild name>,...
         for round in 1 2 3; do
           for L in $libs; do
             if [ $L = tree ]; then LIB=recommendation-models_amd/csrc/librmx.so; else LIB=vbuild/$L/librmx.so; fi
             run ab_${wl}_${L}_$round 200 env RMX_LIB=$LIB python bench.py --workload $wl --steps 200 --warmup 20 --no-companion --no-encoder-record --no-la-record --no-cpu-baseline || exit $?
             python3 -c "import json; d=json.loads([l for l in open('$OUT/ab_${wl}_${L}_$round.log') if l.startswith('{')][-1]); print('$wl $L round $round', round(d['value']/1e6,2), 'M', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})" | tee -a $OUT/ab.txt
           done
         done ;;
    abset:*) spec=${s#abset:}; wl=${spec%%:*}; sets=${spec#*:}; sets=${sets//\// }   # abset:<workload>:k=v/k=v,k2=v2/...
         for round in 1 2 3; do
           for S in $sets; do
             run abset_${wl}_${S//[=,]/_}_$round 200 python bench.py --workload $wl --steps 200 --warmup 20 --no-companion --no-encoder-record --no-la-record --no-cpu-baseline --set "$S" || exit $?
             python3 -c "import json; d=json.loads([l for l in open('$OUT/abset_${wl}_${S//[=,]/_}_$round.log') if l.startswith('{')][-1]); print('$wl $S round $round', round(d['value']/1e6,2), 'M', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()})" | tee -a $OUT/abset.txt
           done
         done ;;
    bsweep:*) sets=${s#bsweep:}; sets=${sets//\// }   # bsweep:k=v/k2=v2 ... : small batches, each knob set
         for B in 1024 4096 8192 16384; do
           for S in $sets; do
             run bsweep_${B}_${S//[=,]/_} 200 python bench.py --batch $B --no-companion --no-encoder-record --no-la-record --parity-only --steps 200 --warmup 10 --set "$S" || exit $?
             python3 -c "import json; d=json.loads([l for l in open('$OUT/bsweep_${B}_${S//[=,]/_}.log') if l.startswith('{')][-1]); print('B $B $S', round(d['value']/1e6,2), 'M', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['stages'].items()}, d['cpu_baseline']['parity_check']['max_abs_diff'])" | tee -a $OUT/bsweep.txt
           done
         done ;;
    fdiag) run fdiag 300 env RMX_LIB=vbuild/fdiag/librmx.so python tools/diag_fused.py ;;
    fdiag:*) v=${s#fdiag:}; run fdiag_$v 300 env RMX_LIB=vbuild/$v/librmx.so python tools/diag_fused.py ;;
    list) run list 120 rocprofv3 -L ;;
    ablines) run ab_lines1 300 python bench.py --no-companion --no-cpu-baseline --steps 200 &&
         run ab_lines0 300 python bench.py --no-companion --no-cpu-baseline --steps 200 --set table_lines=0 &&
         run ab_lines1b 300 python bench.py --no-companion --no-cpu-baseline --steps 200 &&
         run ab_lines0b 300 python bench.py --no-companion --no-cpu-baseline --steps 200 --set table_lines=0 ;;
    lines) for wl in deepfm_sharded dcn_bf16 pnn_bf16 lr_plumbing deepfm_train xdeepfm_train; do
             run line_$wl 400 python bench.py --workload $wl --steps 100 --warmup 10 || exit $?
             grep '^{' "$OUT/line_$wl.log" | tail -n 1 > "$OUT/line_$wl.json"
           done ;;
    lines5) for wl in xdeepfm_cin1 encoder deepfm_sharded dcn_bf16 pnn_bf16 lr_plumbing deepfm_train xdeepfm_train; do
             run line_$wl 400 python bench.py --workload $wl --steps 100 --warmup 10 --no-companion || exit $?
             grep '^{' "$OUT/line_$wl.log" | tail -n 1 > "$OUT/line_$wl.json"
           done ;;
    grid5) for B in 1024 4096 8192 16384 32768 49152 65536 98304 131072; do
             run grid_b$B 300 python bench.py --batch $B --no-companion --no-encoder-record --parity-only --steps 200 --warmup 10 || exit $?
           done ;;
    blas) run probe_blas 300 python tools/probe_blas.py ;;
    profx20) run profx20 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profx20" -o xdeepfm -- \
            python3 bench.py --workload xdeepfm --gpus 1 --steps 20 --warmup 5 ;;
    ab:*) kv=${s#ab:}   # ab:<knob>=<v1>/<v2>: DeepFM and xDeepFM, v1 v2 v1 v2 at 200 / 60 steps
         knob=${kv%%=*}; vals=${kv#*=}; v1=${vals%/*}; v2=${vals#*/}
         i=0
         for v in $v1 $v2 $v1 $v2; do i=$((i+1))
           run ab_${knob}_${v}_${i}_d 300 python bench.py --no-companion --no-cpu-baseline --steps 200 --set $knob=$v || exit $?
           run ab_${knob}_${v}_${i}_x 300 python bench.py --workload xdeepfm --no-cpu-baseline --steps 60 --warmup 5 --set $knob=$v || exit $?
         done ;;
    abt:*) kv=${s#abt:}   # abt:<knob>=<v1>/<v2>: DeepFM / xDeepFM training, v1 v2 v1 v2
         knob=${kv%%=*}; vals=${kv#*=}; v1=${vals%/*}; v2=${vals#*/}; i=0
         for v in $v1 $v2 $v1 $v2; do i=$((i+1))
           run abt_${knob}_${v}_${i}_d 300 python bench.py --workload deepfm_train --steps 60 --warmup 5 --set $knob=$v || exit $?
           run abt_${knob}_${v}_${i}_x 300 python bench.py --workload xdeepfm_train --steps 20 --warmup 3 --set $knob=$v || exit $?
         done ;;
    abw:*) rest=${s#abw:}   # abw:<workload>:<knob>=<v1>/<v2>/...: each value twice, interleaved, 100 steps
         wl=${rest%%:*}; kv=${rest#*:}; knob=${kv%%=*}; vals=$(echo ${kv#*=} | tr '/' ' ')
         for i in 1 2; do
           for v in $vals; do
             run abw_${wl}_${knob}_${v}_${i} 300 python bench.py --workload $wl --no-companion --no-encoder-record --no-cpu-baseline --steps 100 --warmup 10 --set $knob=$v || exit $?
           done
         done ;;
    abb:*) rest=${s#abb:}   # abb:<batch>:<knob>=<v1>/<v2>/...: DeepFM at that batch, each value twice, interleaved
         B=${rest%%:*}; kv=${rest#*:}; knob=${kv%%=*}; vals=$(echo ${kv#*=} | tr '/' ' ')
         for i in 1 2; do
           for v in $vals; do
             run abb_b${B}_${knob}_${v}_${i} 300 python bench.py --batch $B --no-companion --no-encoder-record --parity-only --steps 400 --warmup 20 --set $knob=$v || exit $?
           done
         done ;;
    pmcb:*) B=${s#pmcb:}   # DeepFM at launch batch B: kernel trace, SQ / GRBM counters, HBM fetch / write
         A="python3 bench.py --batch $B --steps 20 --warmup 5 --no-cpu-baseline --no-companion --no-encoder-record --settle-ms 0"
         run prof_b$B 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmcb_$B/prof" -o k -- $A &&
         run pmc_b${B}_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmcb_$B/sq" -o sq -- $A &&
         run pmc_b${B}_grbm 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmcb_$B/grbm" -o grbm -- $A &&
         run pmc_b${B}_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcb_$B/fetch" -o fetch -- $A &&
         run pmc_b${B}_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmcb_$B/tcc" -o tcc -- $A ;;
    trb:*) B=${s#trb:}   # DeepFM at launch batch B: kernel trace only (per-kernel durations and gaps)
         run trace_b$B 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trb_$B" -o k -- \
            python3 bench.py --batch $B --steps 50 --warmup 5 --no-cpu-baseline --no-companion --no-encoder-record --no-la-record --settle-ms 0 ;;
    graph) run probe_graph 300 python tools/probe_graph.py ;;
    wgprobe) for dg in 0 1 2 4 6 0; do   # dW timing probes (wgrad_sq_kernel DG; results wrong by construction)
               run wgprobe_$dg 300 python bench.py --workload deepfm_train --steps 20 --warmup 5 --no-companion --set wgrad_diag=$dg || exit $?
             done ;;
    testk:*) k=${s#testk:}
         run pytest_$k 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k $k ;;
    bench2) run bench_gpus2 400 python bench.py --gpus 2 --steps 20 --warmup 5 ;;
    benchsc) run bench_sharded_companion 400 python bench.py --gpus 1 --steps 20 --warmup 5 --sharded-companion ;;
    bench2s) echo "== bench_gpus2_sharded (expects a clean refusal on a 1-GPU box)" | tee -a "$OUT/steps.log"
         timeout -k 10 300 python bench.py --workload deepfm_sharded --gpus 2 --steps 5 --warmup 1 \
            > "$OUT/bench_gpus2_sharded.log" 2>&1
         echo "== bench_gpus2_sharded rc=$?" | tee -a "$OUT/steps.log"; tail -n 5 "$OUT/bench_gpus2_sharded.log" ;;
    profd) run profd 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profd" -o driver -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench:*) wl=${s#bench:}
         run bench_$wl 400 python bench.py --workload $wl ;;
    benchq:*) wl=${s#benchq:}
         run bench_$wl 400 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline ;;
  esac
done
echo "== all done"
