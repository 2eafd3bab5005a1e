#!/bin/bash
# What outlives `bench.py --gpus 1`?  Lists this session's processes before and after one bench run
# (VERDICT r03 housekeeping: the driver's record shows procs_at_end 1).
OUT=${1:-gpurun_out/procs}
mkdir -p "$OUT"
ps -o pid,ppid,pgid,sid,stat,etime,cmd -s $$ > "$OUT/before.txt" 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench rc=$?" > "$OUT/rc.txt"
sleep 2
ps -o pid,ppid,pgid,sid,stat,etime,cmd -s $$ > "$OUT/after.txt" 2>&1
# this user's processes other than this script's shell and ps itself (python / bench leftovers)
ps -u "$(id -u)" -o pid=,ppid=,comm= | awk -v me=$$ '$1 != me && $2 != me && $3 != "ps" && $3 != "bash"' > "$OUT/user_after.txt"
echo "leftover processes of this user: $(wc -l < "$OUT/user_after.txt")" >> "$OUT/rc.txt"
cat "$OUT/rc.txt" "$OUT/after.txt"
