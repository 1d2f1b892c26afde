#!/bin/bash
# GPU box: interleaved N=1 bench runs over control-plane shapes (API server workers x scheduler
# shards x hollow processes per rank), so box noise spreads evenly over the shapes. One JSON line
# per run under $out; any failing run ends the sweep.
out=${1:-gpurun_out/sweep}
reps=${REPS:-2}
mkdir -p "$out"
for r in $(seq 1 "$reps"); do
  for shape in "3 2 6" "4 2 6" "4 3 6" "5 3 6" "4 2 4"; do
    set -- $shape
    f="$out/w$1_s$2_h$3_r$r.json"
    timeout -k 10 180 python bench.py --steps 20 --warmup 5 --apiserver-workers "$1" --scheduler-shards "$2" \
      --hollow-procs "$3" --xgmi4-steps 0 > "$f" 2> "$f.err" || exit $?
    grep -o '"value": [0-9.]*' "$f" | head -1 | sed "s|^|w$1 s$2 h$3 r$r |"
  done
done
