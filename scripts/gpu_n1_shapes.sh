#!/bin/bash
# GPU box: N=1 bench under several control-plane shapes, REPS runs each (noise estimate).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/n1shapes
for sh in ${SHAPES:-1:1:4 2:1:4 2:2:4}; do
  IFS=: read w s hp <<< "$sh"
  for r in $(seq 1 ${REPS:-2}); do
    log=gpurun_out/n1shapes/w${w}_s${s}_hp${hp}_r$r.log
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --apiserver-workers $w --scheduler-shards $s --hollow-procs $hp > $log 2>&1 || { tail -20 $log; exit 1; }
    python - $log "w=$w s=$s hp=$hp r=$r" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][0])
print(f"{sys.argv[2]}: {d['value']} pods/s p50={d['p50_startup_ms']} p99={d['p99_startup_ms']} phases={d.get('step_phases_ms')} cpu={d['cpu_ms_per_pod']}")
PY
  done
done
echo ALL_OK
