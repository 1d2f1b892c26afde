#!/bin/bash
# GPU box: 1-GPU bench with the rank's hollow nodes in 1 / 2 / 4 / 8 processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/hollow
python -c "import bench; print('cpu_budget', bench.cpu_budget())"
for hp in ${HP_LIST:-1 2 4 8}; do
  for w in ${W_LIST:-1}; do
    log=gpurun_out/hollow/hp${hp}_w${w}.log
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --hollow-procs $hp --apiserver-workers $w > $log 2>&1 || { tail -30 $log; exit 1; }
    python - "$log" "$hp" "$w" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][0])
print(f"hp={sys.argv[2]} w={sys.argv[3]}: {d['value']} pods/s p50={d['p50_startup_ms']}ms p99={d['p99_startup_ms']}ms step={d['ms_per_step']}ms cpu/pod={d['cpu_ms_per_pod']} payload={d['payload_runs']}/{d['payload_failures']}")
PY
  done
done
echo ALL_OK
