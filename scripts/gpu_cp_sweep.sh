#!/bin/bash
# GPU box: control-plane shape sweep (API server workers x scheduler shards) with CPU ranks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/sweep
python -c "import bench; print('cpu_budget', bench.cpu_budget())"
for n in ${SWEEP_N:-4 8}; do
  for cfg in ${SWEEP_CFGS:-1x1 1x2 2x1 2x2}; do
    w=${cfg%x*}; s=${cfg#*x}
    log=gpurun_out/sweep/n${n}_w${w}_s${s}.log
    KAMD_BENCH_FORCE_CPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29700+n)) bench.py --gpus $n --steps 5 --warmup 2 --apiserver-workers $w --scheduler-shards $s > $log 2>&1 || { tail -30 $log; exit 1; }
    python - "$log" "$n" "$cfg" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][0])
print(f"N={sys.argv[2]} w x s={sys.argv[3]}: {d['value']} pods/s p50={d['p50_startup_ms']}ms p99={d['p99_startup_ms']}ms cpu/pod={d['cpu_ms_per_pod']}")
PY
  done
done
echo ALL_OK
