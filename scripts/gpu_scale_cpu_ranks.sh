#!/bin/bash
# GPU box: N=1 GPU bench, then CPU-rank (gloo, no payload) rehearsals of N=2,4 with the auto
# control-plane shape; optional extra shapes via SHAPES="n:w:s:hp ...".
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/scale
summ() { python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][0])
c = d["config"]
print(f"{sys.argv[2]}: {d['value']} pods/s p50={d['p50_startup_ms']} p99={d['p99_startup_ms']} step={d['ms_per_step']}ms w={c['apiserver_workers']} s={c['scheduler_shards']} hp={c.get('hollow_procs_per_rank')} cpu/pod={d['cpu_ms_per_pod']} phases={d.get('step_phases_ms')} step_max={d.get('step_ms_max')} api={d.get('api_call_ms')}")
PY
}
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 > gpurun_out/scale/n1.log 2>&1 || { tail -30 gpurun_out/scale/n1.log; exit 1; }
summ gpurun_out/scale/n1.log "N=1 gpu"
for n in ${NS:-2 4}; do
  KAMD_BENCH_FORCE_CPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps ${STEPS:-10} --warmup 2 > gpurun_out/scale/cpu_n$n.log 2>&1 || { tail -30 gpurun_out/scale/cpu_n$n.log; exit 1; }
  summ gpurun_out/scale/cpu_n$n.log "N=$n cpu-ranks auto"
done
for sh in $SHAPES; do
  IFS=: read n w s hp <<< "$sh"
  log=gpurun_out/scale/cpu_n${n}_w${w}_s${s}_hp${hp}.log
  KAMD_BENCH_FORCE_CPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29700+n)) bench.py --gpus $n --steps ${STEPS:-10} --warmup 2 --apiserver-workers $w --scheduler-shards $s --hollow-procs $hp > $log 2>&1 || { tail -30 $log; exit 1; }
  summ $log "N=$n w=$w s=$s hp=$hp"
done
echo ALL_OK
