#!/bin/bash
# N=1 control-plane shape sweep on the one-GPU box: the driver's bench command per
# (API workers, scheduler shards, hollow processes); each run under its own time limit, the
# sweep stops at the first abnormal exit.
out=${1:-gpurun_out/sweep}
mkdir -p "$out"
# SHAPES="w s h;w s h" overrides the shape list; SKIP_PRE=1 skips the process-group and RPC runs
if [ -z "$SKIP_PRE" ]; then
# the RCCL process-group path of N > 1 on this one GPU: device binding + barriers from threads
KAMD_BENCH_FORCE_PG=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29641 bench.py --steps 5 --warmup 2 > "$out/pg1.json" 2> "$out/pg1.err" || exit $?
echo "pg1 $(tail -1 "$out/pg1.json" | cut -c1-160)" >> "$out/summary.txt"
# CPU per device-plugin RPC on this box (grpc.aio vs grpclite; no GPU use)
timeout -k 10 120 python -m kubernetes_amd.kubemark.rpc_bench > "$out/rpc_bench.jsonl" 2> "$out/rpc_bench.err" || exit $?
fi
IFS=';' read -ra shapes <<< "${SHAPES:-0 0 0;4 2 4;4 3 4;5 3 4;3 2 4;4 2 6;0 0 0}"
i=0
for shape in "${shapes[@]}"; do
  set -- $shape
  i=$((i + 1))
  tag="$i-w$1-s$2-h$3"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --apiserver-workers $1 --scheduler-shards $2 \
      --hollow-procs $3 > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
  echo "$tag $(python -c "import json,sys; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print(d['value'], d['p50_startup_ms'], d['config']['apiserver_workers'], d['config']['scheduler_shards'], d['config']['hollow_procs_per_rank'])")" >> "$out/summary.txt"
done
