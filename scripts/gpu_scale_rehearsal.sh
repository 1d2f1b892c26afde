#!/bin/bash
# GPU box: 1-GPU bench + CPU-rank rehearsal of the N=2,4,8 control-plane scaling (gloo, no payload).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_n1.log 2>&1 || { tail -30 gpurun_out/bench_n1.log; exit 1; }
grep metric gpurun_out/bench_n1.log
for n in 2 4 8; do
  KAMD_BENCH_FORCE_CPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 5 --warmup 2 > gpurun_out/bench_cpu_n$n.log 2>&1 || { tail -30 gpurun_out/bench_cpu_n$n.log; exit 1; }
  grep metric gpurun_out/bench_cpu_n$n.log
done
# single API server process at N=8 for comparison with the auto (multi-worker) default
KAMD_BENCH_FORCE_CPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29620 bench.py --gpus 8 --steps 5 --warmup 2 --apiserver-workers 1 > gpurun_out/bench_cpu_n8_w1.log 2>&1 || { tail -30 gpurun_out/bench_cpu_n8_w1.log; exit 1; }
grep metric gpurun_out/bench_cpu_n8_w1.log
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
echo ALL_OK
