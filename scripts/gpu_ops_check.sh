#!/bin/bash
# GPU box: HIP op tests + diagnostics + rocprof kernel stats. Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -m gpu -x -q > gpurun_out/gpu_ops.log 2>&1 || { echo "gpu_ops failed"; tail -30 gpurun_out/gpu_ops.log; exit 1; }
timeout -k 10 120 ./kubernetes_amd/native/bin/hip-vector-add > gpurun_out/vadd.log 2>&1 || { echo "vadd failed"; cat gpurun_out/vadd.log; exit 1; }
timeout -k 10 120 ./kubernetes_amd/native/bin/xgmi-probe 64 5 > gpurun_out/xgmi.log 2>&1 || { echo "xgmi failed"; cat gpurun_out/xgmi.log; exit 1; }
timeout -k 10 300 python -c "
from kubernetes_amd.ops import hip_kernels as h
print(h.diag_mfma(0,4096,20)); print(h.diag_mfma(0,8192,10)); print(h.diag_hbm(0,1<<30,20))" > gpurun_out/diag.log 2>&1 || { echo "diag failed"; cat gpurun_out/diag.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_diag" -o diag --output-format csv -- python3 -c "
import sys; sys.path.insert(0, '$R')
from kubernetes_amd.ops import hip_kernels as h
print(h.diag_mfma(0,8192,10)); print(h.diag_hbm(0,1<<30,20))" > "$R/gpurun_out/prof_diag.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_diag.log"; exit 1; }
cat "$R/gpurun_out/gpu_ops.log" | tail -3; cat "$R/gpurun_out/vadd.log" "$R/gpurun_out/xgmi.log" "$R/gpurun_out/diag.log"
echo ALL_OK
