#!/bin/bash
# PMC passes (one counter set per run) for the ping-pong GEMM (path 0/3) vs the 8-phase kernel (7) at 8192^3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmcpp
cat > /tmp/pprun.py <<PY
import sys; sys.path.insert(0, "$R")
from kubernetes_amd.ops import hip_kernels as h
h.set_gemm_path(int(sys.argv[1])); print(h.diag_mfma(0, 8192, 3))
PY
cd /tmp && export TMPDIR=/tmp
for path in 3 7; do
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_LDS_CMD_FIFO_FULL SQ_WAVES --output-format csv -d $R/gpurun_out/pmcpp/p$path -o run -- python3 /tmp/pprun.py $path > $R/gpurun_out/pmcpp/p$path.log 2>&1 || exit 1
done
find $R/gpurun_out/pmcpp -name "*.csv" | head
