#!/bin/bash
# PMC passes (one counter set per run) for the fp8 block-scaled ping-pong GEMM vs the bf16 one at
# 8192^3, plus a GRBM pass whose GUI_ACTIVE cycles over the kernel time give the effective clock.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc8
cat > /tmp/f8run.py <<PY
import sys; sys.path.insert(0, "$R")
from kubernetes_amd.ops import hip_kernels as h
print(h.diag_mfma_fp8(0, 8192, 3) if sys.argv[1] == "fp8" else h.diag_mfma(0, 8192, 3))
PY
cd /tmp && export TMPDIR=/tmp
for kind in fp8 bf16; do
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_LDS_CMD_FIFO_FULL SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc8/$kind -o run -- python3 /tmp/f8run.py $kind > $R/gpurun_out/pmc8/$kind.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc8/${kind}_grbm -o run -- python3 /tmp/f8run.py $kind > $R/gpurun_out/pmc8/${kind}_grbm.log 2>&1 || exit 1
done
find $R/gpurun_out/pmc8 -name "*.csv" | head -20
