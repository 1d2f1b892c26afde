set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc
cat > /tmp/g8run.py <<PY
import sys; sys.path.insert(0, "$R")
from kubernetes_amd.ops import hip_kernels as h
h.set_gemm_path(int(sys.argv[1])); print(h.diag_mfma(0, 8192, 3))
PY
cd /tmp && export TMPDIR=/tmp
for path in 0 2; do
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_WAVES -d $R/gpurun_out/pmc/a$path -o run -- python3 /tmp/g8run.py $path > $R/gpurun_out/pmc/a$path.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc/b$path -o run -- python3 /tmp/g8run.py $path > $R/gpurun_out/pmc/b$path.log 2>&1 || exit 1
done
ls -R $R/gpurun_out/pmc | head -30
