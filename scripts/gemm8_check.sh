set -o pipefail
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gemm8_tests.log 2>&1 || { tail -40 gpurun_out/gemm8_tests.log; exit 1; }
tail -3 gpurun_out/gemm8_tests.log
timeout -k 10 300 python -u scripts/gemm_ab.py > gpurun_out/gemm8_ab.log 2>&1 || { cat gpurun_out/gemm8_ab.log; exit 1; }
cat gpurun_out/gemm8_ab.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof8 -o run -- python3 -c "
import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from kubernetes_amd.ops import hip_kernels as h
h.set_gemm_path(0); print(h.diag_mfma(0, 8192, 10))
h.set_gemm_path(2); print(h.diag_mfma(0, 8192, 10))
" > $GRAFT_REPO_ROOT/gpurun_out/prof8.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof8.log; exit 1; }
tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof8.log
echo DONE
