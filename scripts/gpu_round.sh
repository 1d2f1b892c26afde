#!/bin/bash
# One GPU-box pass: GPU tests, the xGMI probe, a short bench. Later GPU steps run only when the
# earlier one ended normally (pytest 0 = pass, 1 = test failures); a timeout (124/137), an abort
# (134) or a crash (139) ends the pass there.
out=${1:-gpurun_out/pass}
mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$out/gputests.log" 2>&1
rc=$?
echo "pytest rc=$rc" > "$out/status.txt"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 60 kubernetes_amd/native/bin/xgmi-probe 64 > "$out/xgmi.json" 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || exit $?
exit $rc
