#!/bin/bash
# One GPU-box pass: GPU tests, the graft smoke, the xGMI probe, the driver's bench command and a
# rocprofv3 kernel-trace of a short bench. A later GPU step runs only when the earlier one ended
# normally (pytest 0 = pass, 1 = test failures); a timeout (124/137), an abort (134) or a crash
# (139) ends the pass there.
out=${1:-gpurun_out/pass}
mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$out/gputests.log" 2>&1
rc=$?
echo "pytest rc=$rc" > "$out/status.txt"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit $?
echo "smoke ok" >> "$out/status.txt"
timeout -k 10 60 kubernetes_amd/native/bin/xgmi-probe 64 > "$out/xgmi.json" 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || exit $?
echo "bench ok" >> "$out/status.txt"
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/rocprof" -o run -- python3 bench.py --steps 5 --warmup 2 > "$out/rocprof_bench.json" 2> "$out/rocprof.err" || exit $?
  echo "rocprof ok" >> "$out/status.txt"
fi
exit $rc
