#!/bin/bash
# GPU box: GPU tests, driver smoke, 1-GPU bench, then a rocprofv3 kernel-trace/stats pass of the
# bench. Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r3
export TMPDIR=/tmp
step() { local name=$1; shift; echo "== $name"; "$@" > "gpurun_out/r3/$name.log" 2>&1; local rc=$?; tail -4 "gpurun_out/r3/$name.log" | cut -c1-600; if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -40 "gpurun_out/r3/$name.log"; exit $rc; fi; }
step pytest_gpu timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5
step rocprof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof -o run -- python3 bench.py --steps 5 --warmup 2
find gpurun_out/r3/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/r3/kernel_stats.csv \;
echo ALL_OK
