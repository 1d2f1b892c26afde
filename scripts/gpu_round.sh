#!/bin/bash
# GPU box: GPU tests, driver smoke, 1-GPU bench. Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; echo "== $name"; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -5 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; fi; }
step pytest_gpu timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 timeout -k 10 600 python bench.py --steps 5 --warmup 2
echo ALL_OK
