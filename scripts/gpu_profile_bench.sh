#!/bin/bash
# GPU box: cProfile every bench process (rank, API server, scheduler) for one 1-GPU bench run,
# then print the top functions of each profile (self time and cumulative).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/prof
export KAMD_PROFILE_DIR=$R/gpurun_out/prof
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/prof/bench.log 2>&1 || { tail -30 gpurun_out/prof/bench.log; exit 1; }
grep metric gpurun_out/prof/bench.log | cut -c1-400
for f in gpurun_out/prof/*.prof; do
  python - "$f" > "${f%.prof}.txt" <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1])
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(70)
PY
done
ls gpurun_out/prof
