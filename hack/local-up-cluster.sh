#!/bin/bash
# Start a single-node MI355X cluster from this checkout (all components as separate processes).
# Usage: hack/local-up-cluster.sh [--fake-gpus N] [--runtime process|stub] [--workdir DIR]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
python -m kubernetes_amd.native.build >/dev/null
cd "$ROOT" && exec python -m kubernetes_amd.cmd.local_up "$@"
