#!/usr/bin/env bash
# Long supervised experiment: settle 300 s, run, auto-resume on crash or
# stall.  Usage: ./run_aggregated_experiment.sh <iterations> [-o DIR]
# The supervisor runs detached (nohup); follow data/runs/<exp>/supervisor.log.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
N="${1:?usage: $0 <iterations> [-o DIR]}"; shift
cd "${ROOT}"
mkdir -p data
nohup python3 -m agentic_traffic_testing_amd.experiments.supervise run -n "${N}" "$@" \
  > data/supervisor.out 2>&1 &
echo "[runner] supervisor pid $! (log: data/supervisor.out, state: data/.experiment_state.json)"
