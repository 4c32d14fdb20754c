#!/usr/bin/env bash
# Repeatable AgentVerse experiment.  Same flags as the reference:
#   ./run_experiment.sh -n <iterations> [-o DIR] [-a AGENT_A_URL] [-p PROM_URL] [-w WAIT_S]
#   ./run_experiment.sh -c -o <existing-experiment-dir>        # resume after a crash
# Output: data/runs/experiment_<ts>/{runs.jsonl, summary.txt, metrics.csv, <run>/..., plots/}
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
PY=python3; [[ -x "${ROOT}/.venv/bin/python3" ]] && PY="${ROOT}/.venv/bin/python3"
cd "${ROOT}"
exec "${PY}" -m agentic_traffic_testing_amd.experiments.runner "$@"
