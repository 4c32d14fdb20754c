#!/usr/bin/env bash
# Minimal scenario smoke run (the reference's MVP runner only echoed placeholders, SURVEY
# §2.2 E7): send one task per /task scenario through Agent A and print the aggregates.
#   ./run_mvp_experiment.sh [agentic_simple|agentic_multi_hop|agentic_parallel|all] [AGENT_A_URL]
set -euo pipefail
SCEN="${1:-all}"; URL="${2:-http://localhost:8101/task}"
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
run() {
  echo "=== scenario $1"
  python3 "${ROOT}/scripts/experiment/query_agent.py" a "Plan a three-day team offsite on a small budget." \
    --scenario "$1" --url "${URL}" --timeout 600 |
    python3 -c 'import json,sys; d=json.load(sys.stdin); print({k: d.get(k) for k in ("task_id","total_llm_calls","total_tokens","total_latency_ms","total_agent_hops")})'
}
case "${SCEN}" in
  all) for s in agentic_simple agentic_multi_hop agentic_parallel; do run "$s"; done ;;
  *) run "${SCEN}" ;;
esac
