"""Every module path of the reference tree resolves in this repo (a user switching from the
reference keeps their ``python -m ...`` commands and imports)."""
import importlib
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# reference file -> importable module path
MODULES = [
    "llm.serve_llm", "llm.hf_cpu_server", "llm.tracing",
    "agents.agent_a.server", "agents.agent_a.main", "agents.agent_a.orchestrator",
    "agents.agent_a.prompts", "agents.agent_b.server", "agents.agent_b.main",
    "agents.common.telemetry", "agents.common.metrics_logger", "agents.common.tracing",
    "agents.common.mcp_client",
    "tools.mcp_tool_db.server", "tools.mcp_servers.coding_server",
    "tools.mcp_servers.finance_server", "tools.mcp_servers.maps_server",
    "tools.mcp_universe.openai_proxy",
]


@pytest.mark.parametrize("mod", MODULES)
def test_reference_module_imports(mod):
    importlib.import_module(mod)


def test_alias_modules_are_the_implementation():
    import agents.agent_a.prompts as p
    import agents.common.telemetry as t
    from agentic_traffic_testing_amd.agents.agent_a import prompts
    from agentic_traffic_testing_amd.agents.common import telemetry

    assert p is prompts and t is telemetry
    for name in ("EXPERT_RECRUITMENT_PROMPT", "HORIZONTAL_DISCUSSION_PROMPT",
                 "VERTICAL_SOLVER_PROMPT", "VERTICAL_REVIEWER_PROMPT", "EXECUTION_PROMPT",
                 "EVALUATION_PROMPT", "FINAL_SYNTHESIS_PROMPT", "SYNTHESIZE_DISCUSSION_PROMPT"):
        assert isinstance(getattr(p, name), str)


def test_llm_tracing_init():
    import llm.tracing

    tr = llm.tracing.init_tracer("llm-backend")
    with tr.start_as_current_span("probe") as sp:
        assert sp.get_span_context().trace_id


@pytest.mark.parametrize("name", [
    "agentverse_workflow.json", "mas_agent_contracts_simple.json",
    "mas_agent_contracts_enhanced.json", "mas_agent_contracts_debate.json",
    "mas_agent_contracts_auction.json"])
def test_templates_at_reference_path(name):
    import json

    with open(os.path.join(ROOT, "agents", "templates", name)) as f:
        json.load(f)
