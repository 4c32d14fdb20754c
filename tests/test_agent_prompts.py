"""AgentVerse prompt templates are workload contract data (reference
agents/agent_a/prompts.py:8-192): pin every template's placeholders and length, the 5-role
vocabulary and the weighted-criteria evaluation text, so a rewrite that changes the config-4
request sizes fails here."""
import string

from agentic_traffic_testing_amd.agents.agent_a import orchestrator as O
from agentic_traffic_testing_amd.agents.agent_a import prompts as P

# template -> (placeholders, character count of the reference text)
EXPECTED = {
    "EXPERT_RECRUITMENT_PROMPT": ({"task", "feedback_context"}, 1131),
    "HORIZONTAL_DISCUSSION_PROMPT": ({"role", "contract", "task", "discussion_history",
                                      "round_num"}, 434),
    "VERTICAL_SOLVER_PROMPT": ({"contract", "task", "previous_proposal", "critiques"}, 214),
    "VERTICAL_REVIEWER_PROMPT": ({"role", "contract", "task", "proposal"}, 417),
    "EXECUTION_PROMPT": ({"role", "contract", "task", "subtask", "decision_context"}, 266),
    "EVALUATION_PROMPT": ({"task", "results", "iteration", "max_iterations",
                           "success_threshold"}, 2297),
    "FINAL_SYNTHESIS_PROMPT": ({"task", "iteration_summary", "results", "evaluation"}, 936),
    "SYNTHESIZE_DISCUSSION_PROMPT": ({"task", "discussion_history"}, 220),
}


def _fields(t: str) -> set:
    return {f for _, f, _, _ in string.Formatter().parse(t) if f}


def test_templates_placeholders_and_sizes():
    for name, (fields, size) in EXPECTED.items():
        t = getattr(P, name)
        assert _fields(t) == fields, name
        # within a few characters of the reference text (whitespace-only differences)
        assert abs(len(t) - size) <= 4, (name, len(t), size)


def test_role_vocabulary_and_weights():
    assert P.ROLES == ("planner", "researcher", "executor", "critic", "summarizer")
    assert "Choose from: planner, researcher, executor, critic, summarizer" in \
        P.EXPERT_RECRUITMENT_PROMPT
    assert abs(sum(P.CRITERIA_WEIGHTS.values()) - 1.0) < 1e-9
    for k, w in P.CRITERIA_WEIGHTS.items():
        assert f"{k.capitalize()}: {int(w * 100)}%" in P.EVALUATION_PROMPT
    assert "[CONSENSUS]" in P.HORIZONTAL_DISCUSSION_PROMPT
    assert "[APPROVED]" in P.VERTICAL_REVIEWER_PROMPT


def test_evaluation_prompt_carries_threshold():
    st = O.AgentVerseState(task_id="t", original_task="do it", max_iterations=3,
                           success_threshold=90)
    orch = O.AgentVerseOrchestrator.__new__(O.AgentVerseOrchestrator)
    orch.max_model_len, orch.eval_max_tokens, orch.margin = 0, 0, 0
    orch.eval_max_chars = 10 ** 6
    orch._tok = None
    prompt = orch.build_evaluation_prompt(st, "[planner]:\nplan")[0]
    assert "Success threshold (score to accept and stop): 90/100" in prompt
    assert "when score < 90 so" in prompt


def test_oracle_evaluation_weighted():
    ev = O.oracle_evaluation("task", 0, threshold=90)
    crit = ev["criteria"]
    assert set(crit) == set(P.CRITERIA_WEIGHTS)
    assert all(0 <= v <= 100 for v in crit.values())
    assert ev["score"] == round(sum(P.CRITERIA_WEIGHTS[k] * v for k, v in crit.items()))
    assert ev["goal_achieved"] == (ev["score"] >= 90)
