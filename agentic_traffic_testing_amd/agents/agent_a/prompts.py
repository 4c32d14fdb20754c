"""Prompt templates for the AgentVerse workflow (role of reference agents/agent_a/prompts.py).

Eight templates drive the 4-stage loop (recruitment, horizontal discussion, vertical
solver / reviewer, execution, evaluation, discussion synthesis, final synthesis).  The
wording is this repo's own; what the workflow depends on is preserved: the JSON schemas
the parsers expect (``experts`` / ``communication_structure`` / ``execution_order`` /
``reasoning`` for recruitment; ``goal_achieved`` / ``score`` / ``criteria`` / ``rationale``
/ ``feedback`` / ``missing_aspects`` / ``should_iterate`` for evaluation) and the
``[CONSENSUS]`` / ``[APPROVED]`` markers the discussion loops look for.
"""

RECRUITMENT = """You coordinate a team of specialist agents. Study the task and decide which \
experts (between 2 and 5) should work on it and how they should communicate.

Task:
{task}
{feedback_context}
Communication structures:
- "horizontal": every expert contributes to an open discussion until they agree.
- "vertical": one solver drafts a plan, the other experts review it, the solver revises.

Reply with JSON only:
{{
  "experts": [
    {{"role": "<short role name>", "responsibilities": "<what this expert covers>",
      "contract": "<instructions that bind this expert>"}}
  ],
  "communication_structure": "horizontal" or "vertical",
  "execution_order": ["<role>", "..."],
  "reasoning": "<one or two sentences on why this team and structure>"
}}"""

HORIZONTAL_DISCUSSION = """Role: {role}
Contract: {contract}

Team task:
{task}

Discussion so far (round {round_num}):
{discussion_history}

Add your view: propose concrete steps, point out problems with earlier suggestions and \
refine them. If you agree with the current plan and have nothing to add, end your message \
with [CONSENSUS]."""

VERTICAL_SOLVER = """You are the solver for this team.
Contract: {contract}

Task:
{task}
{previous_proposal}{critiques}
Write a complete, step-by-step proposal that solves the task. If reviewer critiques are \
shown above, address every one of them explicitly."""

VERTICAL_REVIEWER = """Role: {role} (reviewer)
Contract: {contract}

Task:
{task}

Proposal under review:
{proposal}

Check the proposal for errors, gaps and risks from your role's point of view and list \
specific fixes. If the proposal is acceptable as written, end your reply with [APPROVED]."""

EXECUTION = """Role: {role}
Contract: {contract}

Overall task:
{task}

Agreed approach (excerpt):
{decision_context}

Your assignment:
{subtask}

Carry out your assignment now and report the concrete result."""

EVALUATION = """You are the evaluator of a multi-agent run. Judge whether the team's \
combined output accomplishes the task.

Task:
{task}

Iteration: {iteration} of {max_iterations}

Outputs from the experts:
{results}

Score each criterion from 0 to 20 (completeness, correctness, clarity, relevance, \
actionability); the overall score is their sum (0-100).  Reply with JSON only:
{{
  "goal_achieved": true or false,
  "score": <0-100>,
  "criteria": {{"completeness": <0-20>, "correctness": <0-20>, "clarity": <0-20>,
               "relevance": <0-20>, "actionability": <0-20>}},
  "rationale": "<how the score was reached>",
  "feedback": "<what the next iteration should change>",
  "missing_aspects": ["<gap>", "..."],
  "should_iterate": true or false
}}"""

SYNTHESIZE_DISCUSSION = """Summarise the team discussion below into one decision the \
experts can execute.

Task:
{task}

Discussion transcript:
{discussion_history}

State the agreed approach as a numbered plan and note any point that is still disputed."""

FINAL_SYNTHESIS = """Produce the final answer for the user from the team's work.

Task:
{task}

Iterations:
{iteration_summary}

Expert results:
{results}

Last evaluation:
{evaluation}

Write one coherent, self-contained response that answers the task directly."""

# reference-style aliases (agents/agent_a/prompts.py names)
EXPERT_RECRUITMENT_PROMPT = RECRUITMENT
HORIZONTAL_DISCUSSION_PROMPT = HORIZONTAL_DISCUSSION
VERTICAL_SOLVER_PROMPT = VERTICAL_SOLVER
VERTICAL_REVIEWER_PROMPT = VERTICAL_REVIEWER
EXECUTION_PROMPT = EXECUTION
EVALUATION_PROMPT = EVALUATION
FINAL_SYNTHESIS_PROMPT = FINAL_SYNTHESIS
SYNTHESIZE_DISCUSSION_PROMPT = SYNTHESIZE_DISCUSSION
