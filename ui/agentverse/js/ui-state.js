// Run state of the AgentVerse SPA: a pure reducer over the workflow's SSE events (also fed
// the non-streamed JSON result), per-iteration snapshots for the history / diff views, the
// run timer and LLM-call counter, and the localStorage history.  No DOM access here, so the
// reducer runs unchanged under node in tests/test_ui.py.
const STAGE_IDS = ['recruitment', 'decision', 'execution', 'evaluation', 'synthesis'];

function newRun(task) {
  return {
    task, events: [], requests: [], stages: {}, iteration: 0, maxIterations: null,
    iterations: {},          // iteration number (1-based) -> snapshot of its stages
    discussion: [],          // rounds of the current iteration: {round, responses[], consensus}
    vertical: [],            // vertical review iterations of the current iteration
    executions: [],          // execution_result events of the current iteration
    result: null, error: null, status: 'idle', started: Date.now(), finished: null,
    llmCalls: 0, llmErrors: 0,
  };
}

function snapshotOf(run, it) {
  if (!run.iterations[it]) run.iterations[it] = { iteration: it, stages: {}, discussion: [], vertical: [], executions: [] };
  return run.iterations[it];
}

// Apply one event (name, data) to the run; returns the run.  Event names and payloads are
// the orchestrator's (agents/agent_a/orchestrator.py module doc) plus the client-side
// 'complete', 'fallback', 'cancelled' and 'error'.
function applyRunEvent(run, name, data) {
  data = data || {};
  run.events.push({ name, data, t: Date.now() });
  const it = () => (data.iteration !== undefined && data.iteration !== null ? data.iteration + 1 : (run.iteration || 1));
  switch (name) {
    case 'iteration_start':
      run.iteration = it();
      if (data.max_iterations) run.maxIterations = data.max_iterations;
      run.discussion = []; run.vertical = []; run.executions = [];
      for (const s of STAGE_IDS) if (s !== 'synthesis') run.stages[s] = { state: 'idle' };
      snapshotOf(run, run.iteration);
      run.status = 'running';
      break;
    case 'stage_start':
      run.iteration = it();
      for (const s of Object.keys(run.stages)) if (run.stages[s].state === 'active') run.stages[s].state = 'idle';
      run.stages[data.stage] = { state: 'active', message: data.message || '' };
      run.status = 'running';
      break;
    case 'stage_complete': {
      run.stages[data.stage] = { state: 'done', data };
      if (data.stage !== 'synthesis') snapshotOf(run, it()).stages[data.stage] = data;
      break;
    }
    case 'discussion_round': {
      const r = { round: data.round, responses: data.responses || [], consensus: !!data.consensus };
      run.discussion.push(r);
      snapshotOf(run, it()).discussion.push(r);
      break;
    }
    case 'vertical_iteration': {
      const v = { ...data };
      run.vertical.push(v);
      snapshotOf(run, it()).vertical.push(v);
      break;
    }
    case 'execution_result':
      run.executions.push(data);
      snapshotOf(run, it()).executions.push(data);
      break;
    case 'llm_request':
    case 'llm_error':
      addRequest(run, data);
      break;
    case 'iteration_complete':
      for (const h of data.iteration_history || []) snapshotOf(run, h.iteration + 1).summary = h;
      break;
    case 'workflow_error':
      run.error = data.error || 'workflow error';
      break;
    case 'complete':
      run.result = data;
      for (const r of data.llm_requests || []) addRequest(run, r);
      for (const h of data.iteration_history || []) snapshotOf(run, h.iteration + 1).summary = h;
      // a loaded (non-streamed) run only has the final iteration's stage details
      if (data.stages) {
        const last = data.iterations || (data.iteration_history || []).length || 1;
        const snap = snapshotOf(run, last);
        for (const [k, v] of Object.entries(data.stages)) if (!snap.stages[k]) snap.stages[k] = v;
        if (!snap.discussion.length && data.stages.decision && data.stages.decision.discussion_rounds) {
          snap.discussion = data.stages.decision.discussion_rounds.map((r) => ({
            round: r.round, responses: r.responses || [], consensus: (r.responses || []).every((x) => x.consensus) }));
        }
        for (const [k, v] of Object.entries(data.stages)) run.stages[k] = { state: 'done', data: v };
      }
      if (data.workflow_error) run.error = data.workflow_error;
      run.status = data.workflow_error ? 'partial' : (data.completed ? 'done' : 'incomplete');
      run.finished = Date.now();
      run.iteration = data.iterations || run.iteration;
      break;
    case 'cancelled':
      run.status = 'cancelled';
      run.finished = Date.now();
      for (const s of Object.keys(run.stages)) if (run.stages[s].state === 'active') run.stages[s].state = 'cancelled';
      break;
    case 'error':
      run.error = data.error || 'error';
      run.status = 'error';
      run.finished = Date.now();
      break;
    default:
      break;
  }
  return run;
}

function addRequest(run, r) {
  const key = r.seq !== undefined && r.seq !== null ? r.seq : run.requests.length + 1;
  const i = run.requests.findIndex((x) => x.seq === key);
  if (i >= 0) run.requests[i] = { ...run.requests[i], ...r, seq: key };
  else run.requests.push({ ...r, seq: key });
  run.llmCalls = run.requests.length;
  run.llmErrors = run.requests.filter((x) => x.error).length;
}

// elapsed seconds of a run (live while running)
function runElapsed(run, now) {
  if (!run) return 0;
  const end = run.finished || now || Date.now();
  return Math.max(0, (end - run.started) / 1000);
}

function fmtClock(sec) {
  const s = Math.floor(sec % 60), m = Math.floor(sec / 60) % 60, h = Math.floor(sec / 3600);
  const pad = (x) => String(x).padStart(2, '0');
  return h ? `${h}:${pad(m)}:${pad(s)}` : `${pad(m)}:${pad(s)}`;
}

const State = {
  run: null,
  reset(task) { this.run = newRun(task); return this.run; },
  apply(name, data) { return applyRunEvent(this.run, name, data); },
  history() {
    try { return JSON.parse(localStorage.getItem(AV_CONFIG.historyKey) || '[]'); } catch (e) { return []; }
  },
  remember(result) {
    if (!result || !result.task_id) return;
    const h = this.history().filter((x) => x.task_id !== result.task_id);
    h.unshift({
      task_id: result.task_id, task: result.original_task || '', completed: !!result.completed,
      iterations: result.iterations, duration: result.duration_seconds, at: Date.now(),
      calls: (result.llm_requests || []).length,
      score: result.stages && result.stages.evaluation ? result.stages.evaluation.score : null,
    });
    localStorage.setItem(AV_CONFIG.historyKey, JSON.stringify(h.slice(0, AV_CONFIG.historyLimit)));
  },
  forget(taskId) {
    localStorage.setItem(AV_CONFIG.historyKey, JSON.stringify(this.history().filter((x) => x.task_id !== taskId)));
  },
  clearHistory() { localStorage.removeItem(AV_CONFIG.historyKey); },
};

if (typeof module !== 'undefined') module.exports = { newRun, applyRunEvent, runElapsed, fmtClock, STAGE_IDS };
