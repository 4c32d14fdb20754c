// AgentVerse SPA wiring: run a task (SSE with JSON fallback), reload persisted runs by
// task id (GET /agentverse/<id>, also via ?task_id= / ?taskId=), local history.
(function () {
  const endpointInput = U.$('#endpoint');
  endpointInput.value = localStorage.getItem('agentverse.endpoint') || AV_CONFIG.defaultEndpoint;
  let controller = null;

  function status(msg, cls = '') { const s = U.$('#status'); s.textContent = msg; s.className = cls; }

  function applyEvent(name, data) {
    const run = State.run;
    run.events.push({ name, data });
    R.event(name, data);
    if (name === 'iteration_start') run.iteration = (data.iteration || 0) + 1;
    if (name === 'stage_start') {
      run.iteration = data.iteration || run.iteration;
      for (const s of Object.keys(run.stages)) run.stages[s].active = false;
      run.stages[data.stage] = { ...(run.stages[data.stage] || {}), active: true, done: false, message: data.message };
    }
    if (name === 'stage_complete') run.stages[data.stage] = { active: false, done: true, data };
    if (name === 'llm_request' || name === 'llm_error') State.addRequest(data);
    if (name === 'complete') {
      run.result = data;
      for (const r of data.llm_requests || []) State.addRequest(r);
      State.remember(data);
      R.final(data);
      R.history(openTask, forgetTask);
    }
    R.stages(run);
    R.requests(run);
    R.graph(run);
  }

  async function start() {
    const task = U.$('#task').value.trim();
    if (!task) { status('enter a task first', 'warn'); return; }
    const endpoint = endpointInput.value.trim();
    localStorage.setItem('agentverse.endpoint', endpoint);
    State.reset(task);
    U.$('#events').innerHTML = '';
    R.final(null);
    R.stages(State.run);
    controller = new AbortController();
    U.$('#run').disabled = true;
    U.$('#stop').disabled = false;
    status('running…', 'busy');
    const payload = { task, max_iterations: Number(U.$('#max-iter').value) || 3, success_threshold: Number(U.$('#threshold').value) || 90 };
    try {
      if (!U.$('#stream').checked) {
        const resp = await fetch(endpoint, { method: 'POST', headers: { 'Content-Type': 'application/json' }, body: JSON.stringify({ ...payload, stream: false }), signal: controller.signal });
        if (!resp.ok) throw new Error(`HTTP ${resp.status}`);
        applyEvent('complete', await resp.json());
      } else {
        await runAgentverse({ endpoint, payload, onEvent: applyEvent, signal: controller.signal });
      }
      status(`done in ${((Date.now() - State.run.started) / 1000).toFixed(1)} s`, 'ok');
      history.replaceState(null, '', `?task_id=${encodeURIComponent(State.run.result.task_id)}`);
    } catch (err) {
      status(`failed: ${err.message}`, 'error');
      R.event('error', { error: err.message });
    } finally {
      U.$('#run').disabled = false;
      U.$('#stop').disabled = true;
    }
  }

  async function openTask(taskId) {
    status(`loading ${taskId}…`, 'busy');
    try {
      const rec = await loadAgentverseRun(endpointInput.value.trim(), taskId);
      const result = rec.result || rec;
      State.reset(result.original_task || '');
      U.$('#task').value = result.original_task || '';
      U.$('#events').innerHTML = '';
      for (const [k, v] of Object.entries(result.stages || {})) State.run.stages[k] = { done: true, data: v };
      applyEvent('complete', result);
      status(`loaded ${taskId}`, 'ok');
      history.replaceState(null, '', `?task_id=${encodeURIComponent(taskId)}`);
    } catch (err) {
      status(`could not load ${taskId}: ${err.message}`, 'error');
    }
  }

  function forgetTask(taskId) { State.forget(taskId); R.history(openTask, forgetTask); }

  U.$('#run').addEventListener('click', start);
  U.$('#stop').addEventListener('click', () => controller && controller.abort());
  U.$('#load').addEventListener('click', () => { const id = U.$('#load-id').value.trim(); if (id) openTask(id); });
  U.$('#clear-history').addEventListener('click', () => { State.clearHistory(); R.history(openTask, forgetTask); });
  U.$('#example').addEventListener('change', (e) => { if (e.target.value) U.$('#task').value = e.target.value; });
  fetch('./templates/agentverse_workflow.json').then((r) => (r.ok ? r.json() : null)).then((wf) => {
    if (!wf) return;
    for (const t of wf.example_tasks || []) U.$('#example').appendChild(U.el('option', { value: t.task }, t.name));
    if (wf.workflow_config) U.$('#max-iter').value = wf.workflow_config.max_iterations || 3;
  }).catch(() => {});
  State.reset('');
  R.stages(State.run);
  R.graph(State.run);
  R.history(openTask, forgetTask);
  const initial = U.queryParam('task_id') || U.queryParam('taskId');
  if (initial) openTask(initial);
})();
