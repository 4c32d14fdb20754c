// AgentVerse SPA wiring: run a task (SSE with JSON fallback), cancel it, reload persisted
// runs by task id (GET /agentverse/<id>, also via ?task_id= / ?taskId=), local history,
// run timer + LLM-call counter, flow-view toggles, copy / raw-JSON views.
(function () {
  const endpointInput = U.$('#endpoint');
  endpointInput.value = localStorage.getItem('agentverse.endpoint') || AV_CONFIG.defaultEndpoint;
  let controller = null;
  let ticker = null;

  function status(msg, cls = '') { const s = U.$('#status'); s.textContent = msg; s.className = cls; }

  function tick() { if (State.run) R.timer(State.run); }
  function startTimer() { stopTimer(); ticker = setInterval(tick, 250); }
  function stopTimer() { if (ticker) clearInterval(ticker); ticker = null; tick(); }

  function applyEvent(name, data) {
    State.apply(name, data);
    if (name !== 'complete') R.event(name, data);
    if (name === 'complete') {
      State.remember(data);
      R.final(data);
      R.history(openTask, forgetTask);
    }
    R.all(State.run);
  }

  function setRunning(on) {
    U.$('#run').disabled = on;
    U.$('#stop').disabled = !on;
    document.body.classList.toggle('running', on);
  }

  async function start() {
    const task = U.$('#task').value.trim();
    if (!task) { status('enter a task first', 'warn'); return; }
    const endpoint = endpointInput.value.trim();
    localStorage.setItem('agentverse.endpoint', endpoint);
    State.reset(task);
    State.run.status = 'running';
    U.$('#events').innerHTML = '';
    R.final(null);
    R.all(State.run);
    controller = new AbortController();
    setRunning(true);
    startTimer();
    status('running…', 'busy');
    const payload = {
      task, max_iterations: Number(U.$('#max-iter').value) || 3,
      success_threshold: Number(U.$('#threshold').value) || 90,
    };
    try {
      if (!U.$('#stream').checked) {
        const resp = await fetch(endpoint, { method: 'POST', headers: { 'Content-Type': 'application/json' }, body: JSON.stringify({ ...payload, stream: false }), signal: controller.signal });
        if (!resp.ok) throw new Error(`HTTP ${resp.status}`);
        applyEvent('complete', await resp.json());
      } else {
        await runAgentverse({ endpoint, payload, onEvent: applyEvent, signal: controller.signal });
      }
      status(`done in ${runElapsed(State.run).toFixed(1)} s · ${State.run.llmCalls} LLM calls`, 'ok');
      if (State.run.result && State.run.result.task_id) history.replaceState(null, '', `?task_id=${encodeURIComponent(State.run.result.task_id)}`);
    } catch (err) {
      if (controller && controller.signal.aborted) {
        applyEvent('cancelled', { message: 'cancelled by the user' });
        status(`cancelled after ${runElapsed(State.run).toFixed(1)} s (the server finishes the run; reload it by task id)`, 'warn');
      } else {
        applyEvent('error', { error: err.message });
        status(`failed: ${err.message}`, 'error');
      }
    } finally {
      controller = null;
      setRunning(false);
      stopTimer();
    }
  }

  // Cancel: abort the fetch / SSE stream (the request's AbortController).  Agent A keeps
  // running the workflow server-side and persists it, so it can be reloaded by task id.
  function cancel() {
    if (controller) controller.abort();
  }

  async function openTask(taskId) {
    status(`loading ${taskId}…`, 'busy');
    try {
      const rec = await loadAgentverseRun(endpointInput.value.trim(), taskId);
      const result = rec.result || rec;
      State.reset(result.original_task || '');
      U.$('#task').value = result.original_task || '';
      U.$('#events').innerHTML = '';
      applyEvent('complete', result);
      State.run.finished = State.run.started + 1000 * (result.duration_seconds || 0);
      R.timer(State.run);
      status(`loaded ${taskId}`, 'ok');
      history.replaceState(null, '', `?task_id=${encodeURIComponent(taskId)}`);
    } catch (err) {
      status(`could not load ${taskId}: ${err.message}`, 'error');
    }
  }

  function forgetTask(taskId) { State.forget(taskId); R.history(openTask, forgetTask); }

  U.$('#run').addEventListener('click', start);
  U.$('#stop').addEventListener('click', cancel);
  document.addEventListener('keydown', (e) => {
    if (e.key === 'Escape' && controller) cancel();
    if (e.key === 'Enter' && (e.ctrlKey || e.metaKey) && !controller) start();
  });
  U.$('#load').addEventListener('click', () => { const id = U.$('#load-id').value.trim(); if (id) openTask(id); });
  U.$('#clear-history').addEventListener('click', () => { State.clearHistory(); R.history(openTask, forgetTask); });
  U.$('#example').addEventListener('change', (e) => { if (e.target.value) U.$('#task').value = e.target.value; });
  // flow-view toggles: graph / table / stage filter
  U.$('#view-graph').addEventListener('change', (e) => { R.view.graph = e.target.checked; R.graph(State.run); });
  U.$('#view-table').addEventListener('change', (e) => { R.view.table = e.target.checked; R.requests(State.run); });
  U.$('#stage-filter').addEventListener('change', (e) => { R.view.stage = e.target.value; R.requests(State.run); R.graph(State.run); });
  // final output: copy text / task id / JSON, raw JSON view
  U.$('#copy-final').addEventListener('click', () => U.copy(U.$('#final').textContent).then(() => status('final output copied', 'ok')));
  U.$('#copy-id').addEventListener('click', () => State.run && State.run.result && U.copy(State.run.result.task_id).then(() => status('task id copied', 'ok')));
  U.$('#copy-json').addEventListener('click', () => State.run && State.run.result && U.copy(JSON.stringify(State.run.result, null, 2)).then(() => status('result JSON copied', 'ok')));
  U.$('#toggle-raw').addEventListener('click', () => {
    const raw = U.$('#raw');
    raw.classList.toggle('hidden');
    U.$('#toggle-raw').textContent = raw.classList.contains('hidden') ? 'raw JSON' : 'hide JSON';
  });
  U.$('#download-json').addEventListener('click', () => {
    if (!State.run || !State.run.result) return;
    const blob = new Blob([JSON.stringify(State.run.result, null, 2)], { type: 'application/json' });
    const a = U.el('a', { href: URL.createObjectURL(blob), download: `agentverse_${State.run.result.task_id}.json` });
    document.body.appendChild(a); a.click(); a.remove();
  });
  fetch('./templates/agentverse_workflow.json').then((r) => (r.ok ? r.json() : null)).then((wf) => {
    if (!wf) return;
    for (const t of wf.example_tasks || []) U.$('#example').appendChild(U.el('option', { value: t.task }, t.name));
    if (wf.workflow_config) U.$('#max-iter').value = wf.workflow_config.max_iterations || 3;
  }).catch(() => {});
  State.reset('');
  R.all(State.run);
  R.history(openTask, forgetTask);
  window.addEventListener('resize', () => R.graph(State.run));
  const initial = U.queryParam('task_id') || U.queryParam('taskId');
  if (initial) openTask(initial);
})();
