// Rendering of the stage timeline, live event log, request-flow graph, request table,
// history list and final output.
const R = {
  stages(run) {
    const box = U.$('#stages');
    box.innerHTML = '';
    for (const s of AV_CONFIG.stages) {
      const st = run.stages[s.id] || {};
      const cls = st.done ? 'done' : st.active ? 'active' : 'idle';
      let detail = '';
      if (s.id === 'recruitment' && st.data && st.data.experts) detail = st.data.experts.map((e) => e.role).join(', ') + ` · ${st.data.communication_structure || ''}`;
      if (s.id === 'decision' && st.data) detail = `${st.data.structure || ''} · rounds ${U.nz(st.data.rounds, '–')} · consensus ${st.data.consensus_reached ? 'yes' : 'no'}`;
      if (s.id === 'execution' && st.data) detail = `${U.nz(st.data.success_count, 0)}/${U.nz(st.data.total, 0)} succeeded`;
      if (s.id === 'evaluation' && st.data) detail = `score ${U.nz(st.data.score, '–')} · ${st.data.goal_achieved ? 'goal achieved' : st.data.should_iterate ? 'iterate' : ''}`;
      box.appendChild(U.el('div', { class: `stage ${cls}` },
        U.el('div', { class: 'stage-n' }, String(s.n)),
        U.el('div', { class: 'stage-body' }, U.el('div', { class: 'stage-title' }, s.title),
          U.el('div', { class: 'stage-detail' }, detail || (st.message || '')))));
    }
    U.$('#iteration').textContent = run.iteration ? `iteration ${run.iteration}` : '';
  },

  event(name, data) {
    const log = U.$('#events');
    const summary = (() => {
      if (!data || typeof data !== 'object') return String(U.nz(data, ''));
      if (name === 'llm_request' || name === 'llm_error') return `${data.stage || ''} · ${data.label || ''} → ${U.hostOf(data.endpoint)}${data.error ? ' · ERROR ' + data.error : ''}`;
      if (name === 'stage_start' || name === 'iteration_start') return data.message || data.stage;
      if (name === 'stage_complete') return `${data.stage} complete`;
      if (name === 'execution_result') return `${data.expert} ${data.success ? 'ok' : 'failed'} (${data.completed}/${data.total})`;
      if (name === 'discussion_round') return `round ${data.round} · consensus ${data.consensus ? 'yes' : 'no'}`;
      if (name === 'vertical_iteration') return `solver iteration ${data.solver_iteration} · approved ${data.all_approved ? 'yes' : 'no'}`;
      if (name === 'workflow_error' || name === 'error') return data.error || 'error';
      return data.message || '';
    })();
    const t = new Date().toLocaleTimeString();
    log.prepend(U.el('div', { class: `ev ev-${name}` }, U.el('span', { class: 'ev-t' }, t),
      U.el('span', { class: 'ev-n' }, name), U.el('span', { class: 'ev-s' }, summary)));
  },

  requests(run) {
    const tb = U.$('#requests tbody');
    tb.innerHTML = '';
    for (const r of run.requests) {
      const row = U.el('tr', { class: r.error ? 'err' : '' },
        U.el('td', {}, String(U.nz(r.seq, ''))), U.el('td', {}, String(U.nz(r.iteration, ''))),
        U.el('td', {}, r.stage || ''), U.el('td', {}, r.label || ''),
        U.el('td', {}, r.agent_role || r.source || ''), U.el('td', {}, U.hostOf(r.endpoint)),
        U.el('td', {}, U.fmtSecs(r.duration_seconds)),
        U.el('td', {}, r.llm_meta && r.llm_meta.completion_tokens !== undefined ? `${r.llm_meta.prompt_tokens}/${r.llm_meta.completion_tokens}` : ''),
        U.el('td', {}, r.error ? 'error' : 'ok'));
      const detail = U.el('tr', { class: 'detail hidden' }, U.el('td', { colspan: '9' },
        U.el('div', { class: 'io' }, U.el('h4', {}, 'Prompt'), U.el('pre', {}, r.prompt || '')),
        U.el('div', { class: 'io' }, U.el('h4', {}, 'Response'), U.el('pre', {}, r.response || r.error || '')),
        r.request_id ? U.el('div', { class: 'meta' }, `request_id ${r.request_id}`) : null));
      row.addEventListener('click', () => detail.classList.toggle('hidden'));
      tb.appendChild(row);
      tb.appendChild(detail);
    }
    U.$('#req-count').textContent = `${run.requests.length} LLM calls`;
  },

  // Request-flow graph: Agent A in the middle, one node per endpoint (Agent B workers and
  // the LLM backend), edges weighted by call count, coloured by stage.
  graph(run) {
    const svg = U.$('#flow');
    const W = svg.clientWidth || 520, H = 260;
    svg.setAttribute('viewBox', `0 0 ${W} ${H}`);
    svg.innerHTML = '';
    const targets = {};
    for (const r of run.requests) {
      const key = r.source && r.source.startsWith('agent-b') ? r.source : U.hostOf(r.endpoint) || 'llm';
      targets[key] = targets[key] || { n: 0, err: 0, stages: {} };
      targets[key].n += 1;
      if (r.error) targets[key].err += 1;
      targets[key].stages[r.stage] = (targets[key].stages[r.stage] || 0) + 1;
    }
    const names = Object.keys(targets);
    const cx = 90, cy = H / 2;
    const ns = 'http://www.w3.org/2000/svg';
    const mk = (tag, attrs) => { const n = document.createElementNS(ns, tag); for (const [k, v] of Object.entries(attrs)) n.setAttribute(k, v); return n; };
    names.forEach((name, i) => {
      const y = names.length === 1 ? cy : 30 + (i * (H - 60)) / (names.length - 1);
      const x = W - 130;
      const t = targets[name];
      svg.appendChild(mk('line', { x1: cx + 40, y1: cy, x2: x - 8, y2: y, class: t.err ? 'edge err' : 'edge', 'stroke-width': Math.min(1 + t.n, 9) }));
      const lab = mk('text', { x: (cx + x) / 2, y: (cy + y) / 2 - 4, class: 'edge-label' });
      lab.textContent = `${t.n}× ${Object.keys(t.stages).join('/')}`;
      svg.appendChild(lab);
      svg.appendChild(mk('rect', { x: x - 8, y: y - 14, width: 130, height: 28, rx: 6, class: 'node' }));
      const tx = mk('text', { x: x + 4, y: y + 5, class: 'node-label' });
      tx.textContent = name;
      svg.appendChild(tx);
    });
    svg.appendChild(mk('circle', { cx, cy, r: 40, class: 'node hub' }));
    const a = mk('text', { x: cx, y: cy + 5, class: 'node-label', 'text-anchor': 'middle' });
    a.textContent = 'Agent A';
    svg.appendChild(a);
  },

  final(result) {
    const box = U.$('#final');
    if (!result) { box.textContent = ''; return; }
    const status = result.completed ? 'completed' : result.partial ? 'partial' : 'not completed';
    U.$('#final-meta').textContent = `task ${result.task_id} · ${status} · ${U.nz(result.iterations, '?')} iteration(s) · ${U.fmtSecs(result.duration_seconds)}${result.workflow_error ? ' · error: ' + result.workflow_error : ''}`;
    box.textContent = result.final_output || '';
    const hist = U.$('#iterations');
    hist.innerHTML = '';
    for (const h of result.iteration_history || []) {
      const ev = h.evaluation || {};
      hist.appendChild(U.el('li', {}, `iteration ${h.iteration}: score ${U.nz(ev.score, '–')}${ev.goal_achieved ? ' ✓' : ''} — ${U.truncate(ev.feedback || ev.rationale || '', 140)}`));
    }
  },

  history(onOpen, onForget) {
    const ul = U.$('#history');
    ul.innerHTML = '';
    for (const h of State.history()) {
      const li = U.el('li', {},
        U.el('a', { href: `?task_id=${encodeURIComponent(h.task_id)}`, onclick: (e) => { e.preventDefault(); onOpen(h.task_id); } }, U.truncate(h.task || h.task_id, 60)),
        U.el('span', { class: 'h-meta' }, ` ${h.completed ? '✓' : '…'} ${new Date(h.at).toLocaleString()}`),
        U.el('button', { class: 'x', title: 'forget', onclick: () => onForget(h.task_id) }, '×'));
      ul.appendChild(li);
    }
  },
};
