// Rendering of the AgentVerse SPA: stage timeline, live events, request flow (graph and/or
// table with a stage filter), discussion / review panel, evaluation panel, iteration history
// with per-iteration detail and the change diff against the previous iteration, final output
// with copy / raw-JSON views, run timer + LLM-call counter, and the local history list.
const R = {
  view: { graph: true, table: true, stage: '' },

  stages(run) {
    const box = U.$('#stages');
    box.innerHTML = '';
    for (const s of AV_CONFIG.stages) {
      const st = run.stages[s.id] || {};
      const d = st.data || {};
      let detail = '';
      if (s.id === 'recruitment' && d.experts) detail = d.experts.map((e) => e.role || e).join(', ') + ` · ${d.communication_structure || ''}`;
      if (s.id === 'decision' && st.data) detail = `${d.structure_used || d.structure || ''} · rounds ${(d.discussion_rounds || []).length || U.nz(d.rounds, '–')} · consensus ${d.consensus_reached ? 'yes' : 'no'}`;
      if (s.id === 'execution' && st.data) detail = `${U.nz(d.success_count, 0)} ok / ${U.nz(d.failure_count, 0)} failed`;
      if (s.id === 'evaluation' && st.data) detail = `score ${U.nz(d.score, '–')} · ${d.goal_achieved ? 'goal achieved' : 'below threshold'}`;
      box.appendChild(U.el('div', { class: `stage ${st.state || 'idle'}` },
        U.el('div', { class: 'stage-n' }, String(s.n)),
        U.el('div', { class: 'stage-body' }, U.el('div', { class: 'stage-title' }, s.title),
          U.el('div', { class: 'stage-detail' }, detail || st.message || ''))));
    }
    const max = run.maxIterations ? ` / ${run.maxIterations}` : '';
    U.$('#iteration').textContent = run.iteration ? `iteration ${run.iteration}${max}` : '';
  },

  timer(run) {
    U.$('#timer').textContent = fmtClock(runElapsed(run));
    U.$('#llm-count').textContent = `${run.llmCalls} LLM call${run.llmCalls === 1 ? '' : 's'}` +
      (run.llmErrors ? ` · ${run.llmErrors} failed` : '');
    U.$('#run-state').textContent = run.status;
    U.$('#run-state').className = `badge st-${run.status}`;
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
      if (name === 'iteration_complete') return `${(data.iteration_history || []).length} iteration(s) done`;
      if (name === 'workflow_error' || name === 'error') return data.error || 'error';
      return data.message || '';
    })();
    const t = new Date().toLocaleTimeString();
    log.prepend(U.el('div', { class: `ev ev-${name}` }, U.el('span', { class: 'ev-t' }, t),
      U.el('span', { class: 'ev-n' }, name), U.el('span', { class: 'ev-s' }, summary)));
  },

  // ---- request flow ------------------------------------------------------------------------
  filtered(run) {
    return run.requests.filter((r) => !R.view.stage || r.stage === R.view.stage);
  },

  requests(run) {
    U.$('#requests').classList.toggle('hidden', !R.view.table);
    const tb = U.$('#requests tbody');
    tb.innerHTML = '';
    const reqs = R.filtered(run);
    for (const r of reqs) {
      const m = r.llm_meta || {};
      const row = U.el('tr', { class: r.error ? 'err' : '' },
        U.el('td', {}, String(U.nz(r.seq, ''))), U.el('td', {}, String(U.nz(r.iteration, ''))),
        U.el('td', {}, r.stage || ''), U.el('td', {}, r.label || ''),
        U.el('td', {}, r.agent_role || r.source || ''), U.el('td', {}, U.hostOf(r.endpoint)),
        U.el('td', {}, U.fmtSecs(r.duration_seconds)),
        U.el('td', {}, m.completion_tokens !== undefined ? `${m.prompt_tokens}/${m.completion_tokens}` : ''),
        U.el('td', {}, m.queue_wait_s !== undefined ? U.fmtSecs(m.queue_wait_s) : ''),
        U.el('td', {}, r.error ? 'error' : (r.oracle ? 'ok·oracle' : 'ok')));
      const detail = U.el('tr', { class: 'detail hidden' }, U.el('td', { colspan: '10' },
        U.el('div', { class: 'io' }, U.el('h4', {}, 'Prompt ', R.copyBtn(() => r.prompt || '')), U.el('pre', {}, r.prompt || '')),
        U.el('div', { class: 'io' }, U.el('h4', {}, 'Response ', R.copyBtn(() => r.response || r.error || '')), U.el('pre', {}, r.response || r.error || '')),
        U.el('div', { class: 'meta' }, [r.request_id ? `request_id ${r.request_id}` : '',
          r.start_time_utc ? `started ${r.start_time_utc}` : '',
          r.otel && r.otel.agent_a && r.otel.agent_a.trace_id ? `trace ${r.otel.agent_a.trace_id}` : ''].filter(Boolean).join(' · '))));
      row.addEventListener('click', () => detail.classList.toggle('hidden'));
      tb.appendChild(row);
      tb.appendChild(detail);
    }
    const shown = reqs.length === run.requests.length ? '' : ` (${reqs.length} shown)`;
    U.$('#req-count').textContent = `${run.requests.length} LLM calls${shown}`;
    const sel = U.$('#stage-filter');
    const have = Array.from(new Set(run.requests.map((r) => r.stage).filter(Boolean)));
    const cur = Array.from(sel.options).map((o) => o.value).filter(Boolean);
    if (have.join() !== cur.join()) {
      sel.innerHTML = '';
      sel.appendChild(U.el('option', { value: '' }, 'all stages'));
      for (const s of have) sel.appendChild(U.el('option', { value: s }, s));
      sel.value = R.view.stage;
    }
  },

  // Agent A in the middle, one node per endpoint (Agent B workers and the LLM backend),
  // edges weighted by call count and labelled with the stages that used them.
  graph(run) {
    const svg = U.$('#flow');
    svg.classList.toggle('hidden', !R.view.graph);
    if (!R.view.graph) return;
    const W = svg.clientWidth || 520, H = 260;
    svg.setAttribute('viewBox', `0 0 ${W} ${H}`);
    svg.innerHTML = '';
    const targets = {};
    for (const r of R.filtered(run)) {
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

  // ---- collaborative decision: horizontal rounds or vertical solver / reviewers ------------
  discussion(run) {
    const box = U.$('#discussion');
    box.innerHTML = '';
    const dec = (run.stages.decision && run.stages.decision.data) || {};
    const rounds = run.discussion.length ? run.discussion : (dec.discussion_rounds || []).map((r) => ({
      round: r.round, responses: r.responses || [], consensus: (r.responses || []).every((x) => x.consensus) }));
    const vertical = run.vertical.length ? run.vertical : [];
    if (!rounds.length && !vertical.length && !dec.final_decision) {
      box.appendChild(U.el('p', { class: 'muted' }, 'No discussion yet.'));
      return;
    }
    for (const r of rounds) {
      const sec = U.el('details', { class: 'round', open: 'open' },
        U.el('summary', {}, `Round ${r.round} `, U.el('span', { class: r.consensus ? 'badge ok' : 'badge' }, r.consensus ? 'consensus' : 'open')));
      for (const x of r.responses) {
        sec.appendChild(U.el('div', { class: 'speech' },
          U.el('div', { class: 'who' }, x.expert || x.role || `expert ${U.nz(x.index, '')}`,
            x.consensus ? U.el('span', { class: 'badge ok' }, '[CONSENSUS]') : null),
          U.el('div', { class: 'said' }, U.truncate(x.response || x.output || '', 1200))));
      }
      box.appendChild(sec);
    }
    for (const v of vertical) {
      const sec = U.el('details', { class: 'round', open: 'open' },
        U.el('summary', {}, `Solver iteration ${U.nz(v.solver_iteration, '')} `,
          U.el('span', { class: v.all_approved ? 'badge ok' : 'badge' }, v.all_approved ? 'approved' : 'changes requested')));
      if (v.solution) sec.appendChild(U.el('div', { class: 'speech' }, U.el('div', { class: 'who' }, v.solver || 'solver'), U.el('div', { class: 'said' }, U.truncate(v.solution, 1200))));
      for (const rv of v.reviews || []) {
        sec.appendChild(U.el('div', { class: 'speech review' },
          U.el('div', { class: 'who' }, rv.reviewer || rv.role || 'reviewer', rv.approved ? U.el('span', { class: 'badge ok' }, '[APPROVED]') : null),
          U.el('div', { class: 'said' }, U.truncate(rv.review || rv.response || '', 800))));
      }
      box.appendChild(sec);
    }
    if (dec.final_decision) {
      box.appendChild(U.el('div', { class: 'decision' }, U.el('h4', {}, `Decision (${dec.structure_used || ''}) `, R.copyBtn(() => dec.final_decision)),
        U.el('pre', {}, dec.final_decision)));
    }
  },

  // ---- evaluation: score, criteria, rationale, feedback, missing aspects --------------------
  evaluation(run) {
    const box = U.$('#evaluation');
    box.innerHTML = '';
    const ev = run.stages.evaluation && run.stages.evaluation.data;
    if (!ev) { box.appendChild(U.el('p', { class: 'muted' }, 'Not evaluated yet.')); return; }
    const threshold = Number(U.$('#threshold').value) || 90;
    const score = Number(U.nz(ev.score, 0));
    box.appendChild(U.el('div', { class: 'score-row' },
      U.el('div', { class: 'score' }, String(score)),
      U.el('div', { class: 'gauge' }, U.el('div', { class: score >= threshold ? 'fill ok' : 'fill', style: `width:${Math.max(0, Math.min(100, score))}%` }),
        U.el('div', { class: 'mark', style: `left:${threshold}%`, title: `threshold ${threshold}` })),
      U.el('span', { class: ev.goal_achieved ? 'badge ok' : 'badge warn' }, ev.goal_achieved ? 'goal achieved' : 'iterate')));
    const crit = ev.criteria && typeof ev.criteria === 'object' ? ev.criteria : {};
    const names = Object.keys(crit);
    if (names.length) {
      const tbl = U.el('table', { class: 'criteria' });
      for (const n of names) {
        const v = typeof crit[n] === 'object' && crit[n] ? U.nz(crit[n].score, '') : crit[n];
        const note = typeof crit[n] === 'object' && crit[n] ? (crit[n].comment || crit[n].reason || '') : '';
        tbl.appendChild(U.el('tr', {}, U.el('td', {}, n), U.el('td', {}, String(v)),
          U.el('td', {}, U.el('div', { class: 'bar', style: `width:${Math.min(100, Number(v) * 5) || 0}%` })), U.el('td', { class: 'muted' }, note)));
      }
      box.appendChild(tbl);
    }
    if (ev.rationale) box.appendChild(U.el('p', {}, U.el('b', {}, 'Rationale: '), ev.rationale));
    if (ev.feedback) box.appendChild(U.el('p', {}, U.el('b', {}, 'Feedback: '), ev.feedback));
    if ((ev.missing_aspects || []).length) {
      box.appendChild(U.el('div', {}, U.el('b', {}, 'Missing aspects'), U.el('ul', {}, ev.missing_aspects.map((m) => U.el('li', {}, String(m))))));
    }
  },

  // ---- iteration history: detail per iteration + diff against the previous one ------------
  iterations(run) {
    const box = U.$('#iterations');
    box.innerHTML = '';
    const its = Object.keys(run.iterations).map(Number).sort((a, b) => a - b);
    if (!its.length) { box.appendChild(U.el('p', { class: 'muted' }, 'No iterations yet.')); return; }
    its.forEach((n, k) => {
      const snap = run.iterations[n];
      const f = Diff.facts(snap);
      const head = `Iteration ${n}: score ${U.nz(f.score, '–')}${f.goal ? ' ✓' : ''} · ${f.experts.length} experts · ${f.structure || '–'} · ${f.success} ok / ${f.failures} failed`;
      const det = U.el('details', { class: 'iter' }, U.el('summary', {}, head));
      det.appendChild(U.el('div', { class: 'iter-body' },
        U.el('div', {}, U.el('b', {}, 'Experts: '), f.experts.join(', ') || '–'),
        U.el('div', {}, U.el('b', {}, 'Decision: '), `${f.rounds} round(s), consensus ${f.consensus ? 'yes' : 'no'}`),
        snap.executions.length ? U.el('ul', {}, snap.executions.map((e) => U.el('li', { class: e.success ? '' : 'err' },
          `${e.expert}: ${e.success ? 'ok' : 'failed'} — ${U.truncate(e.output || e.error || '', 200)}`))) : null,
        f.feedback ? U.el('div', {}, U.el('b', {}, 'Feedback: '), f.feedback) : null));
      if (k > 0) {
        const prev = run.iterations[its[k - 1]];
        const btn = U.el('button', { class: 'small' }, `diff vs iteration ${its[k - 1]}`);
        const out = U.el('div', { class: 'diff hidden' });
        btn.addEventListener('click', () => {
          if (!out.childNodes.length) R.renderDiff(out, Diff.iterations(prev, snap));
          out.classList.toggle('hidden');
        });
        det.appendChild(btn);
        det.appendChild(out);
      }
      box.appendChild(det);
    });
  },

  renderDiff(box, d) {
    const sign = (v) => (v === null || v === undefined ? '–' : (v > 0 ? `+${v}` : String(v)));
    box.appendChild(U.el('div', {}, U.el('b', {}, 'Experts: '),
      d.experts.added.map((e) => U.el('span', { class: 'add' }, `+${e} `)),
      d.experts.removed.map((e) => U.el('span', { class: 'del' }, `−${e} `)),
      d.experts.kept.length ? U.el('span', { class: 'muted' }, `(kept ${d.experts.kept.join(', ')})`) : null));
    box.appendChild(U.el('div', {}, U.el('b', {}, 'Structure: '), d.structure.changed ? `${d.structure.from} → ${d.structure.to}` : `${d.structure.to || '–'} (unchanged)`));
    box.appendChild(U.el('div', {}, U.el('b', {}, 'Score: '), `${U.nz(d.score.from, '–')} → ${U.nz(d.score.to, '–')} (${sign(d.score.delta)})`,
      d.goal.to && !d.goal.from ? U.el('span', { class: 'badge ok' }, 'goal reached') : null));
    box.appendChild(U.el('div', {}, U.el('b', {}, 'Decision: '), `rounds ${sign(d.rounds.delta)}, consensus ${d.consensus.from ? 'yes' : 'no'} → ${d.consensus.to ? 'yes' : 'no'}`));
    box.appendChild(U.el('div', {}, U.el('b', {}, 'Execution: '), `successes ${sign(d.execution.success)}, failures ${sign(d.execution.failures)}`));
    if (d.criteria.length) {
      box.appendChild(U.el('table', { class: 'criteria' }, d.criteria.map((c) => U.el('tr', {},
        U.el('td', {}, c.name), U.el('td', {}, String(U.nz(c.from, '–'))), U.el('td', {}, '→'),
        U.el('td', {}, String(U.nz(c.to, '–'))), U.el('td', { class: c.delta > 0 ? 'add' : c.delta < 0 ? 'del' : 'muted' }, sign(c.delta))))));
    }
    if (d.decision.some((x) => x.op !== '=')) {
      box.appendChild(U.el('pre', { class: 'linediff' }, d.decision.map((x) => U.el('div', { class: x.op === '+' ? 'add' : x.op === '-' ? 'del' : '' }, `${x.op === '=' ? ' ' : x.op} ${x.text}`))));
    }
  },

  // ---- final output, copy, raw JSON -------------------------------------------------------------
  copyBtn(getText) {
    const b = U.el('button', { class: 'small copy', title: 'copy to clipboard' }, 'copy');
    b.addEventListener('click', (e) => {
      e.stopPropagation();
      U.copy(getText()).then(() => { b.textContent = 'copied'; setTimeout(() => { b.textContent = 'copy'; }, 1200); },
        () => { b.textContent = 'copy failed'; });
    });
    return b;
  },

  final(result) {
    const box = U.$('#final');
    const raw = U.$('#raw');
    if (!result) { box.textContent = ''; raw.textContent = ''; U.$('#final-meta').textContent = ''; return; }
    const status = result.completed ? 'completed' : result.partial ? 'partial' : 'not completed';
    U.$('#final-meta').textContent = `task ${result.task_id} · ${status} · ${U.nz(result.iterations, '?')} iteration(s) · ${U.fmtSecs(result.duration_seconds)}${result.workflow_error ? ' · error: ' + result.workflow_error : ''}`;
    box.textContent = result.final_output || '';
    raw.textContent = JSON.stringify(result, null, 2);
  },

  history(onOpen, onForget) {
    const ul = U.$('#history');
    ul.innerHTML = '';
    for (const h of State.history()) {
      const li = U.el('li', {},
        U.el('a', { href: `?task_id=${encodeURIComponent(h.task_id)}`, onclick: (e) => { e.preventDefault(); onOpen(h.task_id); } }, U.truncate(h.task || h.task_id, 60)),
        U.el('span', { class: 'h-meta' }, ` ${h.completed ? '✓' : '…'} ${h.score !== null && h.score !== undefined ? 'score ' + h.score + ' · ' : ''}${h.calls ? h.calls + ' calls · ' : ''}${new Date(h.at).toLocaleString()}`),
        U.el('button', { class: 'x', title: 'forget', onclick: () => onForget(h.task_id) }, '×'));
      ul.appendChild(li);
    }
  },

  all(run) {
    R.stages(run);
    R.timer(run);
    R.requests(run);
    R.graph(run);
    R.discussion(run);
    R.evaluation(run);
    R.iterations(run);
  },
};
