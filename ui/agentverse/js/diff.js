// Iteration comparison for the AgentVerse history view: what changed between two
// iterations of a workflow (experts, structure, consensus, execution, evaluation criteria)
// and a line diff of their texts.  Pure functions (tested under node in tests/test_ui.py).
const Diff = {
  // snapshot -> normalised facts (from stage_complete payloads or the iteration summary)
  facts(snap) {
    const st = (snap && snap.stages) || {};
    const sum = (snap && snap.summary) || {};
    const rec = st.recruitment || {};
    const experts = (rec.experts || []).map((e) => (typeof e === 'string' ? e : e.role))
      .concat(rec.experts ? [] : ((sum.recruitment || {}).experts || []));
    const ev = st.evaluation || sum.evaluation || {};
    const dec = st.decision || {};
    const exe = st.execution || {};
    return {
      experts,
      structure: rec.communication_structure || (sum.recruitment || {}).structure || null,
      consensus: dec.consensus_reached !== undefined ? !!dec.consensus_reached : !!(sum.decision || {}).consensus,
      rounds: dec.discussion_rounds ? dec.discussion_rounds.length
        : ((snap && snap.discussion && snap.discussion.length) || (sum.decision || {}).rounds || 0),
      success: exe.success_count !== undefined ? exe.success_count : (sum.execution || {}).success || 0,
      failures: exe.failure_count !== undefined ? exe.failure_count : (sum.execution || {}).failures || 0,
      score: ev.score !== undefined ? ev.score : null,
      goal: !!ev.goal_achieved,
      criteria: ev.criteria && typeof ev.criteria === 'object' ? ev.criteria : {},
      decisionText: dec.final_decision || '',
      feedback: ev.feedback || '',
    };
  },

  iterations(a, b) {
    const A = Diff.facts(a), B = Diff.facts(b);
    const setA = new Set(A.experts), setB = new Set(B.experts);
    const names = Array.from(new Set(Object.keys(A.criteria).concat(Object.keys(B.criteria))));
    const num = (v) => (typeof v === 'number' ? v : (v && typeof v === 'object' && typeof v.score === 'number' ? v.score : null));
    return {
      experts: {
        added: B.experts.filter((e) => !setA.has(e)),
        removed: A.experts.filter((e) => !setB.has(e)),
        kept: B.experts.filter((e) => setA.has(e)),
      },
      structure: { from: A.structure, to: B.structure, changed: A.structure !== B.structure },
      consensus: { from: A.consensus, to: B.consensus },
      rounds: { from: A.rounds, to: B.rounds, delta: B.rounds - A.rounds },
      execution: { success: B.success - A.success, failures: B.failures - A.failures },
      score: { from: A.score, to: B.score, delta: (A.score === null || B.score === null) ? null : B.score - A.score },
      goal: { from: A.goal, to: B.goal },
      criteria: names.map((n) => {
        const f = num(A.criteria[n]), t = num(B.criteria[n]);
        return { name: n, from: f, to: t, delta: f === null || t === null ? null : t - f };
      }),
      decision: Diff.lines(A.decisionText, B.decisionText),
    };
  },

  // LCS line diff -> [{op: '=', '-', '+', text}]; long texts are cut to keep it O(n*m) small
  lines(a, b, limit = 400) {
    const x = String(a || '').split('\n').slice(0, limit);
    const y = String(b || '').split('\n').slice(0, limit);
    const n = x.length, m = y.length;
    const L = Array.from({ length: n + 1 }, () => new Int32Array(m + 1));
    for (let i = n - 1; i >= 0; i--) {
      for (let j = m - 1; j >= 0; j--) {
        L[i][j] = x[i] === y[j] ? L[i + 1][j + 1] + 1 : Math.max(L[i + 1][j], L[i][j + 1]);
      }
    }
    const out = [];
    let i = 0, j = 0;
    while (i < n && j < m) {
      if (x[i] === y[j]) { out.push({ op: '=', text: x[i] }); i++; j++; }
      else if (L[i + 1][j] >= L[i][j + 1]) out.push({ op: '-', text: x[i++] });
      else out.push({ op: '+', text: y[j++] });
    }
    while (i < n) out.push({ op: '-', text: x[i++] });
    while (j < m) out.push({ op: '+', text: y[j++] });
    return out;
  },
};

if (typeof module !== 'undefined') module.exports = { Diff };
