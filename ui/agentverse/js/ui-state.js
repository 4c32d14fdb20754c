// Run state + localStorage history.
const State = {
  run: null,
  reset(task) {
    this.run = { task, events: [], requests: [], stages: {}, iteration: 0, final: null, result: null, started: Date.now() };
    return this.run;
  },
  addRequest(r) {
    const key = U.nz(r.seq, this.run.requests.length + 1);
    const i = this.run.requests.findIndex((x) => U.nz(x.seq, -1) === key);
    if (i >= 0) this.run.requests[i] = { ...this.run.requests[i], ...r };
    else this.run.requests.push({ ...r, seq: key });
  },
  history() {
    try { return JSON.parse(localStorage.getItem(AV_CONFIG.historyKey) || '[]'); } catch (e) { return []; }
  },
  remember(result) {
    if (!result || !result.task_id) return;
    const h = this.history().filter((x) => x.task_id !== result.task_id);
    h.unshift({
      task_id: result.task_id, task: result.original_task || '', completed: !!result.completed,
      iterations: result.iterations, duration: result.duration_seconds, at: Date.now(),
    });
    localStorage.setItem(AV_CONFIG.historyKey, JSON.stringify(h.slice(0, AV_CONFIG.historyLimit)));
  },
  forget(taskId) {
    localStorage.setItem(AV_CONFIG.historyKey, JSON.stringify(this.history().filter((x) => x.task_id !== taskId)));
  },
  clearHistory() { localStorage.removeItem(AV_CONFIG.historyKey); },
};
