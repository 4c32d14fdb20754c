// POST /agentverse with SSE streaming, falling back to a plain JSON request when the
// stream cannot be opened (reference ui/agentverse/js/streaming.js behaviour).
// SSE frames are "event: <name>\ndata: <json>\n\n"; events: iteration_start, stage_start,
// stage_complete, llm_request, llm_error, discussion_round, vertical_iteration,
// execution_result, iteration_complete, workflow_error, complete, error.

function parseSseBlock(block) {
  let event = 'message';
  const data = [];
  for (const line of block.split('\n')) {
    if (line.startsWith('event:')) event = line.slice(6).trim();
    else if (line.startsWith('data:')) data.push(line.slice(5).replace(/^ /, ''));
  }
  if (!data.length) return null;
  const raw = data.join('\n');
  try { return { event, data: JSON.parse(raw) }; } catch (e) { return { event, data: raw }; }
}

async function runAgentverse({ endpoint, payload, onEvent, signal }) {
  const timeoutCtl = new AbortController();
  const timer = setTimeout(() => timeoutCtl.abort(), AV_CONFIG.requestTimeoutMs);
  if (signal) signal.addEventListener('abort', () => timeoutCtl.abort());
  let sawEvent = false;
  try {
    const resp = await fetch(endpoint, {
      method: 'POST',
      headers: { 'Content-Type': 'application/json', Accept: 'text/event-stream' },
      body: JSON.stringify({ ...payload, stream: true }),
      signal: timeoutCtl.signal,
    });
    if (!resp.ok) throw new Error(`HTTP ${resp.status}: ${(await resp.text()).slice(0, 300)}`);
    const ctype = resp.headers.get('Content-Type') || '';
    if (!ctype.includes('text/event-stream') || !resp.body) {
      const body = await resp.json();
      onEvent('complete', body);
      return body;
    }
    const reader = resp.body.getReader();
    const dec = new TextDecoder();
    let buf = '';
    let final = null;
    for (;;) {
      const { value, done } = await reader.read();
      if (done) break;
      buf += dec.decode(value, { stream: true }).replace(/\r\n/g, '\n');
      let idx;
      while ((idx = buf.indexOf('\n\n')) >= 0) {
        const block = buf.slice(0, idx);
        buf = buf.slice(idx + 2);
        const ev = parseSseBlock(block);
        if (!ev) continue;
        sawEvent = true;
        onEvent(ev.event, ev.data);
        if (ev.event === 'complete') final = ev.data;
        if (ev.event === 'error') throw new Error(ev.data && ev.data.error ? ev.data.error : 'stream error');
      }
    }
    if (!final) throw new Error('stream ended without a complete event');
    return final;
  } catch (err) {
    if (sawEvent || timeoutCtl.signal.aborted) throw err;
    // could not stream at all: retry as one blocking JSON request
    onEvent('fallback', { message: `streaming unavailable (${err.message}); retrying without SSE` });
    const resp = await fetch(endpoint, {
      method: 'POST',
      headers: { 'Content-Type': 'application/json' },
      body: JSON.stringify({ ...payload, stream: false }),
      signal: timeoutCtl.signal,
    });
    if (!resp.ok) throw new Error(`HTTP ${resp.status}: ${(await resp.text()).slice(0, 300)}`);
    const body = await resp.json();
    onEvent('complete', body);
    return body;
  } finally {
    clearTimeout(timer);
  }
}

async function loadAgentverseRun(endpoint, taskId) {
  const resp = await fetch(`${U.baseOf(endpoint)}/agentverse/${encodeURIComponent(taskId)}`);
  if (!resp.ok) throw new Error(`HTTP ${resp.status}`);
  return resp.json();
}
