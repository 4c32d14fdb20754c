// Small DOM / formatting helpers shared by the AgentVerse UI.
const U = {
  nz(v, d) { return v === undefined || v === null ? d : v; },
  $(sel, root = document) { return root.querySelector(sel); },
  el(tag, attrs = {}, ...children) {
    const n = document.createElement(tag);
    for (const [k, v] of Object.entries(attrs || {})) {
      if (k === 'class') n.className = v;
      else if (k.startsWith('on') && typeof v === 'function') n.addEventListener(k.slice(2), v);
      else if (v !== undefined && v !== null) n.setAttribute(k, v);
    }
    for (const c of children.flat()) {
      if (c === null || c === undefined) continue;
      n.appendChild(typeof c === 'string' || typeof c === 'number' ? document.createTextNode(String(c)) : c);
    }
    return n;
  },
  esc(s) {
    return String(U.nz(s, '')).replace(/[&<>"']/g, (c) => ({ '&': '&amp;', '<': '&lt;', '>': '&gt;', '"': '&quot;', "'": '&#39;' }[c]));
  },
  fmtSecs(s) {
    if (s === undefined || s === null || isNaN(s)) return '–';
    return s < 1 ? `${(s * 1000).toFixed(0)} ms` : `${Number(s).toFixed(2)} s`;
  },
  truncate(s, n = 160) { s = String(U.nz(s, '')); return s.length > n ? s.slice(0, n) + '…' : s; },
  hostOf(url) { try { return new URL(url).host; } catch (e) { return String(url || ''); } },
  baseOf(endpoint) { return String(endpoint).replace(/\/agentverse\/?$/, ''); },
  queryParam(name) { return new URLSearchParams(location.search).get(name); },
  // clipboard with a fallback for plain-http pages (navigator.clipboard needs a secure context)
  copy(text) {
    text = String(U.nz(text, ''));
    if (typeof navigator !== 'undefined' && navigator.clipboard && window.isSecureContext) {
      return navigator.clipboard.writeText(text);
    }
    return new Promise((resolve, reject) => {
      const ta = U.el('textarea', { style: 'position:fixed;left:-9999px' });
      ta.value = text;
      document.body.appendChild(ta);
      ta.select();
      const ok = document.execCommand('copy');
      ta.remove();
      if (ok) resolve(); else reject(new Error('copy failed'));
    });
  },
};

if (typeof module !== 'undefined') module.exports = { U };
