// AgentVerse UI configuration.  The default endpoint follows the page's host so the UI
// works from any machine that can reach Agent A on :8101 (reference ui/agentverse/js/utils.js).
window.AV_CONFIG = {
  defaultEndpoint: `${location.protocol === 'https:' ? 'https' : 'http'}://${location.hostname || 'localhost'}:8101/agentverse`,
  requestTimeoutMs: 300000,      // 5 minutes, like the reference UI
  historyKey: 'agentverse.history.v2',
  historyLimit: 50,
  stages: [
    { id: 'recruitment', title: 'Expert Recruitment', n: 1 },
    { id: 'decision', title: 'Collaborative Decision', n: 2 },
    { id: 'execution', title: 'Action Execution', n: 3 },
    { id: 'evaluation', title: 'Evaluation', n: 4 },
    { id: 'synthesis', title: 'Final Synthesis', n: 5 },
  ],
};
