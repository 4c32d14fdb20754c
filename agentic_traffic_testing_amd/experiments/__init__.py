"""Experiment pipeline: runner, dashboard-driven Prometheus
scraper, plotting / statistics, log x TCP correlation, single-request helper and the
MCP-Universe / MCP smoke runners.  CLI wrappers live in ``scripts/experiment/``."""
