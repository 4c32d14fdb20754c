"""Deployment topology generators (docker compose, Prometheus/Grafana provisioning)."""
