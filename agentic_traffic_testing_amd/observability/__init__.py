"""Observability plane: TCP metrics collector, Docker mapping
exporter, health check, pcap / telemetry analysis, Grafana dashboard + Prometheus config
generation."""
