"""Compatibility entry points: ``python -m llm.serve_llm`` / ``python -m llm.hf_cpu_server``
(the reference's module paths, infra/docker-compose.yml:27) backed by
``agentic_traffic_testing_amd.serving``."""
