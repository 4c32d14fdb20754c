"""Local demo MCP servers (reference tools/mcp_servers/__init__.py): small, deterministic
stdio tool servers the agents can call; they are standalone processes, not HTTP agents."""
