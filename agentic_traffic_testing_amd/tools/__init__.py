"""Tool plane of the testbed: the HTTP mcp-tool-db, stdio MCP demo
servers (coding / finance / maps), the OpenAI-compatible proxy and MCP-Universe runner."""
