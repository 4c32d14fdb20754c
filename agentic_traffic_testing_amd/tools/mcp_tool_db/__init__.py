"""HTTP "MCP-style" database tool."""
