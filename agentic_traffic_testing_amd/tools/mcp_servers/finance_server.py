"""Synthetic finance MCP server (reference tools/mcp_servers/finance_server.py:17-103).

Tools: ``get_stock_price`` (quote with +-5 jitter so repeated calls differ),
``calculate_portfolio_value`` (base prices); resource ``resource://market/indices``.
All data is fake and deterministic apart from the jitter.
"""
from __future__ import annotations

import random
from datetime import datetime, timezone

from agentic_traffic_testing_amd.tools.mcp import ToolServer

server = ToolServer("finance-server")

STOCKS = {
    "AAPL": (175.50, 2.3),
    "GOOGL": (142.80, -1.2),
    "MSFT": (378.90, 3.5),
    "TSLA": (245.60, -5.2),
}


def _now() -> str:
    return datetime.now(timezone.utc).replace(tzinfo=None).isoformat() + "Z"


@server.tool()
def get_stock_price(symbol: str) -> dict:
    """Synthetic current price for a stock symbol (not market data)."""
    sym = symbol.upper()
    if sym not in STOCKS:
        return {"error": f"Unknown symbol: {sym}", "available_symbols": sorted(STOCKS)}
    base, change = STOCKS[sym]
    return {"symbol": sym, "price": round(base + random.uniform(-5, 5), 2),
            "change_percent": round(change, 2), "timestamp": _now()}


@server.tool()
def calculate_portfolio_value(holdings: dict[str, float]) -> dict:
    """Value a {symbol: shares} portfolio at the synthetic base prices (unknown symbols
    are skipped)."""
    positions, total = [], 0.0
    for symbol, shares in holdings.items():
        sym = symbol.upper()
        if sym not in STOCKS:
            continue
        price = STOCKS[sym][0]
        value = price * float(shares)
        total += value
        positions.append({"symbol": sym, "shares": float(shares), "price": round(price, 2),
                          "value": round(value, 2)})
    return {"total_value": round(total, 2), "positions": positions, "timestamp": _now()}


@server.resource("resource://market/indices")
def list_indices() -> dict:
    """Synthetic snapshot of three market indices."""
    return {"indices": {"S&P 500": 4567.89, "Dow Jones": 35432.10, "NASDAQ": 14234.56},
            "updated": _now()}


if __name__ == "__main__":
    server.run()
