"""Synthetic maps MCP server (reference tools/mcp_servers/maps_server.py:16-108).

Tools: ``geocode_location`` (case-insensitive substring match against four cities) and
``calculate_distance`` (haversine on a 6371 km sphere); resource
``resource://maps/known-locations``.  No external APIs: traffic stays in the testbed.
"""
from __future__ import annotations

import math

from agentic_traffic_testing_amd.tools.mcp import ToolServer

server = ToolServer("maps-server")

PLACES = {
    "new york": (40.7128, -74.0060, "New York", "USA"),
    "london": (51.5074, -0.1278, "London", "UK"),
    "tokyo": (35.6762, 139.6503, "Tokyo", "Japan"),
    "paris": (48.8566, 2.3522, "Paris", "France"),
}
EARTH_RADIUS_KM = 6371.0
KM_TO_MILES = 0.621371


def resolve(address: str) -> dict:
    q = address.lower()
    for key, (lat, lng, city, country) in PLACES.items():
        if key in q:
            return {"address": address, "coordinates": {"latitude": lat, "longitude": lng},
                    "city": city, "country": country, "found": True}
    return {"address": address, "found": False,
            "error": "Location not found in local maps database."}


@server.tool()
def geocode_location(address: str) -> dict:
    """Map a place name to synthetic coordinates (fuzzy substring match)."""
    return resolve(address)


def haversine_km(lat1, lon1, lat2, lon2) -> float:
    p1, p2 = math.radians(lat1), math.radians(lat2)
    dp, dl = p2 - p1, math.radians(lon2 - lon1)
    h = math.sin(dp / 2) ** 2 + math.cos(p1) * math.cos(p2) * math.sin(dl / 2) ** 2
    return 2 * EARTH_RADIUS_KM * math.asin(math.sqrt(h))


@server.tool()
def calculate_distance(location1: str, location2: str) -> dict:
    """Great-circle distance between two known locations."""
    a, b = resolve(location1), resolve(location2)
    if not (a.get("found") and b.get("found")):
        return {"error": "One or both locations could not be resolved."}
    km = haversine_km(a["coordinates"]["latitude"], a["coordinates"]["longitude"],
                      b["coordinates"]["latitude"], b["coordinates"]["longitude"])
    return {"from": location1, "to": location2, "distance_km": round(km, 2),
            "distance_miles": round(km * KM_TO_MILES, 2)}


@server.resource("resource://maps/known-locations")
def list_known_locations() -> dict:
    """The synthetic location catalogue."""
    return {"locations": [{"name": city, "country": country,
                           "coordinates": {"lat": lat, "lng": lng}}
                          for lat, lng, city, country in PLACES.values()]}


if __name__ == "__main__":
    server.run()
