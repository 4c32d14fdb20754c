#!/usr/bin/env python3
"""Dev server for the static UI without Docker: ``python ui/serve.py [--port 3000]``.

Serves ui/ at / and maps ``/chat/templates/*`` and ``/agentverse/templates/*`` to the
agents' template directory, mirroring what ui/Dockerfile copies into the image.
"""
from __future__ import annotations

import argparse
import functools
import os
from http.server import SimpleHTTPRequestHandler, ThreadingHTTPServer

UI = os.path.dirname(os.path.abspath(__file__))
TEMPLATES = os.path.join(os.path.dirname(UI), "agentic_traffic_testing_amd", "agents", "templates")


class Handler(SimpleHTTPRequestHandler):
    def translate_path(self, path):
        clean = path.split("?", 1)[0].split("#", 1)[0]
        for prefix in ("/chat/templates/", "/agentverse/templates/"):
            if clean.startswith(prefix):
                name = os.path.basename(clean[len(prefix):])
                return os.path.join(TEMPLATES, name)
        return super().translate_path(path)

    def log_message(self, *a):
        pass


def make_server(host: str = "0.0.0.0", port: int = 3000) -> ThreadingHTTPServer:
    return ThreadingHTTPServer((host, port), functools.partial(Handler, directory=UI))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=3000)
    a = ap.parse_args()
    srv = make_server(a.host, a.port)
    print(f"[*] UI on http://{a.host}:{srv.server_address[1]}/ (chat, agentverse)", flush=True)
    srv.serve_forever()


if __name__ == "__main__":
    main()
