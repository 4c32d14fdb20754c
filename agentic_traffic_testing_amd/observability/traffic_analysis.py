"""pcap + telemetry analyzer (reference scripts/traffic/analyze_traffic.py:1-421, SURVEY §2.2
O11).

* ``read_pcap`` is a dependency-free classic-pcap reader (scapy is not in the image):
  microsecond / nanosecond magic in either byte order, link types Ethernet (1, incl.
  802.1Q tags), Linux cooked v1 / v2 (113 / 276, what ``tcpdump -i any`` writes) and raw
  IPv4 (101 / 228).  Only IPv4/TCP packets are returned.
* ``analyze_pcap`` groups packets into bidirectional flows (sorted endpoint pair), counts
  SYN / FIN / RST per flow, new connections and bytes per second from the first packet;
  bytes are the captured frame length (``len(pkt)`` in the reference).  Services come
  from the distributed topology's IPs, unknown addresses stay as the IP.
* ``analyze_telemetry`` loads ``*.log`` / ``*.jsonl`` JSONL events and groups them by
  ``task_id`` (sorted by ``timestamp_ms``).
* ``export_csv`` writes ``flows.csv`` and ``timeseries.csv`` (same columns as the
  reference).
"""
from __future__ import annotations

import argparse
import json
import socket
import struct
import sys
from collections import defaultdict
from dataclasses import dataclass
from pathlib import Path

SERVICE_IPS = {
    "172.23.0.10": "agent-a",
    "172.23.0.20": "agent-b-1",
    "172.23.0.21": "agent-b-2",
    "172.23.0.22": "agent-b-3",
    "172.23.0.23": "agent-b-4",
    "172.23.0.24": "agent-b-5",
    "172.23.0.30": "llm-backend",
    "172.23.0.40": "mcp-tool-db",
    "172.23.0.50": "chat-ui",
    "172.23.0.60": "jaeger",
    "172.24.0.10": "mcp-tool-db",
}

TCP_FIN, TCP_SYN, TCP_RST = 0x01, 0x02, 0x04


@dataclass
class TcpPacket:
    ts: float
    src: str
    dst: str
    sport: int
    dport: int
    flags: int
    frame_len: int     # original length on the wire (pcap orig_len)
    payload_len: int


def _ipv4_tcp(buf: bytes, off: int, ts: float, orig_len: int) -> TcpPacket | None:
    if len(buf) < off + 20 or buf[off] >> 4 != 4:
        return None
    ihl = (buf[off] & 0x0F) * 4
    total = struct.unpack_from("!H", buf, off + 2)[0]
    if buf[off + 9] != 6 or len(buf) < off + ihl + 14:
        return None
    src = socket.inet_ntoa(buf[off + 12:off + 16])
    dst = socket.inet_ntoa(buf[off + 16:off + 20])
    t = off + ihl
    sport, dport = struct.unpack_from("!HH", buf, t)
    doff = (buf[t + 12] >> 4) * 4
    flags = buf[t + 13]
    return TcpPacket(ts, src, dst, sport, dport, flags, orig_len, max(0, total - ihl - doff))


def read_pcap(path) -> list[TcpPacket]:
    data = Path(path).read_bytes()
    if len(data) < 24:
        raise ValueError("not a pcap file")
    magic = data[:4]
    table = {b"\xd4\xc3\xb2\xa1": ("<", 1e-6), b"\xa1\xb2\xc3\xd4": (">", 1e-6),
             b"\x4d\x3c\xb2\xa1": ("<", 1e-9), b"\xa1\xb2\x3c\x4d": (">", 1e-9)}
    if magic not in table:
        raise ValueError("unsupported capture format (classic pcap only; convert pcapng "
                         "with `editcap -F pcap`)")
    end, frac = table[magic]
    linktype = struct.unpack_from(end + "I", data, 20)[0] & 0x0FFFFFFF
    out, off = [], 24
    rec = struct.Struct(end + "IIII")
    while off + 16 <= len(data):
        sec, sub, incl, orig = rec.unpack_from(data, off)
        off += 16
        pkt = data[off:off + incl]
        off += incl
        ts = sec + sub * frac
        if linktype == 1:  # Ethernet
            if len(pkt) < 14:
                continue
            eth = struct.unpack_from("!H", pkt, 12)[0]
            l3 = 14
            while eth == 0x8100 and len(pkt) >= l3 + 4:  # VLAN tags
                eth = struct.unpack_from("!H", pkt, l3 + 2)[0]
                l3 += 4
            if eth != 0x0800:
                continue
        elif linktype == 113:  # Linux cooked v1
            if len(pkt) < 16 or struct.unpack_from("!H", pkt, 14)[0] != 0x0800:
                continue
            l3 = 16
        elif linktype == 276:  # Linux cooked v2
            if len(pkt) < 20 or struct.unpack_from("!H", pkt, 0)[0] != 0x0800:
                continue
            l3 = 20
        elif linktype in (101, 228):  # raw IP
            l3 = 0
        else:
            raise ValueError(f"unsupported link type {linktype}")
        p = _ipv4_tcp(pkt, l3, ts, orig)
        if p is not None:
            out.append(p)
    return out


@dataclass
class FlowStats:
    src_ip: str
    dst_ip: str
    src_port: int
    dst_port: int
    src_service: str
    dst_service: str
    packet_count: int = 0
    bytes_total: int = 0
    start_time: float | None = None
    end_time: float | None = None
    syn_count: int = 0
    fin_count: int = 0
    rst_count: int = 0

    @property
    def duration(self) -> float:
        return (self.end_time - self.start_time) if self.start_time is not None else 0.0


def service(ip: str, table: dict | None = None) -> str:
    return (table or SERVICE_IPS).get(ip, ip)


def analyze_packets(pkts: list[TcpPacket], table: dict | None = None) -> dict:
    flows: dict = {}
    cps, bps = defaultdict(int), defaultdict(int)
    first = pkts[0].ts if pkts else None
    last = first
    for p in pkts:
        last = p.ts
        key = tuple(sorted(((p.src, p.sport), (p.dst, p.dport))))
        f = flows.get(key)
        if f is None:
            (a, ap), (b, bp) = key
            f = flows[key] = FlowStats(a, b, ap, bp, service(a, table), service(b, table),
                                       start_time=p.ts)
        f.packet_count += 1
        f.bytes_total += p.frame_len
        f.end_time = p.ts
        sec = int(p.ts - first)
        if p.flags & TCP_SYN:
            f.syn_count += 1
            cps[sec] += 1
        if p.flags & TCP_FIN:
            f.fin_count += 1
        if p.flags & TCP_RST:
            f.rst_count += 1
        bps[sec] += p.frame_len
    pairs = defaultdict(list)
    for f in flows.values():
        pairs[tuple(sorted((f.src_service, f.dst_service)))].append(f)
    return {"duration_seconds": (last - first) if pkts else 0.0,
            "total_packets": sum(f.packet_count for f in flows.values()),
            "total_bytes": sum(f.bytes_total for f in flows.values()),
            "total_flows": len(flows), "flows": list(flows.values()),
            "service_pairs": dict(pairs), "connections_per_second": dict(cps),
            "bytes_per_second": dict(bps), "first_timestamp": first, "last_timestamp": last}


def analyze_pcap(path, table: dict | None = None) -> dict:
    res = analyze_packets(read_pcap(path), table)
    res["pcap_file"] = str(path)
    return res


def analyze_telemetry(directory) -> dict:
    events = []
    d = Path(directory)
    for f in sorted(list(d.glob("*.log")) + list(d.glob("*.jsonl"))):
        for line in f.read_text(errors="replace").splitlines():
            line = line.strip()
            if not line:
                continue
            try:
                ev = json.loads(line)
            except json.JSONDecodeError:
                continue
            if isinstance(ev, dict):
                events.append(ev)
    tasks = defaultdict(list)
    for ev in events:
        if ev.get("task_id"):
            tasks[ev["task_id"]].append(ev)
    for evs in tasks.values():
        evs.sort(key=lambda e: e.get("timestamp_ms", 0))
    return {"total_events": len(events), "total_tasks": len(tasks), "events": events,
            "tasks": dict(tasks)}


def flow_summary(a: dict) -> str:
    lines = ["=" * 70, "TRAFFIC FLOW SUMMARY", "=" * 70,
             f"\nCapture Duration: {a['duration_seconds']:.1f} seconds",
             f"Total Packets:    {a['total_packets']}",
             f"Total Bytes:      {a['total_bytes']} ({a['total_bytes'] / 1024:.1f} KB)",
             f"Total Flows:      {a['total_flows']}", "\n--- Traffic by Service Pair ---",
             f"{'Service Pair':<40} {'Flows':>8} {'Packets':>10} {'Bytes':>12}", "-" * 70]
    for pair, fl in sorted(a["service_pairs"].items(),
                           key=lambda kv: -sum(f.bytes_total for f in kv[1])):
        lines.append(f"{pair[0] + ' <-> ' + pair[1]:<40} {len(fl):>8} "
                     f"{sum(f.packet_count for f in fl):>10} {sum(f.bytes_total for f in fl):>12}")
    lines += ["\n--- Top 10 Flows by Bytes ---",
              f"{'Source':<20} {'Dest':<20} {'Packets':>10} {'Bytes':>12} {'Duration':>10}",
              "-" * 70]
    for f in sorted(a["flows"], key=lambda f: -f.bytes_total)[:10]:
        lines.append(f"{f.src_service + ':' + str(f.src_port):<20} "
                     f"{f.dst_service + ':' + str(f.dst_port):<20} {f.packet_count:>10} "
                     f"{f.bytes_total:>12} {f.duration:>9.2f}s")
    return "\n".join(lines)


def telemetry_summary(t: dict) -> str:
    lines = ["=" * 70, "APPLICATION TELEMETRY SUMMARY", "=" * 70,
             f"\nTotal Events: {t['total_events']}", f"Total Tasks:  {t['total_tasks']}",
             "\n--- Events by Type ---"]
    counts = defaultdict(int)
    for ev in t["events"]:
        counts[ev.get("event_type", "unknown")] += 1
    lines += [f"  {k:<30} {v:>6}" for k, v in sorted(counts.items(), key=lambda kv: -kv[1])]
    if t["tasks"]:
        lines.append("\n--- Sample Task Traces ---")
        for tid, evs in list(t["tasks"].items())[:3]:
            lines.append(f"\nTask: {tid[:8]}...")
            lines += [f"  [{e.get('timestamp_ms', 0)}] {e.get('agent_id', '?')}: "
                      f"{e.get('event_type', '?')}" for e in evs[:5]]
            if len(evs) > 5:
                lines.append(f"  ... and {len(evs) - 5} more events")
    return "\n".join(lines)


def export_csv(a: dict, out_dir) -> list[Path]:
    import pandas as pd

    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    written = []
    if a["flows"]:
        rows = [{"src_service": f.src_service, "dst_service": f.dst_service,
                 "src_ip": f.src_ip, "dst_ip": f.dst_ip, "src_port": f.src_port,
                 "dst_port": f.dst_port, "packets": f.packet_count, "bytes": f.bytes_total,
                 "duration_s": f.duration, "syn_count": f.syn_count,
                 "fin_count": f.fin_count, "rst_count": f.rst_count} for f in a["flows"]]
        p = out / "flows.csv"
        pd.DataFrame(rows).to_csv(p, index=False)
        written.append(p)
    cps, bps = a["connections_per_second"], a["bytes_per_second"]
    if cps or bps:
        secs = sorted(set(cps) | set(bps))
        p = out / "timeseries.csv"
        pd.DataFrame({"second": secs, "new_connections": [cps.get(s, 0) for s in secs],
                      "bytes": [bps.get(s, 0) for s in secs]}).to_csv(p, index=False)
        written.append(p)
    return written


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Analyze captured traffic and agent telemetry")
    ap.add_argument("--pcap", "-p", type=Path)
    ap.add_argument("--telemetry", "-t", type=Path)
    ap.add_argument("--output", "-o", type=Path, default=Path("logs/analysis"))
    ap.add_argument("--csv", action="store_true")
    a = ap.parse_args(argv)
    if not a.pcap and not a.telemetry:
        ap.print_help()
        print("\n[!] Please specify --pcap and/or --telemetry")
        return 1
    pa = None
    if a.pcap:
        if not a.pcap.exists():
            print(f"[!] Pcap file not found: {a.pcap}")
            return 1
        pa = analyze_pcap(a.pcap)
        print(flow_summary(pa))
    if a.telemetry:
        if not a.telemetry.exists():
            print(f"[!] Telemetry directory not found: {a.telemetry}")
            return 1
        print(telemetry_summary(analyze_telemetry(a.telemetry)))
    if a.csv and pa:
        for p in export_csv(pa, a.output):
            print(f"[*] Exported {p}")
    print("\n" + "=" * 70 + "\nANALYSIS COMPLETE\n" + "=" * 70)
    return 0


if __name__ == "__main__":
    sys.exit(main())
