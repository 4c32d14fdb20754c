#!/usr/bin/env bash
# Install tcpdump + BCC tools + bpftrace used by scripts/traffic.
set -euo pipefail
sudo apt-get update
sudo apt-get install -y tcpdump bpfcc-tools bpftrace "linux-headers-$(uname -r)" || \
  sudo apt-get install -y tcpdump bpfcc-tools bpftrace
echo "[ok] tcpconnect/tcplife/tcprtt/tcpretrans available as *-bpfcc"
