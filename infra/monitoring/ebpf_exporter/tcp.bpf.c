// CO-RE BPF programs for ebpf_exporter v2 (see tcp.yaml for the exported metrics).
#include "vmlinux.h"
#include <bpf/bpf_helpers.h>
#include <bpf/bpf_tracing.h>
#include <bpf/bpf_core_read.h>

#define MAX_SLOTS 27

struct {
  __uint(type, BPF_MAP_TYPE_ARRAY);
  __uint(max_entries, MAX_SLOTS);
  __type(key, u32);
  __type(value, u64);
} tcp_rtt_microseconds SEC(".maps");

struct {
  __uint(type, BPF_MAP_TYPE_HASH);
  __uint(max_entries, 16);
  __type(key, u32);
  __type(value, u64);
} tcp_connections_total SEC(".maps");

struct {
  __uint(type, BPF_MAP_TYPE_ARRAY);
  __uint(max_entries, 1);
  __type(key, u32);
  __type(value, u64);
} tcp_retransmits_total SEC(".maps");

static __always_inline u32 log2_slot(u64 v) {
  u32 r = 0;
  while (v > 1 && r < MAX_SLOTS - 1) {
    v >>= 1;
    r++;
  }
  return r;
}

static __always_inline void inc(void* map, u32 key) {
  u64* c = bpf_map_lookup_elem(map, &key);
  if (c) {
    __sync_fetch_and_add(c, 1);
  } else {
    u64 one = 1;
    bpf_map_update_elem(map, &key, &one, BPF_NOEXIST);
  }
}

SEC("kprobe/tcp_rcv_established")
int BPF_KPROBE(on_tcp_rcv, struct sock* sk) {
  struct tcp_sock* ts = (struct tcp_sock*)sk;
  u32 srtt = BPF_CORE_READ(ts, srtt_us) >> 3;
  inc(&tcp_rtt_microseconds, log2_slot(srtt));
  return 0;
}

SEC("tracepoint/sock/inet_sock_set_state")
int on_state(struct trace_event_raw_inet_sock_set_state* ctx) {
  if (ctx->protocol != IPPROTO_TCP) return 0;
  inc(&tcp_connections_total, (u32)ctx->newstate);
  return 0;
}

SEC("kprobe/tcp_retransmit_skb")
int BPF_KPROBE(on_retransmit) {
  inc(&tcp_retransmits_total, 0);
  return 0;
}

char LICENSE[] SEC("license") = "GPL";
