#!/bin/bash
# Round-3 serving-stack evidence: burst-aware HTTP fan-out, config-4/5 workloads (agentverse,
# proxy) on 8B and 70B-TP1, TP=8 same-device graph node dump.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
STAGES=${STAGES:-"fanout av8 px8 av70 px70 tp8"}
for s in $STAGES; do case $s in
  fanout) run r3_http_fanout 500 python bench.py --via http --steps 3 --warmup 1 ;;
  av8) run r3_http_agentverse_8b 600 python bench.py --via http --workload agentverse --steps 2 --warmup 1 --max-tokens-limit 256 ;;
  px8) run r3_http_proxy_8b 600 python bench.py --via http --workload proxy --steps 2 --warmup 1 --max-tokens-limit 256 ;;
  av70) run r3_http_agentverse_70b 700 python bench.py --model llama-3-70b --quantization fp8 --via http --workload agentverse --steps 1 --warmup 1 --max-tokens-limit 128 ;;
  px70) run r3_http_proxy_70b 700 python bench.py --model llama-3-70b --quantization fp8 --via http --workload proxy --steps 1 --warmup 1 --max-tokens-limit 128 ;;
  e70) run r3_llama70b_tp1_fp8 600 python bench.py --model llama-3-70b --quantization fp8 --steps 1 --warmup 1 --verbose ;;
  e70b) run r3_llama70b_tp1_bf16 700 python bench.py --model llama-3-70b --steps 1 --warmup 1 --verbose ;;
  tp8) rm -rf $OUT/graphs; ATTA_GRAPH_DUMP_DIR=$OUT/graphs run r3_tp8_dump 600 python bench.py --parallel tp --gpus 8 --tp-same-device --model llama-70b-tp-slice --steps 1 --warmup 0 --max-tokens 64 --max-num-seqs 8 --verbose \
       && python scripts/gpu/graph_nodes.py $OUT/graphs > $OUT/r3_tp8_graph_nodes.txt; tail -12 $OUT/r3_tp8_graph_nodes.txt ;;
esac; done
