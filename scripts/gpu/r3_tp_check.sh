#!/bin/bash
# Round-3 TP rehearsal on one GPU: graph-captured TP=2/4/8 decode tests, the ADVICE graph
# regression tests, and a TP=8 bench rehearsal with a node dump of the captured graphs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-8} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
TAILN=30 run r3_tp_tests 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_tp.py tests/test_engine.py -k "graph_captured or host_collectives or unfused or ipc_allreduce"
rm -rf $OUT/graphs
ATTA_GRAPH_DUMP_DIR=$OUT/graphs run r3_tp8_bench 600 python bench.py --parallel tp --gpus 8 --tp-same-device --model llama-70b-tp-slice --steps 1 --warmup 0 --max-tokens 64 --max-num-seqs 8 --verbose
python scripts/gpu/graph_nodes.py $OUT/graphs > $OUT/r3_tp8_graph_nodes.txt 2>&1; head -40 $OUT/r3_tp8_graph_nodes.txt
