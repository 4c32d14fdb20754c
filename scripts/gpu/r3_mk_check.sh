#!/bin/bash
# Round-3: TP=8 one-GPU bench rehearsal (graph node dump), persistent decode step tests, and
# short headline benches with and without the persistent step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-8} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
rm -rf $OUT/graphs
if [ "${SKIP_TP:-0}" != 1 ]; then
ATTA_GRAPH_DUMP_DIR=$OUT/graphs run r3_tp8_bench 600 python bench.py --parallel tp --gpus 8 --tp-same-device --model llama-70b-tp-slice --steps 1 --warmup 0 --max-tokens 64 --max-num-seqs 8 --verbose
python scripts/gpu/graph_nodes.py $OUT/graphs > $OUT/r3_tp8_graph_nodes.txt 2>&1; head -30 $OUT/r3_tp8_graph_nodes.txt
fi
TAILN=20 run r3_mk_tests 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_engine.py -k "megakernel"
run r3_bench_mk 600 python bench.py --steps 2 --warmup 1 --verbose --set decode_megakernel=1
run r3_bench_base 600 python bench.py --steps 2 --warmup 1 --verbose
