set -o pipefail
export ATTA_GRAPH_DUMP_DIR=gpurun_out/graphs_push
TAG=r4tp8push STAGES=bench STEPS=1 BENCH_ARGS="--gpus 8 --parallel tp --tp-same-device --model llama-70b-tp-slice --max-tokens 64" bash scripts/gpu/stages.sh || exit 1
python scripts/gpu/graph_nodes.py gpurun_out/graphs_push > gpurun_out/r4_tp8_graph_nodes.txt; rm -rf gpurun_out/graphs_push
unset ATTA_GRAPH_DUMP_DIR
TAG=r4av8b STAGES=http STEPS=1 BENCH_ARGS="--workload agentverse" bash scripts/gpu/stages.sh || exit 1
TAG=r4av70b STAGES=http STEPS=1 BENCH_ARGS="--workload agentverse --model llama-3-70b --quantization fp8" bash scripts/gpu/stages.sh || exit 1
export ATTA_GRAPH_DUMP_DIR=gpurun_out/graphs_nopush
TAG=r4tp8nopush STAGES=bench STEPS=1 BENCH_ARGS="--gpus 8 --parallel tp --tp-same-device --model llama-70b-tp-slice --max-tokens 64 --set tp_fused_push=0" bash scripts/gpu/stages.sh || exit 1
python scripts/gpu/graph_nodes.py gpurun_out/graphs_nopush > gpurun_out/r4_tp8_graph_nodes_nopush.txt; rm -rf gpurun_out/graphs_nopush
TAG=r4pf3k STAGES=profpf TOKENS=3092 SEQS=1 bash scripts/gpu/stages.sh || exit 1
