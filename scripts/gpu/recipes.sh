#!/bin/bash
# Named GPU-box recipes over scripts/gpu/stages.sh (one per measurement this repo's profiles
# cite).  Every step runs under its own time limit; the first failure ends the call.
#
#   bash scripts/gpu/recipes.sh final          # pytest -m gpu, smoke, bench, windowed profiles
#   bash scripts/gpu/recipes.sh <name> [...]   # several recipes in order
#
# Recipes (profiles they produced in round 4):
#   final        tests + smoke + 5-step bench + profbench + 3092-token prefill profile
#                (r4_final_gpu_tier.log, r4_final_profbench_summary.txt, r4_prof_prefill3k_after_summary.txt)
#   driverlike   bench.py --gpus 1 --steps 20 --warmup 5, the driver's invocation (r4_driverlike_bench.log)
#   refresh      HTTP fan-out, 8B fp8, 70B fp8 TP=1 benches (r4_final_secondary.log)
#   tp8          TP=8 rehearsal (8 ranks on one GPU) with graph node dumps, push on / off, and the
#                AgentVerse HTTP runs on 8B and 70B fp8 (r4_tp8_*, r4_http_agentverse_*)
#   tp8fp8       TP=8 x fp8 rehearsal (8 ranks on one GPU, fused push, graph steps in the JSON line)
#   largem       large-M GEMM routing A/B vs the tuned library table (r4_prefill_gemm_largem_ab.txt)
#   flash        flash-prefill tests, microbench, elementwise probe, PMC passes (r4_flash_prefill_rework.txt)
#   burst        windowed profile of the 380-row burst prefill (r4_prof_burst380_summary.txt)
#   small        17 / 85-row prefill profiles and the cached-regime bench with the fused small-prefill
#                path on / off (r4_small_prefill_fused.txt)
# Rounds 5-6:
#   wide         wide small-M GEMM vs the library, graph replay, 33-128 rows (r5_wide_gemm.txt,
#                r6_wide_gemm_sched.txt)
#   midm         mid-M GEMM vs the tuned library and its (row block, split) sweep, 129-640 rows
#                (r6_midm_vs_tuned.txt, r6_midm_sweep.txt)
#   fp8wide      fp8 weights: wide kernel W8 builds vs the library fp8 chain, 8B and 70B shapes
#                (r6_wide_fp8.txt); fp8 mid-M route A/B on the bench (r6_midm_fp8_negative.txt)
#   coldstart    first vs repeat TTFT of every fan-out step shape on a fresh engine
#                (r6_coldstart_*.txt, tests/test_coldstart.py)
#   fanout       per-episode TTFT by phase (r5_fanout_ttft_per_episode.txt)
#   70bfp8       Llama-3-70B fp8 TP=1 bench, fused small-prefill path on / off (r6_70b_fp8.txt)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
S=scripts/gpu/stages.sh
recipe() {
  case $1 in
    final)
      TAG=r4final STAGES="tests smoke bench profbench" STEPS=${STEPS:-5} TEST_TIMEOUT=1000 bash $S &&
      TAG=r4finalpf3k STAGES=profpf TOKENS=3092 SEQS=1 bash $S ;;
    driverlike)
      timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_driverlike_bench.log 2>&1 &&
      tail -1 gpurun_out/r4_driverlike_bench.log ;;
    refresh)
      TAG=r4fin STAGES=http STEPS=3 bash $S &&
      TAG=r4fin_fp8 STAGES=bench STEPS=2 BENCH_ARGS="--quantization fp8" bash $S &&
      TAG=r4fin_70bfp8 STAGES=bench STEPS=1 BENCH_ARGS="--model llama-3-70b --quantization fp8" bash $S ;;
    tp8)
      local tp="--gpus 8 --parallel tp --tp-same-device --model llama-70b-tp-slice --max-tokens 64"
      ATTA_GRAPH_DUMP_DIR=gpurun_out/graphs_push TAG=r4tp8push STAGES=bench STEPS=1 BENCH_ARGS="$tp" bash $S &&
      python scripts/gpu/graph_nodes.py gpurun_out/graphs_push > gpurun_out/r4_tp8_graph_nodes.txt &&
      ATTA_GRAPH_DUMP_DIR=gpurun_out/graphs_nopush TAG=r4tp8nopush STAGES=bench STEPS=1 \
        BENCH_ARGS="$tp --set tp_fused_push=0" bash $S &&
      python scripts/gpu/graph_nodes.py gpurun_out/graphs_nopush > gpurun_out/r4_tp8_graph_nodes_nopush.txt &&
      rm -rf gpurun_out/graphs_push gpurun_out/graphs_nopush &&
      TAG=r4av8b STAGES=http STEPS=1 BENCH_ARGS="--workload agentverse" bash $S &&
      TAG=r4av70b STAGES=http STEPS=1 BENCH_ARGS="--workload agentverse --model llama-3-70b --quantization fp8" bash $S ;;
    tp8fp8)
      # BASELINE config 5 rehearsal: 8 TP ranks on one GPU, fp8 weights, fused push, graphs
      TAG=r5tp8fp8 STAGES=bench STEPS=1 BENCH_ARGS="--gpus 8 --parallel tp --tp-same-device \
        --model llama-70b-tp-slice-fp8 --quantization fp8 --max-tokens 64" bash $S ;;
    largem)
      TAG=r4lm_bf16 STAGES=gemm GEMM_ARGS="--m 2048 2560 3200 4096 --tuned auto --rounds 3" bash $S &&
      TAG=r4lm_fp8 STAGES=gemm GEMM_ARGS="--m 512 1024 2048 3200 --fp8 --rounds 3" bash $S ;;
    flash)
      TAG=r4fa STAGES=tests PYTEST_ARGS="tests/test_kernels_gpu.py" PYTEST_K="prefill or flash or long or norm" \
        TEST_TIMEOUT=400 bash $S &&
      TAG=r4fa STAGES=py PY_ARGS="scripts/gpu/microbench_prefill_attn.py --impls flash" PY_TIMEOUT=300 bash $S &&
      TAG=r4faew STAGES=py PY_ARGS="scripts/gpu/probe_elementwise.py --m 73 382 3200" PY_TIMEOUT=200 bash $S &&
      bash scripts/gpu/run_r4_fa_pmc.sh ;;
    burst)
      TAG=r4burst STAGES=profpf TOKENS=380 SEQS=5 REPS=5 bash $S ;;
    small)
      TAG=r4sp17 STAGES=profpf TOKENS=17 SEQS=1 REPS=10 bash $S &&
      TAG=r4sp85 STAGES=profpf TOKENS=85 SEQS=5 REPS=10 bash $S &&
      TAG=r4sf_on STAGES=bench STEPS=6 BENCH_ARGS="--warmup 5" bash $S &&
      TAG=r4sf_off STAGES=bench STEPS=6 BENCH_ARGS="--warmup 5 --set small_prefill_fused=0" bash $S ;;
    wide)
      timeout -k 10 400 python -u scripts/gpu/bench_wide.py --graph --m 33 48 64 75 80 96 112 128 \
        > gpurun_out/wide_gemm.txt 2>&1 && tail -8 gpurun_out/wide_gemm.txt ;;
    midm)
      timeout -k 10 600 python -u scripts/gpu/bench_wide.py --tuned --m 129 188 256 382 475 640 \
        > gpurun_out/midm_vs_tuned.txt 2>&1 &&
      timeout -k 10 900 python -u scripts/gpu/bench_wide.py --tuned --midm-sweep --m 188 382 475 \
        > gpurun_out/midm_sweep.txt 2>&1 && tail -4 gpurun_out/midm_vs_tuned.txt ;;
    fp8wide)
      timeout -k 10 500 python -u scripts/gpu/bench_wide.py --model 70b --fp8 --tuned --m 33 64 76 96 128 \
        > gpurun_out/wide_70b_fp8.txt 2>&1 &&
      timeout -k 10 300 python -u scripts/gpu/bench_wide.py --fp8 --tuned --m 33 75 128 \
        > gpurun_out/wide_8b_fp8.txt 2>&1 &&
      for v in 0 129-1024; do
        ATTA_MIDM_FP8_ROWS=$v timeout -k 10 400 python -u bench.py --quantization fp8 --steps 2 \
          --warmup 2 > gpurun_out/bench_8bfp8_midm_$v.log 2>&1 || return 1
      done ;;
    coldstart)
      timeout -k 10 600 python -u -m agentic_traffic_testing_amd.bench.coldstart --reps 3 \
        > gpurun_out/coldstart.txt 2>&1 && tail -1 gpurun_out/coldstart.txt ;;
    fanout)
      timeout -k 10 600 python -u scripts/gpu/probe_fanout_ttft.py --episodes 4 --warmup 5 \
        > gpurun_out/fanout_ttft.txt 2>&1 && tail -12 gpurun_out/fanout_ttft.txt ;;
    70bfp8)
      for v in 1 0; do
        timeout -k 10 560 python -u bench.py --model meta-llama/Llama-3-70B-Instruct --quantization fp8 \
          --steps 1 --warmup 1 --set small_prefill_fused=$v > gpurun_out/bench_70bfp8_spf$v.log 2>&1 || return 1
      done ;;
    *) echo "unknown recipe $1"; return 2 ;;
  esac
}
for r in "${@:-final}"; do
  echo "### recipe $r"
  recipe "$r" || { echo "STOP after recipe $r"; exit 1; }
done
