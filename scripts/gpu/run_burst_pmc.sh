#!/bin/bash
# PMC passes over the cached-burst prefill GEMMs (85 rows, padded to the tuned table's 96-row
# bucket): hipBLASLt (tuned table) and the hand-written prefill GEMM side by side, per projection.
# Evidence for what bounds the p50-TTFT step (MFMA busy share, wait share, L2 traffic, HBM bytes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/pmc_burst; mkdir -p $OUT
P="python3 scripts/gpu/bench_prefill_gemm.py --m 96 --iters 10 --copies 2 --rounds 1 --tuned auto"
pass() {
  local name=$1 ctrs=$2
  echo "=== $name: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/$name -o run -- $P > $OUT/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
  python3 scripts/gpu/pmc_summary.py $OUT/$name | head -24
}
pass sq "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" &&
pass fetch "FETCH_SIZE TCP_TCC_READ_REQ_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" &&
pass l2 "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD" &&
grep -h 'M=' $OUT/sq.log
