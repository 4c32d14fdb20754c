#!/bin/bash
# PMC passes over the hand-written prefill GEMM (bf16 gate_up+SiLU M=2600, o+res M=4096 = 4096^3):
# effective clock (GRBM_GUI_ACTIVE / 8 / wall), MFMA-busy share, wait breakdown, LDS, L2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm; mkdir -p $OUT
P="python3 scripts/gpu/bench_prefill_gemm.py --iters 10 --copies 2 --schedule hybrid"
pass() {
  local name=$1 ctrs=$2 only=$3 m=$4
  echo "=== $name ($only M=$m): $ctrs"
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/$name -o run -- $P --only $only --m $m > $OUT/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
  python3 scripts/gpu/pmc_summary.py $OUT/$name | grep -A1 prefill_gemm_kernel | head -4
}
for shape in "gate_up 2600" "o+res 4096"; do
  set -- $shape
  tag=${1//+/}
  pass ${tag}_sq1 "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" $1 $2
  pass ${tag}_l2 "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" $1 $2
done
