#!/bin/bash
# PMC passes over the decode attention kernel (128-token partitions, 8 waves x 1 tile) in the
# headline's decode shapes (scripts/gpu/trace_decode_attention.py: B = 1 at 600 / 3500 tokens,
# B = 5 at 450 / 900): wait share, instruction mix, fetched bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PT=128 CTXS="600;450,450,450,450,450;900,900,900,900,900;3500"
OUT=gpurun_out/pmc_attn; mkdir -p $OUT
P="python3 scripts/gpu/trace_decode_attention.py"
pass() {
  local name=$1 ctrs=$2
  echo "=== $name: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/$name -o run -- $P > $OUT/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
  python3 scripts/gpu/pmc_summary.py $OUT/$name | grep -A1 "decode_attention" | head -8
}
pass sq "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" &&
pass fetch "FETCH_SIZE TCP_TCC_READ_REQ_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" &&
pass mix "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
