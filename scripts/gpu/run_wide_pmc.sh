#!/bin/bash
# PMC passes over the wide small-M GEMM at the cached-burst row count (75 rows, every 8B
# projection, cold weights; scripts/gpu/bench_wide.py eager loop): MFMA busy share, wait
# share, LDS instructions and bank conflicts (the XOR-swizzled x image), fetched bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/pmc_wide; mkdir -p $OUT
P="python3 scripts/gpu/bench_wide.py --m ${M:-75}"
pass() {
  local name=$1 ctrs=$2
  echo "=== $name: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/$name -o run -- $P > $OUT/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
  python3 scripts/gpu/pmc_summary.py $OUT/$name | head -24
}
pass sq "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" &&
pass fetch "FETCH_SIZE TCP_TCC_READ_REQ_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" &&
pass mix "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
