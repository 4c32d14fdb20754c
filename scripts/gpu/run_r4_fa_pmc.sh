# PMC passes over the flash prefill kernel (Hq 32, causal 3092 tokens): instruction mix and
# pipe occupancy.  One pass per counter group (slot limits), each under its own kill timer.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/pmc_fa${FA_TAG:-}; mkdir -p $OUT
P="python3 scripts/gpu/microbench_prefill_attn.py --impls flash --hq 32 --n 3092"
pass() {
  local name=$1 ctrs=$2
  echo "=== $name: $ctrs"
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/$name -o run -- $P > $OUT/$name.log 2>&1
  local rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
  python3 scripts/gpu/pmc_summary.py $OUT/$name | grep -A1 flash_prefill | head -4
}
pass sq1 "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY"
pass sq2 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY"
