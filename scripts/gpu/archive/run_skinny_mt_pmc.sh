set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/pmc_sk; mkdir -p $OUT
timeout -k 10 120 python3 scripts/gpu/probe_skinny_mt.py > $OUT/times.log 2>&1 || exit 1
cat $OUT/times.log
for m in 16 17; do
  for pass in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
    tag=m${m}_$(echo $pass | cut -c1-12 | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/$tag -o run -- python3 scripts/gpu/probe_skinny_mt.py --only-m $m > $OUT/$tag.log 2>&1
    rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/$tag.log; exit $rc; }
    python3 scripts/gpu/pmc_summary.py $OUT/$tag | grep -A1 "skinny_kernel" | head -2
  done
done
