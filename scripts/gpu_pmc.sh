# PMC counters for the emission kernel, one counter group per rocprofv3 pass (kernel trace only, no sys-trace).
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-pmc}
KRE=${2:-k_emit_write}
BARGS=${3:-}   # extra bench.py arguments (e.g. --corrupt)
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
    -d gpurun_out/pmc/${TAG}_$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e $BARGS \
    > gpurun_out/pmc/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${TAG}_$i.log; exit $rc; fi
done
ls gpurun_out/pmc | head -40
