#!/bin/bash
# PMC passes of one kernel on one bench line, one counter group per rocprofv3 pass (kernel trace only, no sys-trace),
# summarised into profiles/pmc_<kernel>_<round>.json (scripts/pmc_summary.py; bench.py reads traffic from it).
# usage: bash scripts/gpu_pmc.sh TAG KERNEL ROUND WORKLOAD RLEN LENGTH [bench args...]
#   e.g. bash scripts/gpu_pmc.sh r04wgs k_emit_tiles r04_wgs wgs 150 3095693981
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; KRE=$2; RND=$3; WL=$4; RLEN=$5; LEN=$6; shift 6
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
    -d gpurun_out/pmc/${TAG}_$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e "$@" \
    > gpurun_out/pmc/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${TAG}_$i.log; exit $rc; fi
done
ALG=$(grep '^{' gpurun_out/pmc/${TAG}_3.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['algorithmic_bytes_per_launch'])")
python3 scripts/pmc_summary.py gpurun_out/pmc $TAG $KRE $RND $RLEN $LEN $ALG $WL
