#!/bin/bash
# Instruction and wait counters (two SQ groups) of the given kernels, for this tree and for another tree of the repo
# checked out under the root (an earlier round's worktree): bash scripts/gpu_pmc_cmp.sh TAG REGEX [DIR [bench args...]]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; KRE=$2; D=${3:-.}; shift 3 2>/dev/null || shift $#
O=$GRAFT_REPO_ROOT/gpurun_out/pmccmp_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/$D"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
    -d $O/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-prime "$@" > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $O/p$i.log; exit $rc; }
done
ls $O
echo done
