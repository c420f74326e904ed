# PMC passes (one rocprofv3 run per counter group) for one kernel regex; groups separated by ';' in $PMC_GROUPS.
# usage: PMC_GROUPS="A B;C D" bash scripts/gpu_pmc_groups.sh TAG KERNEL_REGEX
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-grp}
KRE=${2:-k_emit_tiles}
i=0
IFS=';' read -ra GS <<< "$PMC_GROUPS"
for grp in "${GS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
    -d gpurun_out/pmc/${TAG}_$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/pmc/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${TAG}_$i.log; exit $rc; fi
done
