# FETCH_SIZE and WRITE_SIZE passes only (separate runs) for one kernel regex.
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-bytes}
KRE=${2:-k_emit_tiles}
i=2
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
    -d gpurun_out/pmc/${TAG}_$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/pmc/${TAG}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${TAG}_$i.log; exit $rc; fi
done
