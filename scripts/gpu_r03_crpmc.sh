#!/bin/bash
# PMC passes of the corruption-rows mode on the chr1 corrupt bench (one step): k_cr_cols (SQ group, FETCH_SIZE,
# WRITE_SIZE) and the rows-mode writer k_emit_tiles<2, 4, 2> (FETCH_SIZE, WRITE_SIZE), each counter set in its own
# rocprofv3 pass; summarised into profiles/pmc_k_cr_cols_r03.json and profiles/pmc_k_emit_tiles_r03_corrupt.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {   # tag, kernel regex, counters
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $3 --kernel-include-regex "$2" --output-format csv \
    -d gpurun_out/pmc/$1 -o run -- python3 bench.py --workload chr1 --corrupt --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
    > gpurun_out/pmc/$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$1.log; exit $rc; fi
}
run crc_1 k_cr_cols "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
run crc_2 k_cr_cols "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run crc_3 k_cr_cols "FETCH_SIZE"
run crc_4 k_cr_cols "WRITE_SIZE"
run crw_3 k_emit_tiles "FETCH_SIZE"
run crw_4 k_emit_tiles "WRITE_SIZE"
ALGC=$(grep '^{' gpurun_out/pmc/crc_3.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['corrupt_pass']['algorithmic_bytes_per_launch'])")
ALGW=$(grep '^{' gpurun_out/pmc/crw_3.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['algorithmic_bytes_per_launch'])")
python3 scripts/pmc_summary.py gpurun_out/pmc crc k_cr_cols r03 150 249250621 $ALGC chr1_corrupt && \
python3 scripts/pmc_summary.py gpurun_out/pmc crw k_emit_tiles r03_corrupt 150 249250621 $ALGW chr1_corrupt
