# PMC counters of the corruption pass (one bench step)
mkdir -p gpurun_out/crpmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_cr_inplace|k_emit_tiles" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $R/gpurun_out/crpmc/p1 -o p1 --output-format csv -- python3 $R/bench.py --corrupt --no-cpu-baseline --no-e2e --steps 1 --warmup 0 > $R/gpurun_out/crpmc/b1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_cr_inplace|k_emit_tiles" --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d $R/gpurun_out/crpmc/p2 -o p2 --output-format csv -- python3 $R/bench.py --corrupt --no-cpu-baseline --no-e2e --steps 1 --warmup 0 > $R/gpurun_out/crpmc/b2.log 2>&1 || exit $?
find $R/gpurun_out/crpmc -name "*counter_collection*" | head
