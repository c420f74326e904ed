#!/bin/bash
# Round 4, third call: the remaining writer / gate / unit-order arms on the WGS line; the corruption rows computed
# inside the writer against the row pass (configs[2], chr1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r04e REPS=1 bash scripts/gpu_ab.sh 'base:' 'tail4:MH_WRITER_GATE_TAIL=4' 'flat:MH_EW_FLAT=1' 'g4:MH_EW_GATHER4=1' 'fwdtail4:MH_HAP_FWD=1 MH_WRITER_GATE_TAIL=4' 'copyorder: -- --unit-order copy' 'fwdcopy:MH_HAP_FWD=1 -- --unit-order copy' 'base2:' || exit $?
TAG=r04f REPS=2 BENCH_ARGS='--workload chr1 --corrupt --steps 8 --warmup 2' bash scripts/gpu_ab.sh 'rows:' 'fused:MH_CR_FUSED=1' || exit $?
echo done
