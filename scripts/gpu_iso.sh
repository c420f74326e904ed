#!/bin/bash
# Kernel times in isolation: the WGS bench under rocprofv3 with every kernel serialised (AMD_SERIALIZE_KERNEL=3), so
# no kernel shares the GPU with another — each kernel's own cost, not its cost beside the FASTQ writers.
#   bash scripts/gpu_iso.sh TAG [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/iso_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export AMD_SERIALIZE_KERNEL=3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-prime "$@" > $O/bench.json 2> $O/bench.err || exit $?
python3 scripts/kstats.py $(ls $O/prof/*kernel_stats.csv | head -1) 3 16
echo done
