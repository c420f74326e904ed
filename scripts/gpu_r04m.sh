#!/bin/bash
# Round 4: the end-to-end leg in a fresh process (library runtime, torch runtime, after 200 GB of device memory
# allocated and freed) against the bench's in-process number.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 300 python -u scripts/e2e_fresh.py > $O/e2e_rocm.json 2> $O/e2e_rocm.err || exit $?
cat $O/e2e_rocm.json
timeout -k 10 300 python -u scripts/e2e_fresh.py --torch > $O/e2e_torch.json 2> $O/e2e_torch.err || exit $?
cat $O/e2e_torch.json
timeout -k 10 300 python -u scripts/e2e_fresh.py --frag 200 > $O/e2e_frag.json 2> $O/e2e_frag.err || exit $?
cat $O/e2e_frag.json
echo done
