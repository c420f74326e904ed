#!/bin/bash
# Round 4, second call: the full-size WGS step byte-checked unit by unit (bench --verify)
# and the tumor/normal + BAM line (device deflate of BAM records), the RCCL line at one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 700 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify > $O/verify.json 2> $O/verify.err
rc=$?; echo "verify rc=$rc"; tail -2 $O/verify.err; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/verify.json')); print('verify', d['verify'])"
timeout -k 10 300 python -u bench.py --tumor-normal > $O/tn.json 2> $O/tn.err || exit $?
python3 -c "import json; d=json.load(open('$O/tn.json')); print('tn', d['value'], d['ms_per_step'], d['bam_file_gpu'], d['with_bam_file']['value'])" || true
MH_DIST_BACKEND=nccl timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > $O/nccl1.json 2> $O/nccl1.err || exit $?
python3 -c "import json; d=[json.loads(l) for l in open('$O/nccl1.json') if l.startswith('{')][-1]; print('nccl1', d['value'], d.get('collective_backend'), d.get('world_size_seen'))" || true
echo done
