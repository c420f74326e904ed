# Env-knob sweep of the steady-state bench (writer CU share, decode pass batch, stream priorities)
mkdir -p gpurun_out/sweep
cd "$GRAFT_REPO_ROOT"
run() { echo -n "$1: "; env $1 timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline 2>/dev/null | \
  python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(round(d['ms_per_step'],2))" || exit 1; }
run X=0
run MH_WRITER_CUS=7
run MH_WRITER_CUS=6
run MH_WRITER_CUS=5
run MH_DEC_BATCH=4
run MH_DEC_BATCH=40
run MH_STREAM_PRIO=0
