# Round measurement: GPU tests, default bench (with CPU baseline), rocprofv3 kernel stats of the bench, then the
# FETCH_SIZE / WRITE_SIZE passes of the emission writer.  usage: bash scripts/gpu_final.sh TAG
TAG=${1:-final}
bash scripts/gpu_quick.sh "$TAG" prof || exit $?
bash scripts/gpu_pmc_bytes.sh "pmc_$TAG" k_emit_direct
