# One GPU call: GPU tests, bench, rocprofv3 kernel stats of the bench, then PMC passes of the emission writer.
# usage: bash scripts/gpu_round.sh TAG [kernel-regex]
TAG=${1:-round}
KRE=${2:-k_emit_assemble}
bash scripts/gpu_quick.sh "$TAG" prof || exit $?
bash scripts/gpu_pmc.sh "pmc_$TAG" "$KRE"
