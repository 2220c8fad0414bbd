set -o pipefail
PYTEST_K="checkpoint or estimate_resample or multirank or tracker" bash tools/gpu_session.sh r2s5_v2 tests smoke pmc8 bench8 || exit $?
