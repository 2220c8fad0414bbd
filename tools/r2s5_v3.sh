set -o pipefail
bash tools/gpu_session.sh r2s5_v3 tests smoke || exit $?
