set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_final.sh r3fin4
