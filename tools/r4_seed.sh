set -o pipefail
export TMPDIR=/tmp
bash tools/ab_env.sh seed 3 "seed:" "noseed:OCRK_UNIT_SEED=0" || exit $?
