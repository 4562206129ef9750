# the bench's 2-rank path rehearsed on one GPU at the final HEAD (gloo, both
# ranks on cuda:0; tools/rehearse_2rank.sh)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/rehearse_2rank.sh r04s 20 5
