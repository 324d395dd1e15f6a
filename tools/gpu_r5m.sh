# GPU suite, then A/B of the wide-grid two-workgroups-per-CU attention backward (PIO_ATTN_QR2W)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_env_ab.sh - PIO_ATTN_QR2W=1 PIO_ATTN_QR2W=0 || exit 1
bash tools/gpu_configs.sh mlm256 || exit 1
