# CE head pass 2: one appended dH grid row at a wide vocabulary (the MLM head's launch as before)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6y
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "cross_entropy or ce_ or head or classifier or mlm" -p no:cacheprovider > gpurun_out/r6y/tests.log 2>&1 || { tail -30 gpurun_out/r6y/tests.log; exit 1; }
tail -2 gpurun_out/r6y/tests.log
bash tools/gpu_configs.sh mlm256 seq_clf | grep "ms_per_step\|ce2\|one step" | cut -c1-200
