set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/base
timeout -k 5 60 ./tools/trace/chain_trace 16384 > gpurun_out/base/trace.txt 2>&1 || { echo trace failed; exit 1; }
cat gpurun_out/base/trace.txt
bash tools/gpu_step_profile.sh
