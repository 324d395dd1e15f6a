# LArTPC K/V-projection LN-linear backward: variant / row-count microbench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6j
timeout -k 10 240 python -u tools/lartpc_kv_bench.py > gpurun_out/r6j/kv.log 2>&1 || { tail -20 gpurun_out/r6j/kv.log; exit 1; }
cat gpurun_out/r6j/kv.log
