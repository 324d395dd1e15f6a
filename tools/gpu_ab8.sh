# A/B of the 8-wave chain kernels (PIO_CHAIN8=1, default) vs the 4-wave ones (PIO_CHAIN8=0):
# phase traces, kernel/model tests for both, MLM bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab8
for pr in 1 0; do
  PIO_PRIO=$pr timeout -k 5 60 ./tools/trace/chain_trace 16384 > gpurun_out/ab8/trace_p$pr.txt 2>&1 || { echo trace failed; cat gpurun_out/ab8/trace_p$pr.txt; exit 1; }
  echo "== prio=$pr"; cat gpurun_out/ab8/trace_p$pr.txt
done
for c in 1 0; do
  PIO_CHAIN8=$c timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "sa_layer or ln_linear_post_attn or headline or mlm_fused or deterministic or bf16_dqkv or graph_engine" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab8/test_$c.log 2>&1 || { echo "test chain8=$c failed"; tail -30 gpurun_out/ab8/test_$c.log; exit 1; }
  tail -2 gpurun_out/ab8/test_$c.log
done
for v in "1 1" "1 0" "0 1" "1 1" "1 0" "0 1"; do
  set -- $v
  PIO_CHAIN8=$1 PIO_PRIO=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/ab8/mlm.json 2>gpurun_out/ab8/mlm.err || { echo "bench $v failed"; tail -20 gpurun_out/ab8/mlm.err; exit 1; }
  echo "chain8=$1 prio=$2 $(python -c "import json;d=json.load(open('gpurun_out/ab8/mlm.json'));print(d['ms_per_step'], d['value'])")"
done
