set -o pipefail
mkdir -p gpurun_out/chain
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 1 0; do
  PIO_CHAIN=$c timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "sa_layer or ln_linear_post_attn or post_attn" --timeout 120 --timeout-method thread > gpurun_out/chain/test_$c.log 2>&1 || { echo "test chain=$c failed"; tail -30 gpurun_out/chain/test_$c.log; exit 1; }
  PIO_CHAIN=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/chain/prof_$c -o run -- python tools/chain_bench.py > gpurun_out/chain/bench_$c.log 2>&1 || { echo "prof chain=$c failed"; tail -20 gpurun_out/chain/bench_$c.log; exit 1; }
  PIO_CHAIN=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/chain/mlm_$c.json 2>gpurun_out/chain/mlm_$c.err || { echo "bench chain=$c failed"; tail -20 gpurun_out/chain/mlm_$c.err; exit 1; }
done
for c in 1 0; do cat gpurun_out/chain/test_$c.log | tail -1; grep sa_layer gpurun_out/chain/bench_$c.log; find gpurun_out/chain/prof_$c -name "*kernel_stats.csv" | xargs grep -h "sa_layer" | cut -c1-160; cat gpurun_out/chain/mlm_$c.json | python -c "import json,sys; d=json.load(sys.stdin); print('chain', $c, d['ms_per_step'], d['value'])"; done
