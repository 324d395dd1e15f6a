# A/B of the chain-layout kernels (PIO_CHAIN=1) against the LDS row-pass kernels (PIO_CHAIN=0):
# kernel tests, rocprof kernel stats of tools/chain_bench.py, the MLM bench, phase traces.
set -o pipefail
mkdir -p gpurun_out/chain
cd $GRAFT_REPO_ROOT
timeout -k 5 60 ./tools/trace/chain_trace 16384 > gpurun_out/chain/trace.txt 2>&1 || { echo "trace failed"; tail gpurun_out/chain/trace.txt; exit 1; }
cat gpurun_out/chain/trace.txt
for c in 1 0; do
  PIO_CHAIN=$c timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "sa_layer or ln_linear_post_attn or post_attn" --timeout 120 --timeout-method thread > gpurun_out/chain/test_$c.log 2>&1 || { echo "test chain=$c failed"; tail -30 gpurun_out/chain/test_$c.log; exit 1; }
  PIO_CHAIN=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chain/p$c -o run -- python tools/chain_bench.py > gpurun_out/chain/pb_$c.log 2>&1 || { echo "prof chain=$c failed"; tail -20 gpurun_out/chain/pb_$c.log; exit 1; }
  PIO_CHAIN=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/chain/mlm_$c.json 2>gpurun_out/chain/mlm_$c.err || { echo "bench chain=$c failed"; tail -20 gpurun_out/chain/mlm_$c.err; exit 1; }
done
for c in 1 0; do tail -1 gpurun_out/chain/test_$c.log; python - <<PY
import csv, json
rows = list(csv.DictReader(open("gpurun_out/chain/p$c/run_kernel_stats.csv")))
for r in rows[:2]: print($c, r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1000, 2))
d = json.load(open("gpurun_out/chain/mlm_$c.json")); print("chain", $c, d["ms_per_step"], d["value"])
PY
done
