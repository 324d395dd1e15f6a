set -o pipefail
mkdir -p gpurun_out/chain
cd $GRAFT_REPO_ROOT
for c in 1 0; do
  PIO_CHAIN=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chain/p$c -o run -- python tools/chain_bench.py > gpurun_out/chain/pb_$c.log 2>&1 || { echo "prof chain=$c failed"; tail -20 gpurun_out/chain/pb_$c.log; exit 1; }
done
for c in 1 0; do echo "== chain $c"; find gpurun_out/chain/p$c -name "*kernel_stats.csv" | xargs head -5 | cut -c1-220; done
