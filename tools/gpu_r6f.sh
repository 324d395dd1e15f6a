# PE backward: atomic dQ vs per-key-block dQ slices (deterministic mode) — kernel time from rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
for m in "" "--det"; do
  n=atomic; [ -n "$m" ] && n=slices
  timeout -k 10 120 python tools/pe_attn_bench.py --which bwd --iters 10 $m || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python tools/pe_attn_bench.py --which bwd --iters 5 $m > $O/$n.log 2>&1 || { tail $O/$n.log; exit 2; }
  f=$(find $O/$n -name "*kernel_stats.csv" | head -1); head -6 $f
done
