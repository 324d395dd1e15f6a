# Per-kernel A/B: for each environment setting (args; "-" = defaults) one rocprofv3 kernel-stats
# run of the bench config $BENCH_CFG (default imagenet); prints the stats rows matching $KPAT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
cfg=${BENCH_CFG:-imagenet}
pat=${KPAT:-attn}
mkdir -p gpurun_out/kab
n=0
for e in "$@"; do
  n=$((n + 1))
  [ "$e" = "-" ] && e="PIO_NOTHING=1"
  echo "== $e"
  cd /tmp
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/kab/r$n -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/kab/r$n.log 2>&1 || { echo "run failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/kab/r$n.log; exit 3; }
  cd $GRAFT_REPO_ROOT
  tail -1 gpurun_out/kab/r$n.log | cut -c1-200
  f=$(find gpurun_out/kab/r$n -name "*kernel_stats.csv" | head -1)
  python - "$f" "$pat" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if sys.argv[2] in r["Name"]:
        print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>4} avg_us={float(r["AverageNs"])/1e3:8.1f}')
PY
done
