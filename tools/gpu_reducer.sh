# exposed data-parallel tail on one GPU: the headline step without a reducer and with the forced
# 1-rank reducer (in-graph RCCL collectives, per-bucket AdamW on the side stream), then the kernel
# timeline of a forced step (which buckets' all-reduce + update run after the last backward kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/red
mkdir -p $O
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/plain.json 2> $O/plain.err || { tail $O/plain.err; exit 1; }
PERCEIVER_BENCH_FORCE_REDUCER=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/forced.json 2> $O/forced.err || { tail $O/forced.err; exit 1; }
python - <<'PY'
import json
a = json.load(open("gpurun_out/red/plain.json")); b = json.load(open("gpurun_out/red/forced.json"))
print("plain", a["ms_per_step"], "forced reducer", b["ms_per_step"], "exposed", round(b["ms_per_step"] - a["ms_per_step"], 4), "ms",
      b["config"].get("allreduce_in_graph"), b["config"].get("allreduce_overlap"), b["config"].get("bucket_update"))
PY
PERCEIVER_BENCH_FORCE_REDUCER=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python tools/step_timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/timeline.txt
tail -30 $O/timeline.txt
