# iteration check: GPU tests of the kernels / models touched, the headline bench, a per-step
# kernel breakdown and the phase traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/iter
mkdir -p $O
K=${1:-""}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > $O/test.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/test.log | tail -30
[ $rc -le 1 ] || { echo "test run aborted rc=$rc"; tail -30 $O/test.log; exit $rc; }
[ $rc -eq 0 ] || { tail -60 $O/test.log; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/mlm.json 2>$O/mlm.err || { echo "bench failed"; tail -20 $O/mlm.err; exit 1; }
cat $O/mlm.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/step_breakdown.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/breakdown.md
head -24 $O/breakdown.md
timeout -k 5 60 ./tools/trace/attn_bwd_trace > $O/attn_bwd_trace.txt 2>&1 || { echo trace failed; cat $O/attn_bwd_trace.txt; exit 1; }
head -14 $O/attn_bwd_trace.txt
timeout -k 5 60 ./tools/trace/chain_trace 16384 > $O/chain_trace.txt 2>&1 || { echo trace failed; cat $O/chain_trace.txt; exit 1; }
echo done
