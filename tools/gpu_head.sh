# Full GPU check of HEAD: every gpu test, the MLM headline bench, and a per-step kernel breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/head
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/test.log | tail -30
[ $rc -le 1 ] || { echo "test run aborted rc=$rc"; tail -30 $O/test.log; exit $rc; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/mlm.json 2>$O/mlm.err || { echo "bench failed"; tail -20 $O/mlm.err; exit 1; }
cat $O/mlm.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/step_breakdown.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/breakdown.md
head -60 $O/breakdown.md
timeout -k 5 60 ./tools/trace/attn_bwd_trace > $O/attn_bwd_trace.txt 2>&1 || { echo trace failed; cat $O/attn_bwd_trace.txt; exit 1; }
timeout -k 5 60 ./tools/trace/chain_trace 16384 > $O/chain_trace.txt 2>&1 || { echo trace failed; cat $O/chain_trace.txt; exit 1; }
echo done
