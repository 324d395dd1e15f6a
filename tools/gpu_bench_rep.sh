# repeated MLM bench runs + one kernel-trace profile (variance check on one box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/rep$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/rep$i.log').read().strip().splitlines()[-1]); print('rep $i', d['ms_per_step'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
