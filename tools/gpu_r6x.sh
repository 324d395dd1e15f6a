# A/B (same box): CE head pass 2 — in-tile one-hot for classifier-sized vocabularies, more dH workgroups
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6x
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "cross_entropy or ce_ or head or classifier or mlm or deterministic" -p no:cacheprovider > gpurun_out/r6x/tests.log 2>&1 || { tail -30 gpurun_out/r6x/tests.log; exit 1; }
tail -2 gpurun_out/r6x/tests.log
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=ab_old
    for cfg in seq_clf seq_clf_ft mlm256; do
      (cd $d && timeout -k 10 300 python bench.py --config $cfg --steps 40 --warmup 5) | python -c "import json,sys; print('$t $cfg', json.loads(sys.stdin.read())['ms_per_step'])" | tee -a gpurun_out/r6x/ab.log || exit 3
    done
  done
done
bash tools/gpu_configs.sh seq_clf > /dev/null && grep -h "one step\|ce2" gpurun_out/cfg/seq_clf/breakdown.md | tee -a gpurun_out/r6x/ab.log
