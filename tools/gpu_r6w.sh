# A/B (same box): dropout hash with the per-element index product hoisted (bitwise-identical masks)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6w
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "drop or seq_clf or persist or chain or attn or attention or classifier" -p no:cacheprovider > gpurun_out/r6w/tests.log 2>&1 || { tail -30 gpurun_out/r6w/tests.log; exit 1; }
tail -2 gpurun_out/r6w/tests.log
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=ab_old
    (cd $d && timeout -k 10 300 python bench.py --config seq_clf_ft --steps 40 --warmup 5) | python -c "import json,sys; print('$t seq_clf_ft', json.loads(sys.stdin.read())['ms_per_step'])" | tee -a gpurun_out/r6w/ab.log || exit 3
  done
done
bash tools/gpu_configs.sh seq_clf_ft > /dev/null && head -14 gpurun_out/cfg/seq_clf_ft/breakdown.md | tee -a gpurun_out/r6w/ab.log
