# A/B (same box): sb_wgrad LDS row strides ≡ 32 (mod 128) vs +8; HEAD tree in ab_old/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6v
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sample_block_gpu.py > gpurun_out/r6v/tests.log 2>&1 || { tail -30 gpurun_out/r6v/tests.log; exit 1; }
tail -2 gpurun_out/r6v/tests.log
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=ab_old
    for cfg in mnist imagenet lartpc; do
      (cd $d && timeout -k 10 300 python bench.py --config $cfg --steps 40 --warmup 5) | python -c "import json,sys; print('$t $cfg', json.loads(sys.stdin.read())['ms_per_step'])" | tee -a gpurun_out/r6v/ab.log || exit 3
    done
  done
done
bash tools/gpu_configs.sh mnist > /dev/null && grep -h "sb_wgrad" gpurun_out/cfg/mnist/breakdown.md | tee -a gpurun_out/r6v/ab.log
