# A/B (same box): PE forward offset folding, HEAD tree in ab_old/ vs working tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6r
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=ab_old
    (cd $d && timeout -k 10 120 python tools/pe_attn_bench.py --which fwd --iters 200) | sed "s/^/$t /" | tee -a gpurun_out/r6r/ab.log || exit 1
    (cd $d && timeout -k 10 300 python bench.py --config imagenet --steps 40 --warmup 5) | python -c "import json,sys; print('$t imagenet', json.loads(sys.stdin.read())['ms_per_step'])" | tee -a gpurun_out/r6r/ab.log || exit 2
  done
done
