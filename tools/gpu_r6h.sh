# round-6: slab-traffic A/B of the latent attention backward, then the convergence study at HEAD:
# MLM with 64 latents (the two-wave head-width-16 attention backward, the README run's latent
# count) and 256 latents (the headline: persistent forward), fused bf16 graph vs eager fp32
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/conv6
timeout -k 10 240 python -u tools/slab_ab.py > gpurun_out/conv6/slab_ab.log 2>&1 || { tail -20 gpurun_out/conv6/slab_ab.log; exit 1; }
cat gpurun_out/conv6/slab_ab.log
timeout -k 10 500 python -u tools/convergence.py --task mlm --latents 64 --steps 2000 --seeds 3,4 --out gpurun_out/conv6/r6_convergence_mlm64.json > gpurun_out/conv6/mlm64.log 2>&1 || { tail -20 gpurun_out/conv6/mlm64.log; exit 1; }
tail -4 gpurun_out/conv6/mlm64.log
timeout -k 10 500 python -u tools/convergence.py --task mlm --latents 256 --steps 2000 --seeds 3 --out gpurun_out/conv6/r6_convergence_mlm256.json > gpurun_out/conv6/mlm256.log 2>&1 || { tail -20 gpurun_out/conv6/mlm256.log; exit 1; }
tail -4 gpurun_out/conv6/mlm256.log
