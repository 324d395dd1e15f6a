# round-5 convergence study: fused bf16 (graph) vs eager fp32, MLM at the headline latent count
# (256 × 64) and the image classifier (32 × 128 latents: the per-sample block kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/conv
timeout -k 10 500 python -u tools/convergence.py --task img --steps 1500 --batch 128 --seeds 3,4,5 --out gpurun_out/conv/r5_convergence_img.json > gpurun_out/conv/img.log 2>&1 || { tail -20 gpurun_out/conv/img.log; exit 1; }
tail -4 gpurun_out/conv/img.log
timeout -k 10 650 python -u tools/convergence.py --task mlm --latents 256 --steps 2000 --seeds 3,4 --out gpurun_out/conv/r5_convergence_mlm.json > gpurun_out/conv/mlm.log 2>&1 || { tail -20 gpurun_out/conv/mlm.log; exit 1; }
tail -4 gpurun_out/conv/mlm.log
