# implicit-K/V kernels: GPU tests, then the ImageNet-shape bench for both forward occupancies
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "implicit or pe_gemm or bwd_pe_fused" > gpurun_out/impl_k.log 2>&1 || { tail -40 gpurun_out/impl_k.log; exit 1; }
tail -3 gpurun_out/impl_k.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_gpu.py -k "image_classifier_fused_matches" > gpurun_out/impl_m.log 2>&1 || { tail -40 gpurun_out/impl_m.log; exit 1; }
tail -3 gpurun_out/impl_m.log
for occ in 4 3; do
  PIO_PEF_OCC=$occ timeout -k 10 300 python bench.py --config imagenet --steps 20 --warmup 5 > gpurun_out/impl_bench_$occ.json 2> gpurun_out/impl_bench.err || { tail gpurun_out/impl_bench.err; exit 1; }
  echo "occ=$occ $(python -c "import json;d=json.load(open('gpurun_out/impl_bench_$occ.json'));print(d['ms_per_step'])")"
done
