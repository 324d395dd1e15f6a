# round-end evidence, part 2: the exposed data-parallel tail (forced 1-rank reducer), PMC counters
# of the headline step (CE head VALU / MFMA), and the reference-compute bar of seq_clf_ft
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_reducer.sh || exit 1
bash tools/gpu_pmc_mlm.sh mlm256 || exit 1
mkdir -p gpurun_out/ref
timeout -k 10 400 python bench.py --config seq_clf_ft --backend reference --steps 5 --warmup 2 > gpurun_out/ref/seq_clf_ft.json 2> gpurun_out/ref/seq_clf_ft.err || { tail -20 gpurun_out/ref/seq_clf_ft.err; exit 1; }
cat gpurun_out/ref/seq_clf_ft.json
