# round-6 PMC passes (verdict items 1 and 2): MLM headline and ImageNet steps, eager launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in mlm256 imagenet; do
  bash tools/gpu_pmc_mlm.sh $cfg > /dev/null || exit 1
  mkdir -p gpurun_out/r6s
  python tools/pmc_table.py gpurun_out/pmc_mlm/p1 gpurun_out/pmc_mlm/p2 --top 24 > gpurun_out/r6s/$cfg.md
  cp gpurun_out/pmc_mlm/summary_$cfg.md gpurun_out/r6s/
  cat gpurun_out/r6s/$cfg.md
  rm -rf gpurun_out/pmc_mlm/p1 gpurun_out/pmc_mlm/p2
done
