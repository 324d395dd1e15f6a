# PMC passes over the implicit-K/V attention kernels (one counter group per run)
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/pmc_pe; mkdir -p $out
timeout -k 10 120 python tools/pe_attn_bench.py --iters 20 > $out/bench.log 2>&1 || { tail $out/bench.log; exit 1; }
cat $out/bench.log
timeout -k 5 60 rocprofv3 -L > $out/avail.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python tools/pe_attn_bench.py --iters 3 > $out/kt.log 2>&1 || { tail $out/kt.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python tools/pe_attn_bench.py --iters 2 > $out/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/p$i.log; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/pmc_pe/p*/**/*counter_collection.csv', recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:40]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k, d in agg.items():
        if 'attn' in k:
            print(f.split('/')[2], k, {c: f"{v:.4g}" for c, v in d.items()})
PY
