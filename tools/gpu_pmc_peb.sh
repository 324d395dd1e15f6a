# PMC passes over the factored PE attention backward (tools/pe_attn_bench.py --which bwd: per-sample
# queries, the weight-shared layer_n case) and the forward; one counter group per run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmc_peb; mkdir -p $out
timeout -k 10 120 python tools/pe_attn_bench.py --which both --iters 20 > $out/bench.log 2>&1 || { tail $out/bench.log; exit 1; }
cat $out/bench.log
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python tools/pe_attn_bench.py --which both --iters 2 > $out/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/p$i.log; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/pmc_peb/p*/**/*counter_collection.csv', recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:48]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k, d in agg.items():
        if '_pe' in k:
            print(f.split('/')[2], k, {c: f"{v:.4g}" for c, v in d.items()})
PY
