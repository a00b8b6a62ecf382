# rocprofv3 PMC passes over the v3 prefill attention kernel (16x1024 and 4x4096, GQA 32/8).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -f gpurun_out/pmc_pattn.txt
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/pmc_pattn$i -o run --output-format csv -- python3 tools/bench_prefill_attn.py --variants ${PV:-3} --shapes 16x1024,4x4096 --iters 3 > gpurun_out/pmc_pattn$i.log 2>&1
  echo "== pass $i" >> gpurun_out/pmc_pattn.txt
  python3 tools/pmc_summary.py $(find gpurun_out/pmc_pattn$i -name "*counter_collection.csv" | head -1) --match "attn_prefill_mfma32" >> gpurun_out/pmc_pattn.txt
done
cat gpurun_out/pmc_pattn.txt
