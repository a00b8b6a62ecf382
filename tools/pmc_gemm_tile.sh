# rocprofv3 PMC pass over gemm_tile variants and hipBLASLt on one shape (tools/gemm_tile_one.py)
# usage: [PMC="counters"] bash tools/pmc_gemm_tile.sh "1 4 blas" [extra gemm_tile_one.py args]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
C1=${PMC:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"}
rm -f gpurun_out/pmc_summary.txt
for v in $1; do
  if [ $v = blas ]; then A="--blas"; else A="--variant $v"; fi
  timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmc_$v -o run --output-format csv -- python3 tools/gemm_tile_one.py $A $2 > gpurun_out/pmc_$v.log 2>&1
  echo "== variant $v $2" >> gpurun_out/pmc_summary.txt
  python3 tools/pmc_summary.py $(find gpurun_out/pmc_$v -name "*counter_collection.csv" | head -1) --match "gemm_tile|Cijk" >> gpurun_out/pmc_summary.txt
done
