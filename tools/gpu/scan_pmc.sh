#!/bin/bash
# PMC passes over the ac_scan kernel (one short bench_scan run per pass).
set -o pipefail
mkdir -p gpurun_out/scan_pmc
export TMPDIR=/tmp
ARGS="--arms profiled --iters 2 --docs 1024"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/scan_pmc/a -o a --output-format csv -- python3 tools/bench_scan.py $ARGS > gpurun_out/scan_pmc/a.log 2>&1 || { echo "pass a failed"; tail -20 gpurun_out/scan_pmc/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d gpurun_out/scan_pmc/b -o b --output-format csv -- python3 tools/bench_scan.py $ARGS > gpurun_out/scan_pmc/b.log 2>&1 || { echo "pass b failed"; tail -20 gpurun_out/scan_pmc/b.log; exit 1; }
for p in a b; do
  f=$(find gpurun_out/scan_pmc/$p -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_summary.py "$f" --match ac_scan
  rm -f "$f"
done
