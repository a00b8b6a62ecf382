#!/bin/bash
# Stall breakdown of the decode GEMM at the flagship shapes (M=256): one rocprofv3 --pmc
# pass per shape (8 SQ counters), kernel trace for the time.
set -o pipefail
mkdir -p gpurun_out/stall
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
for cfg in "qkv --n 6144 --k 4096 --bm 256 --bn 128 --s 4" "down --n 4096 --k 14336 --bm 256 --bn 128 --s 8" "gate_up --n 28672 --k 4096 --bm 256 --bn 128 --s 1"; do
  set -- $cfg; name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/stall/$name -o run --output-format csv -- python3 tools/gemm_one.py --m 256 "$@" --iters 20 > gpurun_out/stall/$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/stall/$name.log; exit 1; }
  f=$(find gpurun_out/stall/$name -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$name" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "gemm_tn_kernel" in r.get("Kernel_Name", "")]
agg = collections.defaultdict(float)
for r in rows:
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
n = len({r["Dispatch_Id"] for r in rows}) or 1
w = agg["SQ_WAVE_CYCLES"] or 1
print(sys.argv[2], "dispatches", n, " ".join(f"{k}={v / n:.3g}" for k, v in sorted(agg.items())),
      f"| wait_any/wave={agg['SQ_WAIT_ANY'] / w:.2f} wait_inst_any/wave={agg['SQ_WAIT_INST_ANY'] / w:.2f} "
      f"wait_lds/wave={agg['SQ_WAIT_INST_LDS'] / w:.2f} mfma_busy/busy={agg['SQ_VALU_MFMA_BUSY_CYCLES'] / (agg['SQ_BUSY_CYCLES'] or 1):.2f}")
PY
done
