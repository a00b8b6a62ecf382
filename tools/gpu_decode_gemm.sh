# One GPU call: gemm_dw / gemm_tile numerics, then the M=256 decode projections
# (tools/bench_decode_gemm.py), then (optional) PMC of the gemm_tile variants.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py tests/test_scan_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dw_tests.log 2>&1 || { tail -40 gpurun_out/dw_tests.log; exit 1; }
tail -2 gpurun_out/dw_tests.log
timeout -k 10 400 python -u tools/bench_decode_gemm.py --rounds ${DW_ROUNDS:-4} --out gpurun_out/dw_bench.jsonl
if [ -n "$PMC_VARIANTS" ]; then bash tools/pmc_gemm_tile.sh "$PMC_VARIANTS" && cat gpurun_out/pmc_summary.txt; fi
