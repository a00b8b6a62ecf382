set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_job.sh ingest decode-sched
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_tile_gpu.py > gpurun_out/t_gt.log 2>&1 || { tail -30 gpurun_out/t_gt.log; exit 1; }
tail -2 gpurun_out/t_gt.log
for shp in "--m 32768 --n 6144 --k 4096" "--m 32768 --n 4096 --k 14336" "--m 32768 --n 28672 --k 4096 --silu"; do
  timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 1,5 $shp | tee -a gpurun_out/gtv_m32.jsonl
done
