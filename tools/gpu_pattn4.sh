# prefill attention: v3 (8-wave workgroups) vs v4 (4-wave workgroups, two per CU): numerics + timing
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_prefix_sharing_gpu.py -x -q -k "attn_prefill or prefix" --timeout 120 --timeout-method thread > gpurun_out/pattn4_tests.log 2>&1 || { tail -30 gpurun_out/pattn4_tests.log; exit 1; }
tail -2 gpurun_out/pattn4_tests.log
timeout -k 10 300 python -u tools/bench_prefill_attn.py --variants 3,4,3,4 --shapes 16x1024,4x4096,mixed,64x256 > gpurun_out/pattn4.jsonl 2> gpurun_out/pattn4.err || { tail -5 gpurun_out/pattn4.err; exit 1; }
grep -v SDPA gpurun_out/pattn4.jsonl
