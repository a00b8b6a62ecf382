#!/bin/bash
# One parametrised GPU job runner (replaces the one-off gpu_callNN.sh wrappers):
#   gpurun -- bash tools/gpu_job.sh <job> [<job> ...]
# Every GPU step runs under its own `timeout -k 10`, output goes to gpurun_out/, and the
# script stops at the first failing step (never retries a GPU step).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_PASSES=(
  "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum GRBM_GUI_ACTIVE"
  "TCC_MISS_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum"
  "TCC_EA0_WRREQ_DRAM_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
)
pytest_gpu() {   # pytest_gpu <log> <pytest args...>
  local log=$1; shift
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > "gpurun_out/$log" 2>&1 \
    || { tail -40 "gpurun_out/$log"; return 1; }
  tail -2 "gpurun_out/$log"
}
for job in "$@"; do
  echo "== job $job ($(date +%T))"
  case $job in
    tests)          pytest_gpu gpu_tests.log tests -m gpu ;;
    tests-changed)  pytest_gpu gpu_tests_changed.log tests/test_kernels_gpu.py tests/test_scan_gpu.py tests/test_custom_ar_gpu.py \
                      tests/test_prefix_sharing_gpu.py -m gpu ;;
    smoke)          timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)          timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
                    cat gpurun_out/bench.json ;;
    bench-ab)       # interleaved A/B of one environment knob: AB_ENV=NAME AB_VALS="0 1" AB_REPS=2
                    for i in $(seq ${AB_REPS:-2}); do for v in ${AB_VALS:-0 1}; do
                      env ${AB_ENV}=$v timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} \
                        > gpurun_out/ab_${v}_$i.json 2> gpurun_out/ab_${v}_$i.err || exit 1
                      echo "${AB_ENV}=$v rep $i $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$i.json)" \
                           "$(grep -o '"p50_explanation_latency_ms": [0-9.]*' gpurun_out/ab_${v}_$i.json)"
                    done; done ;;
    ingest)         hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/ingest tools/microbench/ingest.hip
                    timeout -k 10 120 /tmp/ingest | tee gpurun_out/ingest.jsonl ;;
    decode-gemm)    timeout -k 10 300 python -u tools/bench_decode_gemm.py ${DG_ARGS:-} | tee gpurun_out/decode_gemm.jsonl ;;
    decode-pmc)     for i in 0 1 2; do
                      timeout -s KILL 240 rocprofv3 --pmc ${PMC_PASSES[$i]} --kernel-include-regex \
                        "gemm_tn|gemm_pp|rmsnorm|rope_kv|splitk" -d gpurun_out/dpmc_$i -o run --output-format csv \
                        -- python3 tools/decode_step_pmc.py --layers ${DPMC_LAYERS:-4} > gpurun_out/dpmc_$i.log 2>&1 \
                        || { tail -20 gpurun_out/dpmc_$i.log; exit 1; }
                      python3 tools/pmc_summary.py "$(find gpurun_out/dpmc_$i -name '*counter_collection.csv' | head -1)" \
                        --grid > gpurun_out/dpmc_summary_$i.txt
                    done
                    cat gpurun_out/dpmc_summary_*.txt ;;
    profile)        bash tools/profile_flagship.sh ${PROF_ARGS:---steps 2 --warmup 1}
                    head -45 gpurun_out/fl_trace_summary.txt ;;
    tp8)            timeout -k 10 600 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 \
                      --batch 64 --prompt 1024 --gen 48 ${TP_ARGS:-} > gpurun_out/tp8.json 2> gpurun_out/tp8.err
                    tail -3 gpurun_out/tp8.json ;;
    tp8-trace)      rm -rf gpurun_out/prof_tp8
                    timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_tp8 -o run --output-format csv \
                      -- python3 tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 \
                      --prompt 1024 --gen 48 ${TP_ARGS:-} > gpurun_out/tp8_trace.json 2> gpurun_out/tp8_trace.err
                    python3 tools/trace_summary.py gpurun_out/prof_tp8/run_kernel_trace.csv \
                      --out gpurun_out/tp8_trace_by_shape.txt --top 60 --delete
                    tail -2 gpurun_out/tp8_trace.json; head -30 gpurun_out/tp8_trace_by_shape.txt ;;
    tp8-car)        for nb in 32 64; do   # one-shot AR+RMSNorm workgroup count
                      OAMD_CAR_BLOCKS=$nb timeout -k 10 300 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b \
                        --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp_car$nb.log 2>&1 \
                        || { tail -20 gpurun_out/tp_car$nb.log; exit 1; }
                      echo "car_blocks $nb $(grep -o '"p50_ms_per_token": [0-9.]*' gpurun_out/tp_car$nb.log)"
                    done ;;
    scan)           pytest_gpu scan_tests.log tests/test_scan_gpu.py
                    timeout -k 10 400 python -u tools/bench_scan.py --arms ${SCAN_ARMS:-profiled} --iters 20 \
                      > gpurun_out/scan_bench.jsonl
                    cat gpurun_out/scan_bench.jsonl ;;
    rehearse)       # N ranks sharing cuda:0 through torchrun + one REST API server (topology, not scaling)
                    OAMD_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
                      --nproc-per-node ${RANKS:-2} --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${RANKS:-2} \
                      ${BENCH_ARGS:---steps 2 --warmup 1} > gpurun_out/rehearse.json 2> gpurun_out/rehearse.err
                    grep '"metric"' gpurun_out/rehearse.json | tail -1 | cut -c1-1500 ;;
    power)          ( for i in $(seq 1 150); do date +%s.%N; rocm-smi -c -P -t --json 2>/dev/null; sleep 1; done ) \
                      > gpurun_out/power_samples.txt 2>&1 &
                    mon=$!
                    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_power.json \
                      2> gpurun_out/bench_power.err || { kill $mon; tail -5 gpurun_out/bench_power.err; exit 1; }
                    kill $mon || true
                    tail -c 300 gpurun_out/bench_power.json ;;
    blas-names)     # which hipBLASLt kernels F.linear runs on the prefill shapes (tile, MFMA, schedule in the name)
                    rm -rf gpurun_out/prof_blas
                    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_blas -o run --output-format csv \
                      -- python3 tools/gemm_tile_variants.py --variants 1 --m 32768 --n 4096 --k 14336 --rounds 2 \
                      > gpurun_out/blas_names.log 2>&1
                    python3 -c "import csv,collections;c=collections.Counter(r['Kernel_Name'][:200] for r in csv.DictReader(open('gpurun_out/prof_blas/run_kernel_trace.csv')));[print(n,k) for k,n in c.most_common(8)]" \
                      | tee gpurun_out/blas_kernel_names.txt
                    rm -f gpurun_out/prof_blas/run_kernel_trace.csv ;;
    gemm-tile)      timeout -k 10 300 python -u tools/gemm_tile_variants.py ${GTV_ARGS:-} | tee gpurun_out/gtv.jsonl ;;
    pmc-gemm-tile)  bash tools/pmc_gemm_tile.sh "${PMC_VARIANTS:-1 2 blas}"
                    cat gpurun_out/pmc_summary.txt ;;
    *)              echo "unknown job $job"; exit 2 ;;
  esac
done
