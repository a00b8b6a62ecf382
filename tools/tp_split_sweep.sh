cd $GRAFT_REPO_ROOT
for cfg in "256 512" "128 1024" "64 2048" "128 2048"; do
  set -- $cfg
  OAMD_DECODE_MIN_SPLIT=$1 OAMD_DECODE_TARGET_BLOCKS=$2 timeout -k 10 300 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp_$1_$2.log 2>&1 || exit 1
  echo "$1 $2 $(grep -o '"p50_ms_per_token": [0-9.]*' gpurun_out/tp_$1_$2.log)"
done
