set -o pipefail
OUT=gpurun_out/r2s5_fc1g16; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for g in def 4; do
  if [ $g = def ]; then unset VPF_GEMM_GROUP; else export VPF_GEMM_GROUP=$g; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch_$g -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kernel-frames 1 --cpu-seconds 0 --no-graph > $OUT/fetch_$g.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write_$g -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kernel-frames 1 --cpu-seconds 0 --no-graph > $OUT/write_$g.log 2>&1 || exit $?
  python tools/pmc_traffic.py $OUT/fetch_$g $OUT/write_$g > $OUT/traffic_$g.json 2> $OUT/traffic_$g.err || exit $?
  python -c "import json; d=json.load(open('$OUT/traffic_$g.json')); print('group $g', {k: (v['fetch_bytes'], v['write_bytes'], v['traffic_over_algorithmic']) for k, v in d['kernels'].items()})"
done
for rep in 1 2 3; do
  for g in def 4; do
    if [ $g = def ]; then unset VPF_GEMM_GROUP; else export VPF_GEMM_GROUP=$g; fi
    timeout -k 10 300 python bench.py --steps 6 --warmup 2 --cpu-seconds 0 --kernel-frames 2 > $OUT/b_$g_r$rep.log 2>&1 || exit $?
    echo "time group=$g rep=$rep $(tail -1 $OUT/b_$g_r$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["ms_per_step"], "fc1", k["gemm_fc1"]["avg_ms"])')"
  done
done
