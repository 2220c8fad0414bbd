#!/bin/bash
# Frame-level A/B of a variant library against the product on one box: bench.py (no CPU baseline) alternately with the
# product libvpf.so and with VPF_LIB_PATH=ab_libs/libvpf_<variant>.so, REPS pairs, each run under its own time limit.
# usage: bash tools/bench_ab.sh <tag> <variant> [reps] [extra bench.py args...]
TAG=$1; V=$2; REPS=${3:-3}; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $REPS); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --kernel-frames 1 --cpu-baseline off "$@" > $OUT/bab_product_$r.log 2>&1 || exit $?
  VPF_LIB_PATH=ab_libs/libvpf_$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --kernel-frames 1 --cpu-baseline off "$@" > $OUT/bab_${V}_$r.log 2>&1 || exit $?
  python - "$OUT/bab_product_$r.log" "$OUT/bab_${V}_$r.log" <<'PY'
import json, sys
def ms(p):
    t = open(p).read(); i = t.find('{"metric"'); return json.loads(t[i:].split("\n")[0])["ms_per_step"]
a, b = ms(sys.argv[1]), ms(sys.argv[2])
print(f"product {a:.3f} ms   variant {b:.3f} ms   ratio {b / a:.4f}", flush=True)
PY
done
