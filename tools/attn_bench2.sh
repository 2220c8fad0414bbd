#!/bin/bash
# attention-related GPU tests, then two bench runs (frame time + attention kernel average)
set -o pipefail
mkdir -p gpurun_out/attn2
PYTEST_K="attention or attn or tracker or vit" bash tools/gpu_session.sh attn2_tests tests || exit $?
grep -q "failed" gpurun_out/attn2_tests/pytest_gpu.log && exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/attn2/b_r$r.log 2>&1 || exit $?
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/attn2/b_r$r.log') if l.startswith('{')][0]
print('r=$r', d['ms_per_step'], 'attention', d['kernels']['attention']['avg_ms'], 'fc1', d['kernels']['gemm_fc1']['avg_ms'])"
done
