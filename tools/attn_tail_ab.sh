#!/bin/bash
# A/B of the attention kernel's last key step: VPF_ATTN_TAIL=1 (attn_step_tail8) vs 0 (general masked step).
set -o pipefail
mkdir -p gpurun_out/attn_tail
PYTEST_K="attention or attn or tracker or vit" bash tools/gpu_session.sh attn_tail_tests tests || exit $?
grep -q "failed" gpurun_out/attn_tail_tests/pytest_gpu.log && exit 1
for r in 1 2; do for v in 0 1; do
  VPF_ATTN_TAIL=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/attn_tail/b_t${v}_r$r.log 2>&1 || exit $?
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/attn_tail/b_t${v}_r$r.log') if l.startswith('{')][0]
print('tail=$v r=$r', d['ms_per_step'], 'attention', d['kernels']['attention']['avg_ms'])"
done; done
