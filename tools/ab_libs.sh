#!/bin/bash
# Build A/B variants of libvpf.so into ab_libs/ (travels to the GPU box; git-ignored): attention chunks-per-barrier.
# usage: bash tools/ab_libs.sh cpb2 cpb3 ...   then  VPF_LIB_PATH=ab_libs/libvpf_cpb3.so python bench.py ...
set -e
cd "$(dirname "$0")/.."
mkdir -p ab_libs build/ab
C=vitparticlefiltertracker_amd/csrc
OBJS=""
for s in pf_kernels crop gemm_bf16 gemm_mx8 gemm_f32 layernorm cls_attn; do OBJS="$OBJS build/obj/$s.o"; done
for v in "$@"; do
  n=${v#cpb}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fvisibility=hidden \
      -DVPF_ATTN_CPB=$n -c $C/attention.hip -o build/ab/attention_$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_libs/libvpf_$v.so $OBJS build/ab/attention_$v.o
done
