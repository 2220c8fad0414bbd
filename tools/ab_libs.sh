#!/bin/bash
# Build A/B variants of libvpf.so into ab_libs/ (travels to the GPU box; git-ignored): the crop's LDS window size in
# dwords (cropN). The attention's early-V-read switch (round 5's vearlyN) left the product source in round 6 (the N > 256
# steps always read early, the N <= 256 ones never: profiles/r5_lab/attn_vearly_ab.txt). The attention chunks-per-barrier
# (VPF_ATTN_CPB) and GEMM refill-spacing (VPF_ILV_SPACING) macros of rounds 1-3 are in the lab snapshots
# (tools/gemm_lab/*_lab.hip); the product sources fix them (6 and 16).
# usage: bash tools/ab_libs.sh cpb2 crop10240 ...   then  VPF_LIB_PATH=ab_libs/libvpf_cpb2.so python bench.py ...
set -e
cd "$(dirname "$0")/.."
mkdir -p ab_libs build/ab
C=vitparticlefiltertracker_amd/csrc
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fvisibility=hidden"
for v in "$@"; do
  case $v in
    crop*) src=crop; def="-DVPF_CROP_LDS_DW=${v#crop}" ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
  OBJS=""
  for s in pf_kernels crop gemm_bf16 gemm_mx8 gemm_f32 layernorm attention cls_attn; do
    [ $s = $src ] || OBJS="$OBJS build/obj/$s.o"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F $def -c $C/$src.hip -o build/ab/${src}_$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_libs/libvpf_$v.so $OBJS build/ab/${src}_$v.o
done
