#!/bin/bash
# One GPU session: each GPU step under its own time limit; stop at the first crash / timeout / abort.
# Usage: tools/gpu_session.sh <tag> [host] [tests] [scale] [smoke] [bench] [bench_l] [bench8] [prof] [pmc] [pmcmfma] [pmc8]
#        [pfprobe] [cpuframe] [lab]
#   env: PYTEST_K (pytest -k filter for "tests"), LAB_SHAPES / LAB_VARS (gemm_lab filters)
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
ok_or_stop() {  # rc 0 (pass) / 1 (test failures) continue; anything else = crash/timeout -> stop
  local rc=$1 what=$2
  echo "[$what] rc=$rc" | tee -a $OUT/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $what (rc=$rc)" | tee -a $OUT/status.txt; exit $rc; fi
}
rocm-smi --showproductname > $OUT/gpu.txt 2>&1 || true
for step in "$@"; do
  case $step in
    tests)
      VPF_TEST_REPORT_DIR=$OUT/reports timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 900 --timeout-method thread -rf ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
      ok_or_stop $? tests; tail -30 $OUT/pytest_gpu.log ;;
    host)   # the box's CPU share (bench.py cpu_baseline's core count) and model
      { echo "nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') OMP_NUM_THREADS=$OMP_NUM_THREADS";
        cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; free -g | head -2; } > $OUT/host.txt 2>&1
      cat $OUT/host.txt ;;
    scale)  # the benchmark-size parity tests alone (tests/test_gpu_scale.py)
      timeout -k 10 1100 python -u -m pytest tests/test_gpu_scale.py -m gpu -v -p no:cacheprovider --timeout 900 --timeout-method thread -rf > $OUT/pytest_scale.log 2>&1
      ok_or_stop $? scale; tail -15 $OUT/pytest_scale.log ;;
    attnab)
      timeout -k 10 300 python tools/attn_ab.py $ATTN_VARIANTS > $OUT/attn_ab.log 2>&1
      ok_or_stop $? attnab; cat $OUT/attn_ab.log | grep -v amdgpu.ids ;;
    gemmab)   # GEMM_VARIANTS e.g. 1,5,17; GEMM_SHAPES e.g. qkv,proj,fc1,fc2
      timeout -k 10 600 python tools/gemm_ab.py ${GEMM_ROUNDS:-5} ${GEMM_SHAPES:-qkv,proj,fc1,fc2} ${GEMM_VARIANTS:-1,17} > $OUT/gemm_ab.log 2>&1
      ok_or_stop $? gemmab; grep -v amdgpu.ids $OUT/gemm_ab.log ;;
    pfprobe)
      timeout -k 10 300 python tools/pf_probe.py > $OUT/pf_probe.log 2>&1
      ok_or_stop $? pfprobe; cat $OUT/pf_probe.log | grep particles ;;
    cpuframe)
      timeout -k 10 900 python tools/cpu_frame.py > $OUT/cpu_frame.log 2> $OUT/cpu_frame.err
      ok_or_stop $? cpuframe; tail -2 $OUT/cpu_frame.err; cut -c1-600 $OUT/cpu_frame.log ;;
    smoke)
      timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      ok_or_stop $? smoke; tail -5 $OUT/smoke.log ;;
    bench)   # the driver's command (N = 1), with its full-frame cpu_baseline
      timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2> $OUT/bench.err
      ok_or_stop $? bench; tail -3 $OUT/bench.log ;;
    bench_l)
      timeout -k 10 900 python bench.py --arch vit_large_patch14_336 --steps 2 --warmup 1 --cpu-baseline off > $OUT/bench_l.log 2>&1
      ok_or_stop $? bench_l; tail -1 $OUT/bench_l.log | cut -c1-400 ;;
    bench_np)
      VPF_GEMM_PERSISTENT=0 timeout -k 10 900 python bench.py --steps 5 --warmup 2 --cpu-baseline off > $OUT/bench_np.log 2>&1
      ok_or_stop $? bench_np; tail -1 $OUT/bench_np.log | cut -c1-400 ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $OUT/prof.log 2>&1
      ok_or_stop $? prof; tail -3 $OUT/prof.log ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmc_fetch.log 2>&1
      ok_or_stop $? pmc_fetch
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmc_write.log 2>&1
      ok_or_stop $? pmc_write
      python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write > $OUT/pmc_traffic.json 2> $OUT/pmc_traffic.err
      ok_or_stop $? pmc_traffic; cat $OUT/pmc_traffic.json | head -40 ;;
    prof512)   # kernel trace of the 8-GPU share (512 particles): idle gaps between graph kernels
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof512 -o run --output-format csv -- python3 bench.py --particles 512 --steps 5 --warmup 2 --kernel-frames 1 --cpu-baseline off > $OUT/prof512.log 2>&1
      ok_or_stop $? prof512
      python tools/trace_gaps.py $OUT/prof512/run_kernel_trace.csv > $OUT/gaps512.txt 2>&1; cat $OUT/gaps512.txt ;;
    pmcmfma)   # MFMA-busy and clock of every kernel of the bench frame (one pass: 2 SQ + 1 GRBM counters)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_mfma -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmc_mfma.log 2>&1
      ok_or_stop $? pmc_mfma
      python tools/pmc_frame.py $OUT/pmc_mfma --frames 3 > $OUT/pmc_mfma_frame.txt 2>&1
      ok_or_stop $? pmc_frame; cat $OUT/pmc_mfma_frame.txt ;;
    pmc_l)   # PMC traffic of configs[3] (ViT-L/14 @ 336, 4096 particles, bf16): bench.py's roofline.traffic for that line
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmcl_fetch -o p --output-format csv -- python3 bench.py --arch vit_large_patch14_336 --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmcl_fetch.log 2>&1
      ok_or_stop $? pmcl_fetch
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmcl_write -o p --output-format csv -- python3 bench.py --arch vit_large_patch14_336 --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmcl_write.log 2>&1
      ok_or_stop $? pmcl_write
      python tools/pmc_traffic.py $OUT/pmcl_fetch $OUT/pmcl_write --arch vit_large_patch14_336 --particles 4096 --frame 224x224 > $OUT/pmc_traffic_vitl.json 2> $OUT/pmcl_traffic.err
      ok_or_stop $? pmcl_traffic; head -40 $OUT/pmc_traffic_vitl.json ;;
    prof_l)   # rocprofv3 kernel stats of configs[3] (ViT-L/14 @ 336)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof_l -o run --output-format csv -- python3 bench.py --arch vit_large_patch14_336 --steps 2 --warmup 1 --cpu-baseline off > $OUT/prof_l.log 2>&1
      ok_or_stop $? prof_l; tail -1 $OUT/prof_l.log | cut -c1-300 ;;
    pmc8)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc8_fetch -o p --output-format csv -- python3 bench.py --dtype fp8 --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmc8_fetch.log 2>&1
      ok_or_stop $? pmc8_fetch
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc8_write -o p --output-format csv -- python3 bench.py --dtype fp8 --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmc8_write.log 2>&1
      ok_or_stop $? pmc8_write
      python tools/pmc_traffic.py $OUT/pmc8_fetch $OUT/pmc8_write --dtype fp8 > $OUT/pmc_traffic_fp8.json 2> $OUT/pmc8_traffic.err
      ok_or_stop $? pmc8_traffic; head -40 $OUT/pmc_traffic_fp8.json ;;
    pmc8_c4)   # PMC traffic of configs[4]'s per-GPU share (8192 particles, fp8, 1080p)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc8c4_fetch -o p --output-format csv -- python3 bench.py --preset 4 --particles 8192 --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmc8c4_fetch.log 2>&1
      ok_or_stop $? pmc8c4_fetch
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc8c4_write -o p --output-format csv -- python3 bench.py --preset 4 --particles 8192 --steps 1 --warmup 1 --kernel-frames 1 --cpu-baseline off --no-graph > $OUT/pmc8c4_write.log 2>&1
      ok_or_stop $? pmc8c4_write
      python tools/pmc_traffic.py $OUT/pmc8c4_fetch $OUT/pmc8c4_write --dtype fp8 --particles 8192 --frame 1080x1920 > $OUT/pmc_traffic_fp8_c4.json 2> $OUT/pmc8c4_traffic.err
      ok_or_stop $? pmc8c4_traffic; head -40 $OUT/pmc_traffic_fp8_c4.json ;;
    bench_c4)   # configs[4]'s per-GPU share: 8192 particles, fp8, 1080p
      timeout -k 10 900 python bench.py --preset 4 --particles 8192 --steps 5 --warmup 2 --cpu-baseline off > $OUT/bench_c4.log 2>&1
      ok_or_stop $? bench_c4; tail -1 $OUT/bench_c4.log | cut -c1-400 ;;
    bench_shares)   # the 2 / 4 / 8-GPU shares of the 4096-particle frame on one GPU (the scaling proxy)
      for P in 2048 1024 512; do
        timeout -k 10 600 python bench.py --particles $P --steps 10 --warmup 3 --cpu-baseline off > $OUT/bench_p$P.log 2>&1
        ok_or_stop $? bench_p$P; tail -1 $OUT/bench_p$P.log | cut -c1-200
      done ;;
    bench_p512)   # the 8-GPU share of the 4096-particle frame
      timeout -k 10 600 python bench.py --particles 512 --steps 10 --warmup 3 --cpu-baseline off > $OUT/bench_p512.log 2>&1
      ok_or_stop $? bench_p512; tail -1 $OUT/bench_p512.log | cut -c1-400 ;;
    prof_c4)   # rocprofv3 kernel stats of configs[4]'s per-GPU share
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- python3 bench.py --preset 4 --particles 8192 --steps 3 --warmup 1 --cpu-baseline off > $OUT/prof_c4.log 2>&1
      ok_or_stop $? prof_c4; tail -1 $OUT/prof_c4.log | cut -c1-300 ;;
    bench8)
      timeout -k 10 900 python bench.py --dtype fp8 --steps 5 --warmup 2 --cpu-baseline off > $OUT/bench8.log 2>&1
      ok_or_stop $? bench8; tail -1 $OUT/bench8.log | cut -c1-600 ;;
    libab=*)   # libab=<variant>=<cases>: lib_ab.py against ab_libs/libvpf_<variant>.so (tools/variant_lib.py builds it)
      IFS='=' read -r _ vname vcases <<< "$step"
      timeout -k 10 600 python tools/lib_ab.py ${LIBAB_ROUNDS:-7} $vcases ab_libs/libvpf_$vname.so > $OUT/lib_ab_$vname.log 2>&1
      ok_or_stop $? libab_$vname; grep -v amdgpu.ids $OUT/lib_ab_$vname.log ;;
    nsweep)   # N <= 256 attention time per launch over token counts (tools/attn_nsweep.py)
      timeout -k 10 300 python tools/attn_nsweep.py 7 ${NSWEEP_NS:-160,192,197,208,224,240,256} > $OUT/attn_nsweep.log 2>&1
      ok_or_stop $? nsweep; grep -v amdgpu.ids $OUT/attn_nsweep.log ;;
    dist2)   # the N > 1 start on one GPU: 2 ranks over gloo (the full bench path, rehearsal) and 2 ranks over RCCL, which
             # RCCL refuses on one device: the run must end within its timeout, naming rank / world / backend
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --cpu-baseline off > $OUT/dist2_gloo.log 2>&1
      ok_or_stop $? dist2_gloo; grep -h "vpf.distributed\|multi_rank_check" $OUT/dist2_gloo.log | cut -c1-300
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 tools/rccl_probe.py > $OUT/dist2_nccl_one_gpu.log 2>&1
      echo "[dist2_nccl_one_gpu] rc=$? (expected non-zero: RCCL refuses two ranks on one device)" | tee -a $OUT/status.txt
      grep -h "vpf.distributed\|Duplicate\|Error\|error" $OUT/dist2_nccl_one_gpu.log | head -12 | cut -c1-300 ;;
    benchq)   # the bench line without the CPU baseline (per-kernel table, roofline) for quick A/Bs of the product
      timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-baseline off > $OUT/benchq.log 2>&1
      ok_or_stop $? benchq; tail -1 $OUT/benchq.log | cut -c1-700 ;;
    libab)   # same-process A/B of the product library against LIBAB_LIB (default ab_libs/libvpf_direct.so)
      timeout -k 10 600 python tools/lib_ab.py ${LIBAB_ROUNDS:-7} ${LIBAB_CASES:-bf16_qkv,bf16_proj,bf16_fc1,bf16_fc2} ${LIBAB_LIB:-ab_libs/libvpf_direct.so} > $OUT/lib_ab.log 2>&1
      ok_or_stop $? libab; grep -v amdgpu.ids $OUT/lib_ab.log ;;
    lab)
      timeout -k 10 600 tools/gemm_lab/gemm_lab 5 "$LAB_SHAPES" "$LAB_VARS" 1 > $OUT/lab.log 2>&1
      ok_or_stop $? lab; grep -v "inf TFLOP" $OUT/lab.log | tail -40 ;;
  esac
done
echo done | tee -a $OUT/status.txt
