#!/bin/bash
# Round-6 GPU session: GPU parity tests + smoke, then for each workload a bench
# line and a rocprofv3 kernel-trace summary of the same command.  Every GPU step
# has its own time limit; the first failing step ends the script.
# usage: tools/gpu_r04.sh <tag> [workloads...]   (workloads: tests t1 wrn t1fp32 infer stream)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r06}; shift
O=gpurun_out/$TAG
mkdir -p $O
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -c 400 $O/$name.log; echo
  [ $rc -eq 0 ] || exit $rc
}
bp() { # name benchargs...  (bench line + rocprof of the same command)
  local name=$1; shift
  step ${name}_bench 600 python bench.py "$@"
  step ${name}_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${name}_prof -o run -- \
      python bench.py --no-cpu-baseline --no-extra "$@"
}
for w in "$@"; do
  case $w in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread
           step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    testsall) timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/testsall.log 2>&1
              rc=$?; echo "== testsall rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/testsall.log | tail -30
              case $rc in 0|1) ;; *) exit $rc ;; esac ;;
    bdef) step bdef 600 python bench.py ;;
    r64t) step r64t 300 python -u -m pytest tests/test_r64_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    t1x) step t1x_bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra ;;
    wrnq) step wrnq_bench 300 python bench.py --model wrn --classes 2 --steps 8 --warmup 3 --no-cpu-baseline --no-extra ;;
    sqr64) BENCH_ARGS='--model wrn --classes 2' step sqr64 400 bash -c "bash tools/pmc_sq.sh ${TAG}_r64 'k_conv3x3_r64' && python tools/sq_summary.py gpurun_out/pmc_${TAG}_r64 'k_conv3x3_r64<4' 'k_conv3x3_r64<3' 'k_conv3x3_r64<5'" ;;
    fwdps) step fwdps 300 python tools/fwdp_stamps.py ;;
    epp) step epp 400 python -u tools/ep_probe.py ${EPN:-8} && grep -c '"nan": 0, "inf": 0, "n": [0-9]*}}' $O/epp.log ;;
    envab) for r in 1 2 3; do for v in on off; do
             if [ $v = off ]; then export $ABVAR=0; else unset $ABVAR; fi
             step wrn_${ABVAR}_$v 300 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline --no-extra && grep -o '"value": [0-9.]*' $O/wrn_${ABVAR}_$v.log
           done; done; unset $ABVAR ;;
    cbw) step cbw 300 python tools/conv_bench.py --layers ${CBL:-6,7,8} --iters 5 ;;
    sqs3) step sqs3 400 bash -c "bash tools/pmc_sq_cmd.sh ${TAG}_s3 'k_conv_fwd_p' tools/conv_bench.py --layers 8 --passes fwd,dgrad --iters 2 && python tools/sq_summary.py gpurun_out/pmc_${TAG}_s3 'k_conv_fwd_p<128'" ;;
    r64st) step r64st 300 python tools/r64_stamps.py 512 ;;
    sq3r64) BENCH_ARGS='--model wrn --classes 2' step sq3r64 300 bash tools/pmc_sq3.sh ${TAG}_r64mix 'k_conv3x3_r64' ;;
    bnprobe) step bnprobe 300 python tools/bn_moving_probe.py ;;
    settle) step settle 400 python tools/learn_settle.py && step settle32 400 python tools/learn_settle.py fp32 ;;
    learn) step learn 400 python -u -m pytest tests/test_learning_gpu.py -x -v -s --timeout 380 --timeout-method thread ;;
    r64ab) for v in base ${LIBS}; do if [ $v = base ]; then L=$PWD/audio-training_amd/acfe/libacfe_stamps.so; else L=$PWD/abtest/$v.so; fi; echo "== $v"; ACFE_LIB=$L step r64ab_$v 300 python tools/r64_stamps.py 512 && grep -E 'ms,' $O/r64ab_$v.log; done ;;
    bench2) step bench2 600 python -u -m pytest tests/test_bench_gpu.py -x -v --timeout 420 --timeout-method thread ;;
    cpub) step cpub 900 python tools/cpu_baseline.py ;;
    wrnab) for r in 1 2; do for v in new ${LIBS}; do
             if [ $v = new ]; then L=""; else L=$PWD/abtest/$v.so; fi
             ACFE_LIB=$L step wrn_$v 300 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline --no-extra && grep -o '"value": [0-9.]*' $O/wrn_$v.log
           done; done ;;
    libab) for r in 1 2; do for v in new ${LIBS}; do
             if [ $v = new ]; then L=""; else L=$PWD/abtest/$v.so; fi
             ACFE_LIB=$L step t1_$v 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra && grep -o '"value": [0-9.]*' $O/t1_$v.log
           done; done ;;
    melw5) step melt 300 python -u -m pytest tests/test_frontend_gpu.py -x -v --timeout 120 --timeout-method thread && for v in 0 1 2 4 8 0 4; do step mel_$v 120 python tools/mel_bench.py --iters 15 --prenorm --w5 $v && grep ms $O/mel_$v.log; done ;;
    mel) step mel 300 python tools/mel_bench.py --iters 15 && step melpre 300 python tools/mel_bench.py --iters 15 --prenorm ;;
    fetests) step fetests 300 python -u -m pytest tests/test_frontend_gpu.py tests/test_e2e_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    evwrn) step evwrn 900 bash tools/pmc_evidence.sh wrn r06 'k_conv3x3_r64<4, 1, true, true, 64>' 12910141440 \
             'k_conv3x3_r64<4,1,true,true> (wr_resnet b1/b2 conv2a 3x3 64->64 @128x513 with the BN prologue + dropout + BN sums, batch 512)' \
             --model wrn --classes 2 --steps 2 --warmup 1 ;;
    evt1) step evt1 900 bash tools/pmc_evidence.sh t1 r06 'k_conv3x3_1w<1, 2, true, true, false, 64>' 5905580032 \
             'k_conv3x3_1w<1,2,true,true> (wr_resnet_bird s1b0 branch21 3x3 128->128 @128x256 + 2x2 max-pool + dropout + BN sums, batch 512)' \
             --steps 3 --warmup 1 ;;
    evinfer) SELECT=7:3 step evinfer 600 bash tools/pmc_evidence.sh infer_fp32 r06 'k_conv_fwd_g<float, 128, 64' 8606859264 \
             'k_conv_fwd_g<float,128,64> (wr_resnet b1.conv2a 3x3 64->64 @128x513 fp32, batch 256)' \
             --workload infer --steps 2 --warmup 1 ;;
    evstream) SELECT=12:1 step evstream 600 bash tools/pmc_evidence.sh stream_fp32 r06 'k_conv_fwd_g<float, 128, 128' 26832360789 \
             'k_conv_fwd_g<float,128,128> (wr_resnet_bird s1b0 conv21 3x3 128->128 @128x256 fp32; the 3 launches of a step: 1024 / 1024 / 351 windows, averaged)' \
             --workload stream --dtype fp32 --steps 1 --warmup 1 ;;
    e2e) step e2e 900 python bench.py --workload e2e --clips 8192 --steps 20 --warmup 4 ;;
    sqmel) step sqmel 400 bash -c "bash tools/pmc_sq.sh ${TAG}_mel 'k_mel_w4' && python tools/sq_summary.py gpurun_out/pmc_${TAG}_mel k_mel_w4" ;;
    t1) bp t1 --steps 20 --warmup 5 ;;
    t1p) step t1p_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t1p_prof -o run -- \
           python bench.py --no-cpu-baseline --no-extra --steps 10 --warmup 3 ;;
    wrnp) step wrnp_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wrnp_prof -o run -- \
           python bench.py --no-cpu-baseline --no-extra --model wrn --classes 2 --steps 5 --warmup 2 ;;
    layers) step layers_wrn 300 python tools/layer_profile.py 512 wrn && step layers_t1 300 python tools/layer_profile.py 512 ;;
    wrns2d0) ACFE_DGRAD_S2D=0 step wrns2d0_bench 600 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline --no-extra ;;
    wrnx) step wrnx_bench 600 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline --no-extra ;;
    infx) step infx_bench 600 python bench.py --workload infer --steps 5 --warmup 2 --no-cpu-baseline ;;
    strx) step strx_bench 600 python bench.py --workload stream --dtype fp32 --steps 3 --warmup 1 --no-cpu-baseline ;;
    inf0) ACFE_CONVG_CMAJ=0 step inf0_bench 600 python bench.py --workload infer --steps 5 --warmup 2 --no-cpu-baseline ;;
    str0) ACFE_CONVG_CMAJ=0 step str0_bench 600 python bench.py --workload stream --dtype fp32 --steps 3 --warmup 1 --no-cpu-baseline ;;
    wrnp0) ACFE_DGRAD_S2D=0 step wrnp0_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wrnp0_prof -o run -- \
           python bench.py --no-cpu-baseline --no-extra --model wrn --classes 2 --steps 5 --warmup 2 ;;
    s2db) step s2db 300 python tools/s2d_bench.py && ACFE_DGRAD_S2D=0 step s2db0 300 python tools/s2d_bench.py ;;
    trwrn) step trwrn 700 bash tools/step_traffic.sh wrn_r06 --model wrn --classes 2 ;;
    trt1) step trt1 700 bash tools/step_traffic.sh t1_r06 ;;
    wrnsub0) ACFE_SUB_FUSE=0 step wrnsub0_bench 600 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline --no-extra ;;
    e1ab) for v in base e1only base e1only; do
            if [ $v = base ]; then L=""; else L=$PWD/abtest/$v.so; fi
            ACFE_LIB=$L step s2d_$v 300 python tools/s2d_bench.py
            ACFE_LIB=$L step t1_$v 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
            ACFE_LIB=$L step wrn_$v 300 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline --no-extra
          done ;;
    apab) for v in ${APV:-base ap512 base ap512}; do
            if [ $v = base ]; then L=""; else L=$PWD/abtest/$v.so; fi
            ACFE_LIB=$L step ap_$v 300 bash -c "python tools/apply_bench.py 512 128 513 64 && python tools/apply_bench.py 512 64 128 64 && python tools/apply_bench.py 512 64 257 128"
          done ;;
    prob) step prob 300 bash -c "python tools/pro_bench.py && python tools/pro_bench.py 512 64 128" ;;
    resab) for v in new old new old; do
             if [ $v = new ]; then L=""; else L=$PWD/abtest/oldtree.so; fi
             ACFE_LIB=$L step wrn_$v 300 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline --no-extra && grep -o '"value": [0-9.]*' $O/wrn_$v.log
           done ;;
    t1nx) step t1nx_bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra ;;
    t1f0) ACFE_BN_BWD_FUSE=0 step t1f0_bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra ;;
    wrnnx) step wrnnx_bench 600 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline ;;
    wrnf0) ACFE_BN_BWD_FUSE=0 step wrnf0_bench 600 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline ;;
    ptk) step ptk 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$PTK" ;;
    ptka) timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$PTK" > $O/ptka.log 2>&1
          rc=$?; echo "== ptka rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/ptka.log | tail -40
          case $rc in 0|1|5) ;; *) exit $rc ;; esac ;;
    convtests) step convtests 600 python -u -m pytest tests/test_production_gpu.py tests/test_fused_gpu.py \
                 tests/test_ops_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    fusetests) step fusetests 600 python -u -m pytest tests/test_production_gpu.py -m gpu -k "reduce_fus" -x -v \
                 --timeout 120 --timeout-method thread ;;
    wrn0) ACFE_BN_REDUCE_FUSE=0 step wrn0_bench 600 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline ;;
    t10) ACFE_BN_REDUCE_FUSE=0 step t10_bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    wrnp0) ACFE_BN_PROLOGUE_1W=0 step wrnp0_bench 600 python bench.py --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline ;;
    protests) step protests 600 python -u -m pytest tests/test_production_gpu.py tests/test_model_gpu.py -m gpu -k "prologue or model" -v \
                 --timeout 120 --timeout-method thread ;;
    wrn) bp wrn --model wrn --classes 2 --steps 10 --warmup 3 --no-cpu-baseline ;;
    t1fp32) bp t1fp32 --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline ;;
    infer) bp infer --workload infer --steps 5 --warmup 2 ;;
    stream) bp stream --workload stream --dtype fp32 --steps 3 --warmup 1 ;;
  esac
done
echo done
