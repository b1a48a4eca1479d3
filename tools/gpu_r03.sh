#!/bin/bash
# Round-3 GPU session driver: each step has its own time limit; the first
# failing step ends the script.  usage: tools/gpu_r03.sh TAG STEP...
#   steps: new (new parity tests), tests (all -m gpu), smoke, bench, prof, e2e, wrn, infer
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -6 $O/$name.log
  [ $rc -eq 0 ] || exit $rc
}
PYT="python -u -m pytest -x -v -s --timeout 240 --timeout-method thread"
for s in "$@"; do
  case $s in
    new) step new 900 $PYT -m gpu tests/test_dp_gpu.py tests/test_ops_gpu.py tests/test_frontend_gpu.py \
           tests/test_production_gpu.py::test_strided_dgrad_wr_resnet_production tests/test_e2e_gpu.py \
           "tests/test_model_gpu.py::test_block_bf16_train_fixed_bounds" ;;
    model) step model 900 $PYT -m gpu tests/test_model_gpu.py tests/test_e2e_gpu.py tests/test_dp_gpu.py tests/test_frontend_gpu.py ;;
    pmcp) step pmcp 400 bash tools/pmc_pool.sh r03 'k_conv3x3_1w<1' ;;
    sqp) step sqp 400 bash -c "bash tools/pmc_sq.sh ${TAG}_p1w 'k_conv3x3_1w' && python tools/sq_json.py gpurun_out/pmc_${TAG}_p1w 'k_conv3x3_1w<1' r03 && python tools/sq_summary.py gpurun_out/pmc_${TAG}_p1w 'k_conv3x3_1w<2'" ;;
    sqmelr) step sqmelr 400 bash -c "bash tools/pmc_sq.sh ${TAG}_mel 'k_mel_w2' && python tools/sq_summary.py gpurun_out/pmc_${TAG}_mel k_mel_w2" ;;
    stamps) step stamps 200 python tools/pool1w_stamps.py ;;
    sqmel) step sqmel 400 bash tools/pmc_sq.sh ${TAG}_mel 'k_mel_w2' ;;
    sq64) step sq64 400 bash tools/pmc_sq.sh ${TAG}_r64 'k_conv3x3_rows<64, 8, [034], true, true>|k_wgrad3x3_halo<64, false' ;;
    bnb) step bnb 300 bash -c "python tools/bn_bench.py --C 64 && python tools/bn_bench.py --C 128" ;;
    bnab) step bnab 400 bash -c 'for r in 1 2; do for L in base bnold; do if [ $L = base ]; then E=""; else E=$PWD/abtest/$L.so; fi; echo "== $L"; ACFE_LIB=$E python tools/bn_bench.py --C 64 || exit 1; ACFE_LIB=$E python tools/bn_bench.py --C 128 || exit 1; done; done' ;;
    c16) step c16 600 $PYT -m gpu tests/test_ops_gpu.py tests/test_fused_gpu.py -k "16 or c16 or 513" ;;
    wrn) step wrn 600 python bench.py --model wrn --classes 2 --no-cpu-baseline ;;
    blk) step blk 600 $PYT -m gpu "tests/test_model_gpu.py::test_block_bf16_train_fixed_bounds" ;;
    tests) step tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
            python bench.py --no-cpu-baseline --steps 10 --warmup 3 ;;
    e2e) step e2e 900 python bench.py --workload e2e --clips ${CLIPS:-8192} --steps 40 --warmup 4 --no-cpu-baseline ;;
    wrnprof) step wrnprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wprof -o run -- \
            python bench.py --model wrn --classes 2 --no-cpu-baseline --steps 10 --warmup 3 ;;
    infer) step infer 600 python bench.py --workload infer --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
