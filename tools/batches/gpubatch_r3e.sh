# round 3: graphed-inference + parity tests, SQ counters on the five 16-bit conv shapes with the
# most time in a bf16 step, the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py::test_graphed_small_chunk_inference_equals_eager tests/test_parity16_gpu.py::test_predictor_f16_vs_torch_autocast tests/test_configs4_gpu.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r3e_new.log 2>&1
rc=$?
grep -E "PASS|FAIL|classes|S=|Error" gpurun_out/r3e_new.log | tail -20
case $rc in 0|1) ;; *) echo "tests rc=$rc: stop"; exit $rc;; esac
SPECS=""
run_shape () {  # name, conv_bench args
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq_${n}_a -o run -- python3 tools/conv_bench.py "$@" > gpurun_out/sq_${n}_a.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq_${n}_b -o run -- python3 tools/conv_bench.py "$@" > gpurun_out/sq_${n}_b.log 2>&1 || return 1
  SPECS="$SPECS $n=gpurun_out/sq_${n}_a,gpurun_out/sq_${n}_b"
}
C="--dtype bf16 --trunks bathy --reps 3"
run_shape fwdbn_1x1_64to256_64 $C --shape 64,256,1,1,0,64 --only fwd --fused || exit 1
run_shape fwd_1x1_64to256_64 $C --shape 64,256,1,1,0,64 --only fwd || exit 1
run_shape fwdbn_3x3_64_64 $C --shape 64,64,3,1,1,64 --only fwd --fused || exit 1
run_shape fwdbn_3x3_256_16 $C --shape 256,256,3,1,1,16 --only fwd --fused || exit 1
run_shape dgrad_1x1_64to256_64 $C --shape 64,256,1,1,0,64 --only dgrad || exit 1
run_shape fwdbn_1x1_1024to256_16 $C --shape 1024,256,1,1,0,16 --only fwd --fused || exit 1
python3 tools/sq_shapes.py gpurun_out/round3_sq_shapes_bf16.json $SPECS || exit 1
timeout -k 10 700 python -u bench.py > gpurun_out/r3e_bench.log 2> gpurun_out/r3e_bench.err || { tail -20 gpurun_out/r3e_bench.err; exit 1; }
tail -c 1500 gpurun_out/r3e_bench.log
echo done
