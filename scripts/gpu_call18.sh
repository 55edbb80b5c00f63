cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4n
for v in nw8 nw8w5; do
  SKA_SDP_FUNC_LIB_DIR=variants/$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wstack or wtower" > gpurun_out/r4n/pre_$v.log 2>&1 || { tail -20 gpurun_out/r4n/pre_$v.log; exit 1; }
  tail -1 gpurun_out/r4n/pre_$v.log
done
SKA_SDP_FUNC_LIB_DIR=variants/p512 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "test_es_gpu or test_es_fft_gpu or config2" > gpurun_out/r4n/pre_p512.log 2>&1 || { tail -20 gpurun_out/r4n/pre_p512.log; exit 1; }
tail -1 gpurun_out/r4n/pre_p512.log
scripts/kt_variants.sh gpurun_out/r4n/es/ab new:ska-sdp-func_amd p512:variants/p512 new2:ska-sdp-func_amd p5122:variants/p512 || exit 1
python3 scripts/ab_table.py gpurun_out/r4n/es new p512 new2 p5122 --top 14
scripts/gpu_r4_tower.sh gpurun_out/r4n new:ska-sdp-func_amd nw8:variants/nw8 nw8w5:variants/nw8w5
