mkdir -p gpurun_out/r5_bis
T="tests/test_mlp3.py::test_mlp3_one_launch_grads_vs_fp32_autograd"
for f in test_arena test_bench test_bn test_checkpoint_writer test_comm test_conv1x1_stats test_conv3x3 test_conv_fork test_conv_pick test_conv_wgrad test_ddp_gpu test_dispatch test_examples test_failures test_fused_validation test_graph_step test_horovod test_kernels test_metrics; do
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/$f.py "$T" > gpurun_out/r5_bis/$f.log 2>&1
  rc=$?
  echo "$f rc=$rc $(tail -1 gpurun_out/r5_bis/$f.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc $rc"; break; fi
done
