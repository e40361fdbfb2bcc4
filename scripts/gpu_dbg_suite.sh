# debug: the whole GPU suite up to the failing MNIST fidelity test, one process, thread census
mkdir -p gpurun_out/r5_bis2
F="tests/test_arena.py tests/test_bench.py tests/test_bn.py tests/test_checkpoint_writer.py tests/test_comm.py tests/test_conv1x1_stats.py tests/test_conv3x3.py tests/test_conv_fork.py tests/test_conv_pick.py tests/test_conv_wgrad.py tests/test_ddp_gpu.py tests/test_dispatch.py tests/test_examples.py tests/test_failures.py tests/test_fused_validation.py tests/test_graph_step.py tests/test_horovod.py tests/test_kernels.py tests/test_metrics.py"
RLA_DBG_THREADS=1 timeout -k 10 900 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu $F "tests/test_mlp3.py::test_mlp3_one_launch_grads_vs_fp32_autograd" > gpurun_out/r5_bis2/suite_upto.log 2>&1
echo "rc=$?"; grep -a "threads before\|passed\|failed" gpurun_out/r5_bis2/suite_upto.log | cut -c1-3000
