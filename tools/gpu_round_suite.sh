cd /root/repo
export PYTHONUNBUFFERED=1
R=tests/cxx/build
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r03a_gpu_suite.log 2>&1
echo "suite rc=$?" >> gpurun_out/r03a_gpu_suite.log
timeout -k 10 300 $R/DirectSortHTest_hip > gpurun_out/r03a_HTest.log 2>&1; echo "rc=$?" >> gpurun_out/r03a_HTest.log
timeout -k 10 300 $R/DirectSortH2Test_hip > gpurun_out/r03a_H2Test.log 2>&1; echo "rc=$?" >> gpurun_out/r03a_H2Test.log
timeout -k 10 300 $R/DirectSortNTest_hip > gpurun_out/r03a_NTest.log 2>&1; echo "rc=$?" >> gpurun_out/r03a_NTest.log
timeout -k 10 300 $R/SincTest_hip > gpurun_out/r03a_Sinc.log 2>&1; echo "rc=$?" >> gpurun_out/r03a_Sinc.log
timeout -k 10 300 $R/DirectSortBenchmark_hip > gpurun_out/r03a_DSBench.log 2>&1; echo "rc=$?" >> gpurun_out/r03a_DSBench.log
