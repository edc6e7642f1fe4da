set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -3 gpurun_out/gemm_tests.log
timeout -k 10 120 python -u tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 && cat gpurun_out/gemm_bench.log
ASR_GEMM_KK256=0 timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep dW
bash tools/gpu_check.sh
