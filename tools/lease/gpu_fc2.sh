set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/fc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fc_kbench.py > gpurun_out/fc_kbench3.jsonl 2>&1 || exit $?
cut -c1-150 gpurun_out/fc_kbench3.jsonl
