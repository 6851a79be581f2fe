# Round-3 validation: whole GPU suite + smoke, the 1-GPU bench line, the Pong kernel profile.
set -o pipefail
mkdir -p gpurun_out
bash tools/lease/gpu_tests_all.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
tail -c 600 gpurun_out/bench_default.json
bash tools/prof_pong.sh
