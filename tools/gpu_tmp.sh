export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "shared or c3" > gpurun_out/gpu_shared.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --profile-reps 1 > gpurun_out/bench_c3.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1
