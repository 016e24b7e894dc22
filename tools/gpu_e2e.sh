# host pipeline on the GPU box: the C test, then the e2e leg of bench (no other legs)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c_abi.py > gpurun_out/e2e.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline --no-file-crc --no-snappy --no-lz4 --no-seek >> gpurun_out/e2e.log 2>&1
