# 64k config on the GPU box: bigwave parity tests, then timings + stamps
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_spill.py tests/test_gpu_fullsize.py > gpurun_out/big.log 2>&1
timeout -k 10 300 python -u tools/abl_multi.py --rounds 3 --config 64k --blocks 65536 full bwnocrc bwnocopy > gpurun_out/big_t.log 2>&1
