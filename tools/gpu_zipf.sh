# zipf config on the GPU box: determinism, timings + stamps (zipf, 4k), decode parity tests
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/determinism.py zipf > gpurun_out/zipf.log 2>&1
timeout -k 10 300 python -u tools/abl_multi.py --rounds 5 --config zipf full stamps >> gpurun_out/zipf.log 2>&1
timeout -k 10 300 python -u tools/abl_multi.py --rounds 5 --config 4k full stamps >> gpurun_out/zipf.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_spill.py tests/test_gpu_fullsize.py >> gpurun_out/zipf.log 2>&1
