# codec step on the GPU box: shipped build, bytes compared every run; then parity tests
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/codec_probe.py --steps 20 full cstamps > gpurun_out/codec_lane.log 2>&1
timeout -k 10 200 python -u tools/codec_probe.py --data 4k --steps 20 full >> gpurun_out/codec_lane.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py tests/test_gpu_lz4.py tests/test_gpu_spill.py >> gpurun_out/codec_lane.log 2>&1
