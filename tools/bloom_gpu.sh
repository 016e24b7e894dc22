# Device bloom build on the GPU box: parity tests (the shipped scatter path, the gather path
# TPZ_BLOOM_GATHER, the atomic kernel TPZ_BLOOM_ATOMIC), tools/bloom_probe.py timings of each and
# a rocprofv3 kernel trace of the shipped path.
set -e
mkdir -p gpurun_out/bl2
timeout -k 10 200 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_seek.py tests/test_gpu_table.py -x -q --timeout 170 --timeout-method thread > gpurun_out/bl2/test.log 2>&1
TPZ_BLOOM_GATHER=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 170 --timeout-method thread -k "bloom or golden" > gpurun_out/bl2/test_gather.log 2>&1
TPZ_BLOOM_ATOMIC=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 170 --timeout-method thread -k "bloom or golden" > gpurun_out/bl2/test_atomic.log 2>&1
timeout -k 10 200 python -u tools/bloom_probe.py full > gpurun_out/bl2/probe.log 2>&1
TPZ_BLOOM_GATHER=1 timeout -k 10 200 python -u tools/bloom_probe.py full > gpurun_out/bl2/probe_gather.log 2>&1
TPZ_BLOOM_ATOMIC=1 timeout -k 10 200 python -u tools/bloom_probe.py full > gpurun_out/bl2/probe_atomic.log 2>&1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bl2/prof -o run -- python3 tools/bloom_probe.py full > gpurun_out/bl2/probe_prof.log 2>&1
TPZ_BLOOM_GATHER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bl2/prof_gather -o run -- python3 tools/bloom_probe.py full > gpurun_out/bl2/probe_prof_gather.log 2>&1
