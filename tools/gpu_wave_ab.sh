#!/bin/bash
# Diagnostic: parity tests of the decode, then interleaved timing of the wave-path variants on
# the 4k and zipf configs (tools/abl_multi.py).
set -o pipefail
mkdir -p gpurun_out/wave_ab
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_decode.py tests/test_gpu_bad_entry.py tests/test_gpu_spill.py tests/test_gpu_fullsize.py} -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/wave_ab/pytest.log 2>&1 || { tail -40 gpurun_out/wave_ab/pytest.log; exit 1; }
tail -2 gpurun_out/wave_ab/pytest.log
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 9 --steps 10 ${VARIANTS:-full oldwave r1} > gpurun_out/wave_ab/abl_4k.jsonl 2> gpurun_out/wave_ab/abl_4k.err || exit 1
cat gpurun_out/wave_ab/abl_4k.jsonl
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 7 --steps 10 --config zipf ${VARIANTS2:-full oldwave} > gpurun_out/wave_ab/abl_zipf.jsonl 2> gpurun_out/wave_ab/abl_zipf.err || exit 1
cat gpurun_out/wave_ab/abl_zipf.jsonl
