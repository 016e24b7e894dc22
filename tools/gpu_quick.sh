#!/bin/bash
# Quick GPU check: parity tests + interleaved variant timing (VARIANTS="full ...").
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u tools/abl_multi.py --rounds 7 ${VARIANTS:-full stamps} > gpurun_out/abl.jsonl 2> gpurun_out/abl.err
