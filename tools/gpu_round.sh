#!/bin/bash
# One GPU-box round: GPU parity tests, the bench line, interleaved variant timing, rocprof.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 400 python -u tools/abl_multi.py --rounds 5 ${VARIANTS:-full stamps f64 memonly loadonly nocrc nocopy} > gpurun_out/abl.jsonl 2> gpurun_out/abl.err &&
if [ -n "$PROFILE" ]; then bash profiles/run_profiles.sh gpurun_out/prof; fi
