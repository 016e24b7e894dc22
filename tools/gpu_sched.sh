#!/bin/bash
# A/B of AMDGPU scheduling strategies for the decode unit (4k, zipf).
CONFIGS="4k zipf" VARIANTS="full smaxilp smaxmemoryclause siterativeilp" exec bash tools/gpu_r4l.sh
