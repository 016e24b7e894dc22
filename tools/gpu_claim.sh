#!/bin/bash
# A/B: chunks claimed two ahead (no atomic optimizer in the decode unit) vs before.
CONFIGS="4k zipf 64k" VARIANTS="preclaim full" exec bash tools/gpu_r4l.sh
