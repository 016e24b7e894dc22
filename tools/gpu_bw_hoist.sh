#!/bin/bash
# A/B: bigwave CRC padding shift issued before the first group's loads (full) vs at the block's end (bwprev).
CONFIGS="64k" VARIANTS="full" bash tools/gpu_r4l.sh
