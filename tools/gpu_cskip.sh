#!/bin/bash
# A/B: CRC lanes before the payload switched off (cskip) vs shipped.
CONFIGS="4k zipf" VARIANTS="full cskip" exec bash tools/gpu_r4l.sh
