#!/bin/bash
# A/B: value-length reads issued inside the previous block combine (full) vs before (prehook).
CONFIGS="4k zipf" VARIANTS="prehook full" exec bash tools/gpu_r4l.sh
