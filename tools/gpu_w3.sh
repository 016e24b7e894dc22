#!/bin/bash
# A/B of the per-window copy_fast3 selection (zipf, 4k) after the parity tests.
CONFIGS="zipf 4k" VARIANTS="prew3 full" exec bash tools/gpu_r4l.sh
