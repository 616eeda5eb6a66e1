#!/bin/bash
# leader inbox prefetch: off (base) / 1 / 2 records per sender, C3 steady
# state, alternated; then the parity suite on lpf1
tools/exp_variants.sh r03_lpf base lpf1 lpf2 base2 lpf1 lpf2 || exit 1
DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/lpf1.so tools/gpu_step.sh 600 gpurun_out/r03_lpf/parity.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_elections.py tests/test_gpu_fullsize.py -k "not c5" -m gpu || exit 1
