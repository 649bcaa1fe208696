#!/bin/bash
# round 4, second GPU batch: the per-rank DSGD ring, the staleness-model Hogwild bands, the
# full-size checks, then the default bench line (C4 headline + c2 / c3 / c5 keys)
source scripts/gpu_steps.sh
step r4b_multi 600 $PYT --timeout 300 tests/test_multi_gpu.py
step r4b_bands 900 $PYT --timeout 600 tests/test_edge_cases_gpu.py tests/test_bmf_gpu.py -k "hogwild or c2_shape"
step r4b_full 600 $PYT --timeout 500 tests/test_full_scale_gpu.py
step r4b_bench 900 python -u bench.py
