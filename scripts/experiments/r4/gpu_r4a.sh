#!/bin/bash
# round 4, first GPU batch: N > 1 shards of BPR / WRMF on one GPU, the grouped BPR sampler, the
# Hogwild order-noise bands, and the full-size C3 / C5 quality checks
source scripts/gpu_steps.sh
step r4a_multi 600 $PYT --timeout 300 tests/test_multi_gpu.py
step r4a_bprgrp 300 $PYT --timeout 240 tests/test_bpr_grouped_gpu.py tests/test_bpr_c3_replica_gpu.py
step r4a_bands 600 $PYT --timeout 400 tests/test_edge_cases_gpu.py -k hogwild tests/test_bmf_gpu.py -k "hogwild or c2_shape"
step r4a_full 900 $PYT --timeout 800 tests/test_full_scale_gpu.py
