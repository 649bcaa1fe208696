#!/bin/bash
# C3 replica under the default BPR mode: concurrency (MML_HOGWILD_MIN_CHUNK) vs dAUC, true k=128 oracle
set -e
O=gpurun_out/r2i
mkdir -p $O
T="timeout -k 10"
for mc in 16384 65536 262144; do
  MML_HOGWILD_MIN_CHUNK=$mc $T 300 python -u scripts/exp_xcd.py c3rep > $O/c3rep_mc$mc.log 2>&1
done
cp scripts/exp_xcd_oracle.json $O/
