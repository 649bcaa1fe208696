#!/bin/bash
# WeightedBPRMF at 1.9M events: run-to-run spread of the item-side access modes
set -e
O=gpurun_out/r2h
mkdir -p $O
T="timeout -k 10"
for m in 0 0 4 4 6 3; do
  EXP_WEIGHTED=mid MML_BPR_XCD=$m $T 200 python -u scripts/exp_xcd.py weighted >> $O/weighted_mid.log 2>&1
done
