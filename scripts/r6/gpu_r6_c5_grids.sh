#!/bin/bash
# Round 6: grid caps of C5's row kernels (experiments build exp_libs/base), C5 device ms per
# iteration, alternating; every row is independent, so the model is the same for every grid.
#   MML_WRMF_GRAM_GRID   the hot items' split Gram (default 512)
#   MML_WRMF_RESID_GRID  the users' first-pass residual (default 8,192)
#   MML_WRMF_XHH_GRID    the fp64 dense term (default 2,048)
#   MML_WRMF_RV_GRID     the kept-factor substitutions (default 4,096)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_steps.sh
export MML_LIB_PATH=exp_libs/base/libmml_hip.so
for rep in 1 2; do
  step r6cg_default_$rep 240 python -u scripts/c5_iter.py --iters 4
  for g in 2048 8192; do MML_WRMF_GRAM_GRID=$g step r6cg_gram${g}_$rep 240 python -u scripts/c5_iter.py --iters 4; done
  for g in 32768; do MML_WRMF_RESID_GRID=$g step r6cg_resid${g}_$rep 240 python -u scripts/c5_iter.py --iters 4; done
  for g in 8192; do MML_WRMF_XHH_GRID=$g step r6cg_xhh${g}_$rep 240 python -u scripts/c5_iter.py --iters 4; done
  for g in 16384; do MML_WRMF_RV_GRID=$g step r6cg_rv${g}_$rep 240 python -u scripts/c5_iter.py --iters 4; done
done
