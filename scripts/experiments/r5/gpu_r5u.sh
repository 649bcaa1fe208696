#!/bin/bash
# Round 5, batch U: stream priorities for the item half's pipeline (experiments build): the side
# stream at the least / greatest priority, the context's stream at the greatest; 4 and 8 ranges.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
source scripts/gpu_steps.sh
for v in "4 none none" "4 least none" "4 greatest none" "4 none greatest" "8 none greatest" "1 none none" "4 none none"; do
    set -- $v
    (
        export MML_LIB_PATH=variants/exp/libmml_hip.so MML_WRMF_PIPE=$1
        if [ "$2" != none ]; then export MML_WRMF_PIPE_PRIO=$2; fi
        if [ "$3" != none ]; then export MML_CTX_STREAM_PRIO=$3; fi
        step r5u_c5_p$1_s$2_c$3_$RANDOM 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline
    ) || exit $?
done
