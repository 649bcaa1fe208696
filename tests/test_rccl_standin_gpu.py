"""The library's RCCL communicator branches at 2-8 ranks on one GPU (8 ranks,
the deployment width).

tests/rccl_ranks.py runs in a fresh subprocess with libmml_hip_standin.so (the library's own
objects linked against the checking stand-in tests/rccl_standin/standin.cpp instead of librccl):
every rank a host thread with its own context and a communicator from mml_ctx_comm_init, as under
torch.distributed.run.  BiasedMF and BPRMF user-shard averaging (ncclAllReduce ncclAvg), WRMF row
shards (grouped ncclBroadcast all-gather, ncclAllReduce ncclMax refinement decision) and the DSGD
ring (paired ncclSend / ncclRecv, ncclBroadcast) must equal the peer-copy transport bit for bit,
and the stand-in must see every rank issue the same collectives with equal counts and every send
pair with a recv of the same count (BiasedMatrixFactorization.cs:205-215, MultiCoreBPRMF.cs:49-63,
WRMF.cs:79-92).  This is readiness of the communicator code, not a scaling number.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_communicator_branches_equal_peer_transport():
    lib = os.path.join(ROOT, "tests", "rccl_standin", "libmml_hip_standin.so")
    assert os.path.exists(lib), "build the stand-in first (make -C tests/rccl_standin)"
    env = dict(os.environ, MML_LIB_PATH=lib, MML_STANDIN_TIMEOUT="20")
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_ranks.py")],
                       env=env, capture_output=True, text=True, timeout=840)
    print(p.stdout[-6000:])
    print(p.stderr[-3000:])
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    rep = res["report"]
    assert res["ok"] and not rep["errors"] and rep["unmatched_sends"] == 0, rep
    calls = {s["scenario"]: s["calls"] for s in res["scenarios"]}
    # every communicator branch ran: the averages, the all-gathers, the ring's transfers
    for name in ("bmf2", "bmf3", "bmf4", "bmf8", "bpr2", "bpr3", "bpr4", "bpr8"):
        assert calls[name]["allreduce"] > 0, calls[name]
    for name in ("wrmf2_k64", "wrmf2_k256", "wrmf3_k256", "wrmf4_k256", "wrmf8_k256"):
        assert calls[name]["broadcast"] > 0, calls[name]
    assert calls["wrmf2_k256"]["allreduce"] > 0  # the refinement's ncclMax decisions
    assert calls["wrmf8_k256"]["allreduce"] > 0
    for name in ("ring2", "ring3", "ring4", "ring8", "ring8_g16"):
        assert calls[name]["send"] > 0 and calls[name]["send"] == calls[name]["recv"], calls[name]
        assert calls[name]["broadcast"] > 0, calls[name]
