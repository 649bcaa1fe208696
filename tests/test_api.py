"""Host-side API mirror (no GPU): discovery by type name (Extensions.cs:170-244), MultiCoreBPRMF's
configuration and visit order (MultiCoreBPRMF.cs:42-53, MultiCore.cs:79-92), the Gpus option."""
import numpy as np

import mymedialite_amd as M
from mymedialite_amd import _native as N


def test_create_by_name_like_the_reference():
    assert type(M.create_rating_predictor("BiasedMatrixFactorization")).__name__ == \
        "BiasedMatrixFactorization"
    # namespace prefix optional, case-insensitive (Assembly.GetType(name, false, true))
    assert type(M.create_rating_predictor("MyMediaLite.RatingPrediction.svdplusplus")).__name__ \
        == "SVDPlusPlus"
    assert type(M.create_item_recommender("multicorebprmf")).__name__ == "MultiCoreBPRMF"
    assert type(M.create_recommender("MyMediaLite.ItemRecommendation.WRMF")).__name__ == "WRMF"
    assert M.create_rating_predictor("NoSuchRecommender") is None
    assert "MultiCoreBPRMF" in M.list_recommenders("ItemRecommendation")
    assert "SocialMF" in M.list_recommenders("RatingPrediction")
    try:
        M.create_recommender("BPRMF")
        raise AssertionError("expected IOError")
    except IOError:
        pass


def test_multicore_bprmf_defaults_and_to_string():
    m = M.MultiCoreBPRMF()
    assert (m.UniformUserSampling, m.WithReplacement, m.MaxThreads) == (False, False, 100)
    m.configure("max_threads=8 num_factors=20")
    assert m.MaxThreads == 8 and m.NumFactors == 20
    assert str(m).startswith("MultiCoreBPRMF num_factors=20 ") and str(m).endswith("max_threads=8")
    assert m._sampler() == N.BPR_SAMPLER_UNIFORM_PAIR


def test_multicore_bprmf_order_is_partition_indices():
    """Train(): index_blocks = Feedback.PartitionIndices(MaxThreads): RandomIndex dealt round-robin
    into the blocks; the GPU visit order is the blocks concatenated."""
    u = np.arange(10, dtype=np.int32) % 4
    i = np.arange(10, dtype=np.int32) % 3
    m = M.MultiCoreBPRMF(MaxThreads=3)
    m.feedback = M.PosOnlyFeedback(u, i)
    M.Random.set_seed(9)
    order = m._order_before_init()
    M.Random.set_seed(9)
    idx = M.Random.get_instance().shuffle(np.arange(10, dtype=np.int32))
    np.testing.assert_array_equal(order, np.concatenate([idx[0::3], idx[1::3], idx[2::3]]))
    assert sorted(order.tolist()) == list(range(10))


def test_gpus_option_selects_a_multi_device_context():
    m = M.BiasedMatrixFactorization()
    assert N.device_arg(m) == 0
    m.configure("gpus=0,1,2,3")
    assert N.device_arg(m) == [0, 1, 2, 3]
    b = M.BPRMF(Device=2)
    assert N.device_arg(b) == 2


def test_auto_schedule_switches_to_hogwild_at_scale():
    """Schedule="auto": the reference's sequential loop below AUTO_EXACT_MAX training ratings,
    Hogwild from there on (the exact schedules run at ~2e7 ratings/s whatever the GPU, DESIGN.md
    section 3; noted once on stderr); MaxThreads > 1 keeps the reference's DSGD at any size."""
    from mymedialite_amd import rating_prediction as RP
    small = M.Ratings(np.zeros(10, np.int32), np.arange(10, dtype=np.int32),
                      np.ones(10, np.float32))
    n = RP.AUTO_EXACT_MAX
    big = M.Ratings(np.arange(n, dtype=np.int32) % 1000, np.arange(n, dtype=np.int32) % 997,
                    np.ones(n, np.float32))
    for cls in (M.BiasedMatrixFactorization, M.MatrixFactorization,
                M.SigmoidItemAsymmetricFactorModel):
        m = cls()
        assert m.schedule() == "ordered"
        m.ratings = small
        assert m.schedule() == "ordered"
        m.ratings = big
        assert m.schedule() == "hogwild", cls
        m.Schedule = "ordered"
        assert m.schedule() == "ordered"
    # an explicit MaxThreads > 1 asks for the reference's deterministic DSGD: kept at any size
    # (a silent switch to the racy schedule would surprise such a caller)
    m = M.BiasedMatrixFactorization(MaxThreads=8)
    m.ratings = small
    assert m.schedule() == "dsgd"
    m.ratings = big
    assert m.schedule() == "dsgd"
    m.NaiveParallelization = True
    assert m.schedule() == "hogwild"
