"""mymedialite_amd -- MI355X-native training path for MyMediaLite's matrix-factorization recommenders.

The per-rating / per-sample loops run in libmml_hip.so (hand-written HIP for gfx950, C ABI in
include/mml.h); this package is the host-side mirror of the reference's recommender API.
"""
from .data import (DeviceRatingFile, IdentityMapping, Mapping, PosOnlyFeedback, Ratings, read_items,
                   read_ratings)
from .random import Random, SystemRandom
from .recommender import (create_item_recommender, create_rating_predictor, create_recommender,
                          list_recommenders)
from .item_recommendation import (BPRMF, WRMF, MultiCoreBPRMF, SoftMarginRankingMF,
                                  WeightedBPRMF)
from .rating_prediction import (BiasedMatrixFactorization, MatrixFactorization,
                                SigmoidItemAsymmetricFactorModel,
                                SigmoidUserAsymmetricFactorModel, SocialMF,
                                SigmoidCombinedAsymmetricFactorModel, SigmoidSVDPlusPlus,
                                SVDPlusPlus)

__all__ = ["BiasedMatrixFactorization", "MatrixFactorization", "SocialMF",
           "SigmoidItemAsymmetricFactorModel", "SigmoidUserAsymmetricFactorModel",
           "SigmoidCombinedAsymmetricFactorModel", "SVDPlusPlus", "SigmoidSVDPlusPlus", "BPRMF", "WRMF",
           "SoftMarginRankingMF", "WeightedBPRMF", "MultiCoreBPRMF", "Ratings",
           "PosOnlyFeedback", "Mapping", "IdentityMapping", "read_ratings", "read_items", "Random",
           "DeviceRatingFile",
           "SystemRandom", "create_rating_predictor", "create_item_recommender",
           "create_recommender", "list_recommenders"]
