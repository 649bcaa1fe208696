"""Experiment: C1 hogwild RMSE vs oracle for the current MML_HOGWILD_MIN_CHUNK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from mymedialite_amd import BiasedMatrixFactorization, Random, Ratings  # noqa: E402
from mymedialite_amd.synthetic import ml100k_standin  # noqa: E402

tu, ti, tv, eu, ei, ev = ml100k_standin()
r = Ratings(tu, ti, tv)
st = O.bmf_train(tu, ti, tv, r.max_user_id + 1, r.max_item_id + 1, r.scale_min, r.scale_max,
                 seed=1, k=10, num_iter=30)
p = O.bmf_predict(eu, ei, st["U"], st["V"], st["bu"], st["bi"], st["global_bias"],
                  st["min_rating"], st["range_"])
ref = O.rating_eval(p, ev)[0]
for sched in ("ordered", "hogwild"):
    Random.set_seed(1)
    m = BiasedMatrixFactorization(NumFactors=10, Schedule=sched)
    m.ratings = r
    m.train()
    print(f"min_chunk={os.environ.get('MML_HOGWILD_MIN_CHUNK')} {sched}: "
          f"RMSE {m.evaluate(Ratings(eu, ei, ev))['RMSE']:.6f} oracle {ref:.6f}", flush=True)
