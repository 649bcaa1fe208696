"""Recommender base + the reference's option binding.

``configure("num_factors=10 reg_u=0.02")`` reproduces Extensions.Configure / SetProperty
(src/MyMediaLite/Extensions.cs:46-165, RecommenderParameters.cs:29-60): whitespace-split
``key=value`` pairs, names normalised (underscores removed, upper-cased) and matched as a PREFIX of
every public property in culture-sorted order; every match is set.  The quirk that ``reg_u=`` also
hits ``Regularization`` (whose setter overwrites RegI) is therefore kept.
"""
from __future__ import annotations

import re
import sys


def _normalize(name: str) -> str:
    return name.replace("_", "").upper()


def parse_parameters(arg_string: str) -> dict:
    """RecommenderParameters(string) (RecommenderParameters.cs:33-60)."""
    out = {}
    for tok in re.split(r"\s", arg_string):
        if len(tok) == 0:
            continue
        pair = tok.split("=")
        if len(pair) != 2:
            raise ValueError(f"Too many '=' in argument '{tok}'.")
        k, v = pair
        if k in out:
            raise ValueError(f"{k} is used twice as an argument.")
        if len(v) == 0:
            raise ValueError(f"{k} has an empty value.")
        out[k] = v
    return out


def _parse_bool(v: str) -> bool:
    s = v.strip().lower()
    if s == "true":
        return True
    if s == "false":
        return False
    raise ValueError(f"String '{v}' was not recognized as a valid Boolean.")


class Recommender:
    """Common surface of IRecommender / IIterativeModel (IRecommender.cs:33-75,
    IIterativeModel.cs:22-28).  Subclasses declare ``PROPERTIES = {Name: type}`` where type is
    'float', 'double', 'int', 'uint', 'bool', 'string' or a tuple of enum names."""

    PROPERTIES: dict = {}

    def configure(self, parameters: str, report_error=None):
        report_error = report_error or (lambda s: print(s, file=sys.stderr))
        try:
            for k, v in parse_parameters(parameters).items():
                self.set_property(k, v, report_error)
        except ValueError as e:
            report_error(f"{e}\n\n{self}\n")
        return self

    def set_property(self, key: str, val: str, report_error=None):
        report_error = report_error or (lambda s: print(s, file=sys.stderr))
        names = sorted(self.PROPERTIES, key=lambda s: (s.lower(), s))
        nkey = _normalize(key)
        found = False
        for name in names:
            if not _normalize(name).startswith(nkey):
                continue
            found = True
            t = self.PROPERTIES[name]
            if isinstance(t, tuple):
                if val not in t:
                    raise ValueError(f"Requested value '{val}' was not found.")
                setattr(self, name, val)
            elif t in ("float", "double"):
                setattr(self, name, float(val))
            elif t == "int":
                setattr(self, name, 2147483647 if val == "inf" else int(val))
            elif t == "uint":
                setattr(self, name, 4294967295 if val == "inf" else int(val))
            elif t == "bool":
                setattr(self, name, _parse_bool(val))
            elif t == "string":
                setattr(self, name, val)
            else:
                report_error(f"Parameter '{key}' has unknown type '{t}'")
        if not found:
            report_error(f"Recommender {type(self).__name__} does not have a parameter named "
                         f"'{nkey}'.\n{self}")


# ------------------------------------------------------------------ discovery by type name
def _registry(namespace: str) -> dict:
    """TYPE_NAME (lower-cased) -> class for the GPU recommenders of one namespace."""
    from . import item_recommendation, rating_prediction
    mod = rating_prediction if namespace == "RatingPrediction" else item_recommendation
    out = {}
    for obj in vars(mod).values():
        # the class's own TYPE_NAME (a subclass inherits its parent's until it declares one)
        name = vars(obj).get("TYPE_NAME") if isinstance(obj, type) else None
        if name and name.startswith(f"MyMediaLite.{namespace}."):
            out[name.lower()] = obj
    return out


def create_rating_predictor(typename: str):
    """Extensions.CreateRatingPredictor(string) (Extensions.cs:170-182): the namespace prefix is
    optional and the name matches case-insensitively (Assembly.GetType(name, false, true)); None
    when no such GPU recommender exists."""
    if not typename.startswith("MyMediaLite.RatingPrediction."):
        typename = "MyMediaLite.RatingPrediction." + typename
    cls = _registry("RatingPrediction").get(typename.lower())
    return cls() if cls is not None else None


def create_item_recommender(typename: str):
    """Extensions.CreateItemRecommender(string) (Extensions.cs:216-228)."""
    if not typename.startswith("MyMediaLite.ItemRecommendation"):
        typename = "MyMediaLite.ItemRecommendation." + typename
    cls = _registry("ItemRecommendation").get(typename.lower())
    return cls() if cls is not None else None


def create_recommender(typename: str):
    """Extensions.CreateRecommender(string) (Extensions.cs:187-195)."""
    if typename.startswith("MyMediaLite.RatingPrediction."):
        return create_rating_predictor(typename)
    if typename.startswith("MyMediaLite.ItemRecommendation."):
        return create_item_recommender(typename)
    raise IOError(f"Unknown recommender namespace in type name '{typename}'")


def list_recommenders(namespace: str) -> list:
    """The type names create_* finds (cf. Extensions.ListRecommenders, Extensions.cs:292-312)."""
    return sorted(c.TYPE_NAME.split(".")[-1] for c in _registry(namespace).values())
