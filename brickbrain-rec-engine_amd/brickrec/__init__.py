"""brickrec — MI355X-native scoring engine for the similar-sets / hybrid-recommendation hot
path of davidry777/Brickbrain-Rec-Engine.

Layers: ``_lib`` (ctypes over libbrickrec.so, the C-ABI in include/brickrec.h),
``engine.ItemIndex`` (device-resident index + batched search), and the drop-ins that keep
the reference's call signatures: ``recommenders`` (recommendation_system.py),
``constraints`` (hard_constraint_filter.py), ``semantic`` (NLPRecommender.semantic_search),
``api`` (FastAPI routes) and ``distributed`` (row-sharded index over RCCL).
"""
from ._lib import BrickrecError  # noqa: F401
from .engine import ItemIndex, Predicate, bits_from_bool, bool_from_bits  # noqa: F401

__version__ = "0.1.0"
