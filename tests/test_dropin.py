"""Drop-in recommenders / constraint filter over the reference's synthetic catalogue, on
CPU with the oracle-backed index stand-in (the device runs are in test_dropin_gpu.py)."""
import pytest

import _dropin_checks as D
from _oracle_index import OracleIndex


@pytest.fixture(scope="module")
def world():
    return D.build_world()


@pytest.fixture
def hy(world, monkeypatch):
    D.pin_year(monkeypatch)
    return D.make_hybrid(world, OracleIndex)


def test_prepare_features_reproduces_reference_matrix(hy, golden):
    D.check_features(hy, golden)


def test_get_similar_sets(hy, golden):
    D.check_similar_sets(hy, golden)


def test_collaborative_filtering(hy, golden):
    D.check_cf(hy, golden)


def test_constraint_filter(hy, golden):
    D.check_constraint_masks(hy, golden)


def test_hybrid(hy, golden):
    D.check_hybrid(hy, golden)


def test_combine_and_weights(hy):
    from brickrec.recommenders import RecommendationResult as RR
    hy.engine.ensure_catalog()
    rows = hy.engine.catalog.set_nums
    c = [RR(rows[0], "a", 0.9, ["x"], "t", 2000, 10), RR(rows[1], "b", 0.5, [], "t", 2000, 10)]
    f = [RR(rows[1], "b", 1.0, ["y"], "t", 2000, 10), RR(rows[2], "c", 0.2, [], "t", 2000, 10)]
    out = hy._combine_recommendations(c, f, 3)
    assert [r.set_num for r in out] == [rows[1], rows[0], rows[2]]
    assert out[0].reasons == ["Community: y"] and out[1].reasons == ["Content: x"]
    hy.set_weights(1, 3)
    assert (hy.content_weight, hy.collaborative_weight) == (0.25, 0.75)


def test_empty_constraint_result(hy):
    from brickrec.constraints import create_constraint_set_values
    recs, res = hy.get_recommendations(user_id=1, liked_set=None, top_k=5,
                                       constraints=create_constraint_set_values(required_themes=["no-such"]))
    assert recs == [] and res.valid_set_nums == []
