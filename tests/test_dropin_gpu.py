"""Drop-in recommenders / constraint filter on the device (HIP ItemIndex through the C-ABI)
against the reference's golden outputs — the same checks test_dropin.py runs on CPU."""
import numpy as np
import pytest

import _dropin_checks as D

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    return D.build_world()


@pytest.fixture
def hy(world, monkeypatch):
    D.pin_year(monkeypatch)
    h = D.make_hybrid(world, None)   # None -> the HIP ItemIndex
    yield h
    if h.engine.index is not None:
        h.engine.index.close()


def test_device_index_is_native(hy):
    from brickrec.engine import ItemIndex
    hy.engine.ensure_index()
    assert isinstance(hy.engine.index, ItemIndex)


def test_get_similar_sets(hy, golden):
    D.check_similar_sets(hy, golden)


def test_collaborative_filtering(hy, golden):
    D.check_cf(hy, golden)


def test_constraint_filter(hy, golden):
    D.check_constraint_masks(hy, golden)


def test_hybrid(hy, golden):
    D.check_hybrid(hy, golden)


def test_recommend_batch_matches_per_request(hy):
    """The one-call device hybrid (blend on the device) == the per-request path."""
    cb, cf = hy.content_recommender, hy.collaborative_recommender
    cb.prepare_features()
    cf.train_svd_model()
    users = [1, 2, 7, 19, 42, 50]
    liked = [cb.set_lookup[i] for i in (0, 13, 77, 150, 400, 999)]
    names, scores = hy.recommend_batch(liked, users, top_k=10)
    for b in range(len(users)):
        recs, _ = hy.get_recommendations(user_id=users[b], liked_set=liked[b], top_k=10)
        assert [r.set_num for r in recs] == names[b]
        np.testing.assert_allclose([r.score for r in recs], scores[b], atol=1e-5, rtol=0)
