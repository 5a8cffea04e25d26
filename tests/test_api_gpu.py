"""The FastAPI drop-in routes (brickrec.api: /recommendations, /recommendations/constrained,
/sets/similar/semantic, /recommendations/batch — recommendation_api.py:432-498, 501-598,
1501-1585) served from the HIP ItemIndex (libbrickrec on the device): every route check of
test_api.py, run against the device index instead of the CPU stand-in, plus the route ->
index wiring and the error mapping (HTTP 500 with the error text, recommendation_api.py:496-498)."""
import pytest

import test_api as T
from test_api import (test_batch_route, test_collaborative_route, test_constrained_route,  # noqa: F401
                      test_content_route_matches_reference, test_embedding_route_is_opt_in, test_errors,
                      test_health, test_hybrid_route_returns_list, test_similar_semantic_sql_pinned,
                      test_similar_semantic_sql_route)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def client():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    yield from T.make_client(None)   # None -> the HIP ItemIndex


def test_routes_serve_from_device_index(client):
    from brickrec.engine import ItemIndex
    rec = client.app.state.recommender
    assert client.post("/recommendations", json={"set_num": rec.content_recommender.set_lookup[3], "top_k": 5,
                                                 "recommendation_type": "content"}).status_code == 200
    assert isinstance(rec.engine.index, ItemIndex)


def test_device_error_maps_to_500(client, monkeypatch):
    """A failure inside the device index surfaces as HTTP 500 with the error text, as the
    reference wraps every exception (recommendation_api.py:496-498)."""
    from brickrec import _lib
    from brickrec.engine import ItemIndex
    rec = client.app.state.recommender
    rec.engine.ensure_index()

    def boom(self, *a, **k):
        raise _lib.BrickrecError("bb_search: injected device failure")
    monkeypatch.setattr(ItemIndex, "search", boom)
    r = client.post("/recommendations", json={"set_num": rec.content_recommender.set_lookup[3], "top_k": 5,
                                              "recommendation_type": "content"})
    assert r.status_code == 500
    assert "injected device failure" in r.json()["detail"]
