"""HTTP API contract: /chat, /history (reference src/app.py) and the pool worker /, /health,
/query (reference src/devices/*_api.py), on echo pools."""
import pytest

from distributed_llm_amd.config import LARGE, SMALL
from distributed_llm_amd.orchestrator import Router
from distributed_llm_amd.pools.base import EchoPool, FaultInjectingPool
from distributed_llm_amd.pools.worker import create_worker_app
from distributed_llm_amd.server.app import BASE_CONFIG, HISTORY_LIMIT, create_app

# the reference reply's keys (src/app.py:83-91 success, :98-106 error; App.tsx:115-123 reads them)
REF_KEYS = {"reply", "device", "reasoning", "method", "confidence", "cache_hit", "tokens"}
CHAT_KEYS = REF_KEYS
REF_APP = "/root/reference/src/app.py"


def _reference_reply_keys():
    """Keys of every jsonify({...}) reply in the reference's /chat with a "reply" key (None when
    the reference tree is not present, e.g. on a GPU box)."""
    import ast
    import os
    if not os.path.exists(REF_APP):
        return None
    out = []
    for node in ast.walk(ast.parse(open(REF_APP).read())):
        if isinstance(node, ast.Call) and getattr(node.func, "id", "") == "jsonify" and node.args \
                and isinstance(node.args[0], ast.Dict):
            keys = {k.value for k in node.args[0].keys if isinstance(k, ast.Constant)}
            if "reply" in keys:
                out.append(keys)
    return out


def test_reply_keys_match_reference_source():
    got = _reference_reply_keys()
    if got is None:
        pytest.skip("reference tree not present")
    assert got == [REF_KEYS, REF_KEYS]


@pytest.fixture()
def client():
    app = create_app(config=dict(BASE_CONFIG), pools={SMALL: EchoPool(SMALL, 6), LARGE: EchoPool(LARGE, 20)})
    return app.test_client()


def test_chat_contract(client):
    r = client.post("/chat", json={"message": "Thank you!", "strategy": "heuristic", "session_id": "s1"})
    assert r.status_code == 200
    d = r.get_json()
    # tokens: the reference counts the returned text (src/router.py:286, TokenCounter)
    from distributed_llm_amd.router.tokens import TokenCounter
    want = TokenCounter().count_tokens({"role": "assistant", "content": d["reply"]})
    assert set(d) == CHAT_KEYS and d["device"] == SMALL and d["tokens"] == want
    # the bundled UI opts in to an eighth key with the turn's timing; /metrics keeps the last one
    d2 = client.post("/chat", json={"message": "Thank you!", "session_id": "s2", "include_timing": True}).get_json()
    assert set(d2) == CHAT_KEYS | {"timing"}
    assert set(d2["timing"]) == {"latency_ms", "routing_ms", "ttft_ms", "failover"} and d2["timing"]["failover"] is False
    assert client.get("/metrics").get_json()["last_timing"]["session_id"] == "s2"
    assert r.headers["Access-Control-Allow-Origin"] == "*"
    h = client.get("/history?session_id=s1").get_json()
    assert [m["role"] for m in h] == ["user", "assistant"] and h[1]["content"] == d["reply"]


def test_blank_message_400(client):
    r = client.post("/chat", json={"message": "   "})
    assert r.status_code == 400 and r.get_json() == {"error": "No message provided"}


def test_token_counting_alias_and_bad_strategy(client):
    assert client.post("/chat", json={"message": "hi", "strategy": "token-counting"}).status_code == 200
    r = client.post("/chat", json={"message": "hi", "strategy": "nonsense"})
    assert r.status_code == 500 and r.get_json()["error"].startswith("Failed to switch strategy")


def test_history_cap_and_clear(client):
    for i in range(8):
        client.post("/chat", json={"message": f"question {i}?", "strategy": "token", "session_id": "cap"})
    h = client.get("/history?session_id=cap").get_json()
    assert len(h) == HISTORY_LIMIT
    assert client.delete("/history?session_id=cap").get_json() == {"cleared": "cap"}
    assert client.get("/history?session_id=cap").get_json() == []


def test_error_rolls_back_history():
    class Boom(EchoPool):
        def process(self, h):
            raise RuntimeError("dead")

    router = Router("token", config={"cache_enabled": False, "enable_failover": False},
                    pools={SMALL: EchoPool(SMALL), LARGE: EchoPool(LARGE)})

    def broken(history):
        raise RuntimeError("kaboom")
    router.route_query = broken
    c = create_app(router=router).test_client()
    r = c.post("/chat", json={"message": "hi", "strategy": "token", "session_id": "e"})
    assert r.status_code == 500
    d = r.get_json()
    assert set(d) == CHAT_KEYS and d["device"] == "error" and d["reasoning"] == "kaboom"
    assert c.get("/history?session_id=e").get_json() == []


def test_metrics(client):
    client.post("/chat", json={"message": "hello"})
    m = client.get("/metrics").get_json()
    assert m["strategy"] == "hybrid" and "cache" in m and set(m["pools"]) == {SMALL, LARGE}


def test_worker_endpoints():
    c = create_worker_app(EchoPool(SMALL, 4)).test_client()
    assert c.get("/").data == b"Test again: Server is running!\n"
    assert c.get("/health").get_json() == {"ok": True}
    r = c.post("/query", json={"query": [{"role": "user", "content": "hello"}]})
    assert r.status_code == 200 and "response" in r.get_json()
    assert c.post("/query", json={}).status_code == 400
    assert c.post("/query", json={"query": 5}).status_code == 400
    rb = c.post("/query", json={"queries": [[{"role": "user", "content": "a"}], "b"]})
    assert len(rb.get_json()["responses"]) == 2
    err = create_worker_app(FaultInjectingPool(EchoPool(SMALL), mode="error")).test_client()
    r = err.post("/query", json={"query": "x"})
    assert r.status_code == 500 and "error" in r.get_json()


def test_browser_client_served(client):
    r = client.get("/")
    assert r.status_code == 200
    body = r.get_data(as_text=True)
    # same request contract as the reference React client (App.tsx:101-109)
    assert "/chat" in body and "session_id" in body and "token-counting" in body
    # routing-metadata panel of ChatMessage.tsx:56-92: device badge, cache badge, method, confidence,
    # tokens, reasoning (+ timing line and dark mode)
    for needle in ("cache_hit", "r.method", "r.confidence", "r.tokens", "r.reasoning", "latency_ms", "ttft_ms",
                   "dllm_dark"):
        assert needle in body, needle
