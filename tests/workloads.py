"""Processor configs of the BASELINE.json workloads, shared by
the parity tests and bench.py.  Test/bench infrastructure.

The generator (odigos_amd/csrc/gen_batch.cpp) writes raw service numbers
0..63 into res_svc / res_svc_str; the configs below name "svc-NN" services
in an order that makes the engine's interned id of "svc-NN" equal NN
(ids are assigned in first-appearance order over global, service and
endpoint rules), so generated batches need no remapping.  Raw numbers beyond
the interned range name no rule service.
"""
from __future__ import annotations

# generator routes: /api/v{1,2}/<word>[/{id}][/<word>] (gen_batch.cpp)
_LAT_ROUTES = ["/api/v1", "/api/v2", "/api", "/api/v1/", "/health", "/api/v2/", "/a", "/api/v1",
               "/api/v2", "/api", "/api/v1", "/x", "/api/v2", "/api/v1", "/api", "/api/v2"]


def c3_sampling_config() -> dict:
    """C3: global error rule (fallback 10), 4 service_name rules, 16 http_latency
    rules (thresholds 50-2000 ms, fallback 0-25) over 12 services."""
    service_rules = [
        {"name": f"svc-{k:02d}", "type": "service_name",
         "rule_details": {"service_name": f"svc-{k:02d}", "sampling_ratio": [100.0, 50.0, 0.0, 75.0][k],
                          "fallback_sampling_ratio": [5.0, 10.0, 0.0, 20.0][k]}}
        for k in range(4)]
    # latency services: ids 2..13 (2 and 3 shared with service rules), some with two rules
    lat_svcs = [2, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 4, 5, 2, 6, 13]
    endpoint_rules = []
    for j, s in enumerate(lat_svcs):
        endpoint_rules.append({
            "name": f"lat-{j}", "type": "http_latency",
            "rule_details": {"http_route": _LAT_ROUTES[j], "service_name": f"svc-{s:02d}",
                             "threshold": [50, 80, 100, 150, 200, 300, 500, 750, 1000, 1500, 2000, 60, 90, 120, 400, 70][j],
                             "fallback_sampling_ratio": [0, 5, 10, 25, 0, 15, 20, 0, 5, 25, 10, 0, 0, 5, 25, 12.5][j]}})
    return {
        "global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}],
        "service_rules": service_rules,
        "endpoint_rules": endpoint_rules,
    }


# ---- sampling configs beyond one GPU rule table (tests/test_sampling_chunks.py) ----
_WIDE_ROUTES = ["/api/v1", "/api/v2", "/api", "/api/v1/", "/health", "/api/v2/", "/a", "/x", "/api/v1/users",
           "/api/v2/orders", "/", "/api/v1/items/"]
_WIDE_THRESH = [50, 80, 100, 150, 200, 300, 500, 750, 1000, 1500, 2000, 60, 90, 120, 400, 70]


def _wide_lat(j, svc):
    return {"name": f"lat-{j}", "type": "http_latency",
            "rule_details": {"http_route": _WIDE_ROUTES[(j * 5) % len(_WIDE_ROUTES)], "service_name": f"svc-{svc:02d}",
                             "threshold": _WIDE_THRESH[j % len(_WIDE_THRESH)],
                             "fallback_sampling_ratio": [0, 5, 10, 25, 0, 15, 20, 12.5, 33.3, 7][j % 10]}}


def _wide_svc(k, name_id):
    return {"name": f"s{k}", "type": "service_name",
            "rule_details": {"service_name": f"svc-{name_id:02d}", "sampling_ratio": float((k * 37) % 101),
                             "fallback_sampling_ratio": float(k % 7)}}


def wide_latency_config():
    """150 http_latency rules (3 chunks) at the endpoint level over services
    0..63 (first appearance in id order), after the C3 error and service rules."""
    svc = [_wide_svc(k, k) for k in range(4)]
    return {"global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}],
            "service_rules": svc,
            "endpoint_rules": [_wide_lat(j, j % 64) for j in range(150)]}


def wide_latency2_config():
    """100 http_latency rules (2 chunks: 64 + 36) over services 0..63."""
    cfg = wide_latency_config()
    cfg["endpoint_rules"] = cfg["endpoint_rules"][:100]
    return cfg


def wide_latency_split_config():
    """2 chunks whose latency services differ: 70 global-level rules over
    services 0..9 (the first chunk takes 64), then 12 endpoint-level rules over
    services 14..25, which have rules in the second chunk only."""
    return {"global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}]
            + [_wide_lat(j, j % 10) for j in range(70)],
            "service_rules": [_wide_svc(k, 10 + k) for k in range(4)],
            "endpoint_rules": [_wide_lat(400 + j, 14 + j) for j in range(12)]}


def wide_mixed_config():
    """Chunk boundaries inside and across levels: 80 latency rules in the
    global level (services 0..39), 100 service_name rules over services
    40..139 (only ids < 64 occur in the generator's batches), 70 latency rules
    in the endpoint level."""
    return {"global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}]
            + [_wide_lat(j, j % 40) for j in range(80)],
            "service_rules": [_wide_svc(k, 40 + k) for k in range(100)],
            "endpoint_rules": [_wide_lat(200 + j, j % 64) for j in range(70)]}


def many_services_config(n_services=1200):
    """More distinct service names than dense per-service tables fit beside
    a rule table in LDS (12 B per service): 64 global-level http_latency
    rules over services 0..63, one service_name rule per service 0..n-1 (the
    generator's batches hold ids < 64 only), 24 endpoint-level http_latency
    rules over services 10..33.  Each rule chunk then indexes its own
    services (chunk-local ids)."""
    return {"global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}]
            + [_wide_lat(j, j) for j in range(64)],
            "service_rules": [_wide_svc(k, k) for k in range(n_services)],
            "endpoint_rules": [_wide_lat(300 + j, 10 + j) for j in range(24)]}


def wide_attr_config():
    """span_attribute rules split over two rule chunks (their attr_match bits
    0..13 in the first, 14..39 in the second): 40 latency rules (services
    0..39), 50 service_name rules (services 40..89), 40 json span_attribute
    rules (bits from the attr_match column), 30 latency rules."""
    attr = [{"name": f"a{j}", "type": "span_attribute",
             "rule_details": {"service_name": f"svc-{j % 40:02d}", "attribute_key": "body", "condition_type": "json",
                              "operation": "is_valid_json", "sampling_ratio": float((j * 13) % 101),
                              "fallback_sampling_ratio": float(j % 5)}} for j in range(40)]
    return {"global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}]
            + [_wide_lat(j, j) for j in range(40)],
            "service_rules": [_wide_svc(k, 40 + k) for k in range(50)] + attr,
            "endpoint_rules": [_wide_lat(300 + j, j % 64) for j in range(30)]}


def wide_attr100_config():
    """More than 64 span_attribute rules (attr_match in two 64-bit words): 40
    service_name rules (services 0..39), then 100 json span_attribute rules
    over services 0..63 in the service level (their bits 0..99: chunk cuts at
    24 and 88, the middle chunk's bits straddle the two words), 20 latency
    rules at the endpoint level."""
    attr = [{"name": f"a{j}", "type": "span_attribute",
             "rule_details": {"service_name": f"svc-{(40 + j) % 64:02d}", "attribute_key": "body",
                              "condition_type": "json", "operation": "is_valid_json",
                              "sampling_ratio": float((j * 29) % 101), "fallback_sampling_ratio": float(j % 9)}}
            for j in range(100)]
    return {"global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}],
            "service_rules": [_wide_svc(k, k) for k in range(40)] + attr,
            "endpoint_rules": [_wide_lat(500 + j, j % 64) for j in range(20)]}


def long_routes_config():
    """Tables beyond the 12 KiB LDS budget through route bytes alone: 40
    latency rules whose http_route is ~400 bytes (the first 7 bytes match)."""
    rules = []
    for j in range(40):
        r = _wide_lat(j, j % 16)
        r["rule_details"]["http_route"] = "/api/v1" + "/" + "z" * (380 + j)
        rules.append(r)
    rules += [_wide_lat(100 + j, j % 16) for j in range(8)]
    return {"global_rules": [{"name": "errors", "type": "error", "rule_details": {"fallback_sampling_ratio": 10}}],
            "service_rules": [], "endpoint_rules": rules}


def check_interning(cfg: dict) -> None:
    from tests.oracle_lib import intern_services
    for name, k in intern_services(cfg).items():
        assert name == f"svc-{k:02d}", (name, k)
