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


def check_interning(cfg: dict) -> None:
    from tests.oracle_lib import intern_services
    for name, k in intern_services(cfg).items():
        assert name == f"svc-{k:02d}", (name, k)
