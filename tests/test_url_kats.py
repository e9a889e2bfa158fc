"""odigosurltemplate known-answer tests, transcribed from the reference's
processor_test.go / factory_test.go (tests/golden/url_kats.json).

Each case is run twice:
* CPU: host columnariser -> oracle (oracle/url.c) -> host apply, which pins
  the oracle and the host layer against the reference's expected outputs;
* GPU (@gpu): the full ConsumeTraces path through the HIP engine.
"""
import json
from pathlib import Path

import pytest

from odigos_amd import host
from tests.oracle_lib import UrlOracle

GOLD = json.loads((Path(__file__).parent / "golden" / "url_kats.json").read_text())


def _case_traces(service, span_name, kind, attrs):
    res = {}
    if service:
        # generateTraceData (processor_test.go:13-26)
        res = {"service.name": service, "k8s.namespace.name": "default", "k8s.deployment.name": service}
    return host.traces(host.resource_spans(res, [host.span(name=span_name, kind=kind, attributes=attrs)]))


def _all_cases():
    out = []
    for g in GOLD["groups"]:
        for c in g["cases"]:
            out.append(dict(cfg=g["config"], traces=_case_traces(c["span"], c["span"], c["kind"], c["attrs"]),
                            name=c["expect_name"], key=c["expect_key"], value=c["expect_value"],
                            id=f'{g["test"]}:{c["line"]}:{c["name"]}'))
    for c in GOLD["rule_cases"]["cases"]:
        cfg = {}
        if "rules" in c:
            cfg["templatization_rules"] = c["rules"]
        if "custom_ids" in c:
            cfg["custom_ids"] = c["custom_ids"]
        attrs = {"http.request.method": "GET", "url.path": c["path"]}
        out.append(dict(cfg=cfg, traces=_case_traces("test-service-name", "GET", 2, attrs)
                        if False else host.traces(host.resource_spans(
                            {"service.name": "test-service-name", "k8s.namespace.name": "default",
                             "k8s.deployment.name": "test-service-name"},
                            [host.span(name="GET", kind=2, attributes=attrs)])),
                        name=c["expect_name"], key="http.route", value=c["expect_route"],
                        id=f'rules:{c["line"]}:{c["name"]}'))
    ie = GOLD["include_exclude"]
    for c in ie["cases"]:
        cfg = {}
        if "include" in c:
            cfg["include"] = {"k8s_workloads": c["include"]}
        if "exclude" in c:
            cfg["exclude"] = {"k8s_workloads": c["exclude"]}
        attrs = {"http.request.method": "GET", "url.path": "/user/1234"}
        tr = host.traces(host.resource_spans(
            {"service.name": "test-service-name", "k8s.namespace.name": "default",
             "k8s.deployment.name": "test-service-name"},
            [host.span(name="GET", kind=2, attributes=attrs)]))
        if c["templated"]:
            out.append(dict(cfg=cfg, traces=tr, name="GET /user/{id}", key="http.route", value="/user/{id}",
                            id=f'include_exclude:{c["line"]}:{c["name"]}'))
        else:
            out.append(dict(cfg=cfg, traces=tr, name="GET", key="http.route", value=None,
                            id=f'include_exclude:{c["line"]}:{c["name"]}'))
    return out


CASES = _all_cases()


def _check(out_traces, case):
    sp = out_traces["resourceSpans"][0]["scopeSpans"][0]["spans"][0]
    assert sp["name"] == case["name"], case["id"]
    v = host.find_attr(sp, case["key"]) if case["key"] else None
    if case["value"] is None:
        assert v is None, f'{case["id"]}: unexpected {case["key"]}={v}'
    else:
        assert v is not None, f'{case["id"]}: missing {case["key"]}'
        assert host.as_string(v) == case["value"], case["id"]


def test_fixture_count():
    # 24 + 4 + 5 + 3 + 9 + 6 default cases, 20 rule/custom-id cases, 7 include/exclude
    assert len(CASES) == 78


@pytest.mark.parametrize("case", CASES, ids=[c["id"] for c in CASES])
def test_kat_oracle(case):
    proc = host.Processor("odigosurltemplate", case["cfg"])
    hb = proc.columnarize(case["traces"])
    orc = UrlOracle(case["cfg"])
    assert orc.process(hb.cols, hb.outs) == 0
    _check(hb.apply(), case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["id"] for c in CASES])
def test_kat_gpu(case):
    proc = host.Processor("odigosurltemplate", case["cfg"])
    _check(proc.consume(case["traces"]), case)


@pytest.mark.parametrize("rule", [c["rule"] for c in GOLD["invalid_rules"]["cases"]])
def test_invalid_rules_rejected(rule):
    # TestInvalidRules (factory_test.go:33-58): CreateTraces returns an error
    with pytest.raises(ValueError):
        host.Processor("odigosurltemplate", {"templatization_rules": [rule]})
    with pytest.raises(ValueError):
        UrlOracle({"templatization_rules": [rule]})


def test_default_config_and_validation():
    # TestCreateDefaultConfig / config.go:103-157
    host.Processor("odigosurltemplate", {})
    bad = [
        {"exclude": {"k8s_workloads": [{"namespace": "", "kind": "Deployment", "name": "x"}]}},
        {"include": {"k8s_workloads": [{"namespace": "ns", "kind": "Pod", "name": "x"}]}},
        {"include": {"k8s_workloads": [{"namespace": "ns", "kind": "Deployment", "name": ""}]}},
        {"custom_ids": [{"regexp": "(unclosed"}]},
    ]
    for cfg in bad:
        with pytest.raises(ValueError):
            host.Processor("odigosurltemplate", cfg)


@pytest.mark.gpu
def test_gpu_long_segments_and_wide_groups():
    # segments longer than a 64-bit window and groups whose byte range outgrows
    # the plan kernel's stage are planned by url_plan_slow_kernel and emitted
    # by url_emit_slow_kernel; the result must equal the oracle's
    import random
    rng = random.Random(0x0D16_0A11)
    spans = []
    for k in range(300):
        shape = rng.randrange(5)
        if shape == 0:
            path = "/" + "".join(rng.choice("abcxyz") for _ in range(rng.randrange(65, 200)))
        elif shape == 1:
            path = "/v1/" + "".join(rng.choice("0123456789") for _ in range(rng.randrange(65, 120))) + "/items"
        elif shape == 2:
            path = "/" + "ab" * rng.randrange(33, 60) + "/" + "9" * rng.randrange(7, 90)
        elif shape == 3:
            path = "/" + "/".join(f"seg{i}" for i in range(rng.randrange(400, 700)))   # a 3-5 KB path
        else:
            path = "/users/%d/orders/%s" % (rng.randrange(10**9), "".join(rng.choice("0123456789abcdef") for _ in range(32)))
        spans.append(host.span(name="GET", kind=rng.choice([2, 3]), attributes={"http.request.method": "GET", "url.path": path}))
    res = {"service.name": "svc", "k8s.namespace.name": "default", "k8s.deployment.name": "svc"}
    tr = host.traces(host.resource_spans(res, spans))
    proc = host.Processor("odigosurltemplate", {})
    hb = proc.columnarize(tr)
    assert UrlOracle({}).process(hb.cols, hb.outs) == 0
    want = hb.apply()
    got = host.Processor("odigosurltemplate", {}).consume(tr)
    assert got == want


@pytest.mark.gpu
def test_gpu_groups_over_the_stage_planned_in_subsets():
    # 80-140 byte paths of ordinary segments: a group's paths alone outgrow the
    # plan kernel's 3 KB stage (about 7 chunks of 16 bytes per path), so
    # url_plan_slow_kernel plans each group in lane subsets with the list
    # planner; a few lanes carry a 65+ byte segment, whose subset falls back
    # to per-lane planning.  The result must equal the oracle's.
    import random
    import uuid
    rng = random.Random(0x0D16_0A12)

    def segment():
        k = rng.randrange(8)
        if k == 0:
            return str(rng.randrange(10 ** rng.randrange(1, 12)))
        if k == 1:
            return str(uuid.UUID(int=rng.getrandbits(128)))
        if k == 2:
            return "".join(rng.choice("0123456789abcdef") for _ in range(rng.randrange(8, 40)))
        if k == 3:
            return "2024-%02d-%02d" % (rng.randrange(1, 13), rng.randrange(1, 29))
        if k == 4:
            return "user%d@example.com" % rng.randrange(1000)
        return "".join(rng.choice("abcdefghijklmnopqrstuvwxyz-_") for _ in range(rng.randrange(2, 14)))

    spans = []
    for k in range(640):
        parts = []
        while sum(len(p) + 1 for p in parts) < rng.randrange(80, 140):
            parts.append(segment())
        if rng.random() < 0.02:
            parts.append("z" * rng.randrange(65, 90))
        path = "/" + "/".join(parts) + ("/" if rng.random() < 0.05 else "")
        spans.append(host.span(name="GET", kind=rng.choice([2, 3]),
                               attributes={"http.request.method": "GET", "url.path": path}))
    res = {"service.name": "svc", "k8s.namespace.name": "default", "k8s.deployment.name": "svc"}
    tr = host.traces(host.resource_spans(res, spans))
    proc = host.Processor("odigosurltemplate", {})
    hb = proc.columnarize(tr)
    assert UrlOracle({}).process(hb.cols, hb.outs) == 0
    want = hb.apply()
    got = host.Processor("odigosurltemplate", {}).consume(tr)
    assert got == want


def test_url_class_words_host(tmp_path):
    # the lookup + bit-transpose class words of url_plan_kernel's bitmaps
    # (odigos_amd/csrc/url_classes.hpp, compiled for the host) against per-byte
    # predicates of templatize.go's character classes: every byte value at
    # every row position, then random rows (tests/lut_check.cpp)
    import subprocess
    from pathlib import Path
    src = Path(__file__).with_name("lut_check.cpp")
    exe = tmp_path / "lut_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), str(src)], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-2000:]
