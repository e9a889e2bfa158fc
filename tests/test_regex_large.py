"""Regexps whose DFA has thousands of states (custom ids, templatization
rules, span_attribute regex conditions): the DFA compiler takes up to about
two million states (uint16 state ids up to 65535, uint32 beyond; 65279 in
round 4, 4096 before).  The DFA is checked against
the oracle's Pike VM (oracle/regex.c, no state bound) on the host and, on
the GPU, through URL templatization against the oracle chain."""
import ctypes as C
import json
import random

import numpy as np
import pytest

from odigos_amd import native
from tests.oracle_lib import Regex
from tests.test_unicode_regex import _cols_from_paths, _dfa

# (a|b)*a(a|b){k}: "an 'a' k+1 characters from the end of some prefix" — the
# unanchored search tracks the last k+1 characters, 2^(k+1) DFA states
BIG = [r"(a|b)*a(a|b){12}", r"[ab]*b[ab]{11}c", r"^(?:a|b)*a(?:a|b){13}$"]


def _ab_strings(rng, n):
    out = []
    for _ in range(n):
        k = rng.randrange(0, 40)
        s = "".join(rng.choice("ab") for _ in range(k))
        if rng.random() < 0.2:
            s += rng.choice(["c", "x", "", "ac"])
        out.append(s)
    return out


@pytest.mark.parametrize("pattern", BIG)
def test_large_dfa_vs_oracle(pattern):
    rng = random.Random(hash(pattern) & 0xFFFF)
    orc = Regex(pattern)
    for s in _ab_strings(rng, 60):   # (osehost_regex_match compiles the DFA on every call)
        b = s.encode()
        assert _dfa(pattern, b) == orc.match(b), (pattern, s)


def test_wide_dfa_vs_oracle():
    # 2^18 states: uint32 state ids (refused before round 5)
    pattern = r"(a|b)*a(a|b){17}"
    rng = random.Random(17)
    orc = Regex(pattern)
    for s in _ab_strings(rng, 12):
        b = s.encode()
        assert _dfa(pattern, b) == orc.match(b), (pattern, s)


def test_dfa_state_bound_still_refuses():
    # 2^22 states: past the state bound, refused (never approximated)
    assert native.lib().osehost_regex_match(r"(a|b)*a(a|b){21}".encode(), b"ab", 2) == -2   # too large


def test_engine_accepts_large_dfa_custom_id():
    cfg = {"odigosurltemplate": {"custom_ids": [{"regexp": "^" + BIG[0] + "$", "template_name": "ab"}]}}
    h = C.c_void_p()
    rc = native.lib().ose_engine_create(json.dumps(cfg).encode(), C.byref(h))
    assert rc in (0, native.OSE_EDEVICE), (rc, native.last_error())
    if rc == 0:
        native.lib().ose_engine_destroy(h)


LARGE_URL_CFG = {
    "custom_ids": [{"regexp": r"^(?:a|b)*a(?:a|b){12}$", "template_name": "ab"}],
    "templatization_rules": [r"/s/{seq:^[ab]*b[ab]{11}$}/{rest}"],
}


WIDE_URL_CFG = {
    "custom_ids": [{"regexp": r"^(?:a|b)*a(?:a|b){16}$", "template_name": "ab"}],   # 2^17 states: uint32 ids
    "templatization_rules": [r"/s/{seq:^[ab]*b[ab]{16}$}/{rest}"],
}


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [LARGE_URL_CFG, WIDE_URL_CFG], ids=["uint16", "uint32"])
def test_gpu_url_parity_large_dfa(cfg):
    import torch
    from odigos_amd.batch import DeviceBatch, Engine, HostOutputs
    from tests.oracle_lib import UrlOracle
    rng = random.Random(0x0D1600E1)
    paths = []
    for _ in range(40_000):
        segs = ["".join(rng.choice("ab") for _ in range(rng.randrange(1, 30))) for _ in range(rng.randrange(1, 5))]
        if rng.random() < 0.2:
            segs = ["s"] + segs[:2]
        paths.append(("/" + "/".join(segs)).encode())
    cols, _keep = _cols_from_paths(paths)
    eng = Engine({"odigosurltemplate": cfg})
    db = DeviceBatch(cols)
    eng.process_device(db, native.STAGE_TEMPLATE)
    torch.cuda.synchronize()
    ho = HostOutputs(cols)
    assert UrlOracle(cfg).process(cols, ho.outs, 4) == 0
    n = cols.n_spans
    np.testing.assert_array_equal(db.out_numpy("url_out", n=n), ho.view("url_out", np.uint8)[:n])
    used = db.used()
    assert used == int(ho.used[0])
    np.testing.assert_array_equal(db.out_numpy("tmpl_arena", n=used), ho.bufs["tmpl_arena"][:used])
    assert b"{ab}" in ho.bufs["tmpl_arena"][:used].tobytes()
