"""The C ABI (CPU only): libwsgpu.so loads, exports every symbol include/wsgpu.h
declares, and its host-only entry points agree with the oracle.  No device calls."""
import ctypes as C
import os

import numpy as np
import pytest

from tests.golden import fixtures, make_golden
from tests import wsgen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    from snf4j_amd import _lib  # built by conftest.pytest_configure
    return _lib


def test_exports_every_header_symbol(L):
    syms = L.header_symbols()
    assert len(syms) >= 20
    raw = C.CDLL(L.LIB_PATH)
    missing = [s for s in syms if not hasattr(raw, s)]
    assert not missing, missing
    assert L.lib.wsg_version() == 1
    assert L.lib.wsg_num_kernels() >= 5


def test_bench_library_exports_wsbench_header():
    """libwsbench.so (bench/test support) exports what include/wsbench.h declares,
    and the codec library does not carry the bench-only entry points."""
    import re
    from snf4j_amd import _lib
    import benchsupport
    with open(os.path.join(ROOT, "include", "wsbench.h")) as fh:
        syms = sorted(set(re.findall(r"\b(wsb_[a-z_]+)\(", fh.read())))
    assert syms == ["wsb_copy_ceiling", "wsb_synth_frames", "wsb_synth_uniform"]
    raw = C.CDLL(benchsupport.LIB_PATH)
    assert all(hasattr(raw, s) for s in syms)
    codec = C.CDLL(_lib.LIB_PATH)
    for s in ("wsg_synth_uniform", "wsg_synth_frames", "wsg_copy_ceiling"):
        assert not hasattr(codec, s), s


def test_library_is_gfx950_code_object(L):
    with open(L.LIB_PATH, "rb") as fh:
        blob = fh.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_frame_available_matches_oracle_kat(L, oracle):
    from snf4j_amd.context import frame_available
    av = fixtures.load("available")
    for c in av["big"]:
        data = fixtures.unhex(c["data"])
        r, err, d1, d2 = frame_available(data, c["len"])
        if "error" in c:
            assert r == -1 and oracle.format_error(err, d1, d2) == c["error"]
        else:
            assert r == c["expect"]
    for c in av["frames"]:
        data = make_golden.frame(c["data_spec"], 0)
        n = c["expected_len"]
        for ln in list(range(0, min(n, 40))) + [n, n + 1]:
            r = frame_available(data, ln)[0]
            assert r == oracle.Decoder(True, True, 2400).available(data, 0, ln), (c, ln)


def test_frame_available_random_headers(L, oracle):
    from snf4j_amd.context import frame_available
    rng = np.random.default_rng(3)
    for _ in range(3000):
        h = rng.integers(0, 256, 14, dtype=np.uint8).tobytes()
        ln = int(rng.integers(0, 1 << 31))
        r, err, d1, d2 = frame_available(h, ln)
        dec = oracle.Decoder(False, False, 65536)
        try:
            exp = dec.available(h, 0, ln)
            assert r == exp
        except oracle.InvalidFrame as e:
            assert r == -1 and (err, d1, d2) == (e.err, e.detail, e.detail2)


def test_check_header_matches_oracle(L, oracle):
    from snf4j_amd.context import check_header, decoder_cfg
    rng = np.random.default_rng(5)
    for trial in range(400):
        cm, ext = bool(trial & 1), bool(trial & 2)
        kind = wsgen.INJECT_KINDS[trial % len(wsgen.INJECT_KINDS)]
        f = wsgen.bad_frame(rng, kind, not cm, 512)
        hl = 2 + (4 if f[1] & 0x80 else 0) + {126: 2, 127: 8}.get(f[1] & 0x7F, 0)
        frag = bool(rng.integers(0, 2))
        err, det = check_header(decoder_cfg(cm, ext, 512), frag, f[:hl])
        dec = oracle.Decoder(cm, ext, 512, True)
        if frag:  # put the oracle decoder inside a fragmented message first
            dec.decode(wsgen.build_frame(2, False, 0, b"", not cm, (1, 2, 3, 4)))
        try:
            dec.decode(f[:hl])
            oerr = 0
        except oracle.InvalidFrame as e:
            oerr, odet = e.err, e.detail
        if oerr in (12, 13):  # close status/reason need the payload: not header rules
            oerr = 0
        assert err == oerr, (kind, f.hex())
        if err:
            assert det == odet


def test_encoded_length(L, oracle):
    from snf4j_amd.context import encoded_length
    for n in [0, 1, 125, 126, 127, 0xFFFE, 0xFFFF, 0x10000, 100000, 1 << 31]:
        for cm in (False, True):
            assert encoded_length(n, cm) == oracle.encoded_length(n, cm)


def test_error_messages_match_oracle(L, oracle):
    from snf4j_amd.context import error_message
    for code in range(1, 17):
        for d in (0, 1, 126, 131072, -1):
            assert error_message(code, d, 2147483633) == oracle.format_error(code, d, 2147483633)


def test_no_device_means_loud_failure(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from snf4j_amd import Context
    with pytest.raises(Exception):
        Context(0)


def test_synth_generator_oracle_is_valid_utf8(L, oracle):
    wire, off, sf = oracle.synth_uniform(11, 64, 4096, 16, opcode=1, masked=True, text=True)
    b = oracle.Batch(False, False, 65536, True, len(sf) - 1)
    payload, desc, res = b.decode(wire, off, sf)
    assert (res["error"] == 0).all() and res["n_delivered"].sum() == 64
    # about 70 % ASCII bytes
    frac = (payload < 0x80).mean()
    assert 0.45 < frac < 0.9
